"""pt_mat4_inverse against glm::inverse as the reference's own build computes
it (tests/golden/mat4_inverse.npz from oracle/glm_inverse_probe.cpp):
TransformedPrimitive's invTransform (Primitive.hpp:37) takes every instanced
ray to object space, so one rounding apart moves the hit (a rotation about z
after a translation did, before the inverse spelled out GCC's contractions)."""
import numpy as np
import pytest

from pathtracing_amd import native as N
from tests.golden.fixtures import GOLDEN


def test_mat4_inverse_bit_exact_vs_reference_glm():
    fx = np.load(GOLDEN / "mat4_inverse.npz", allow_pickle=False)
    A, want = fx["m"], fx["inv"]
    got = np.stack([N.mat4_inverse(m.reshape(4, 4)).reshape(16) for m in A])
    bad = np.nonzero((got.view(np.uint32) != want.view(np.uint32)).any(1))[0]
    assert bad.size == 0, f"{bad.size} of {len(A)} matrices differ, first {bad[:8].tolist()}"


@pytest.mark.parametrize("k", [0, 3500, 5000])
def test_mat4_inverse_fixture_kinds(k):
    # the fixture holds instance-like, axis-rotation and general matrices
    fx = np.load(GOLDEN / "mat4_inverse.npz", allow_pickle=False)
    m = fx["m"][k].reshape(4, 4)
    assert np.isfinite(fx["inv"][k]).all()
    if k < 4500:
        np.testing.assert_array_equal(m[:, 3][:3], 0)  # affine: glm column-major, row 3 = (0, 0, 0, 1)


def test_oracle_and_device_inverse_formula_bit_exact_vs_reference_glm():
    """The oracle's mat4_inverse_ -- the operations the device's anim_inverse
    (pt_shading.h) runs for an AnimatedPrimitive at each ray's time -- against
    the reference build's own glm::inverse on all 6000 fixture matrices,
    pure translations included (their zero signs follow the contractions)."""
    import ctypes as C
    import sys
    sys.path.insert(0, str(GOLDEN.parents[1] / "oracle"))
    import oracle
    L = oracle.lib()
    L.oracle_mat4_inverse.argtypes = [C.c_void_p, C.c_void_p]
    L.oracle_mat4_inverse.restype = None
    fx = np.load(GOLDEN / "mat4_inverse.npz", allow_pickle=False)
    A, want = np.ascontiguousarray(fx["m"], np.float32), fx["inv"]
    got = np.zeros_like(A)
    for k in range(A.shape[0]):
        L.oracle_mat4_inverse(A[k].ctypes.data, got[k].ctypes.data)
    bad = np.nonzero((got.view(np.uint32) != want.view(np.uint32)).any(1))[0]
    assert bad.size == 0, f"{bad.size} of {len(A)} matrices differ, first {bad[:8].tolist()}"
