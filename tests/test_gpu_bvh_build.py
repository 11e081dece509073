"""GPU tests of the device BVH build (pt_bvh4_build_device, SURVEY.md §8f
rank 3): byte-identical to the host build (itself byte-identical to the
reference, tests/test_reference_parity.py) on edge cases, random and
degenerate box sets, and — through the scene path — against the reference's
own BVH arrays in the golden fixtures.  Bar: bit-exact (integer / index work
and min/max of the inputs)."""
import numpy as np
import pytest

from fixtures import NAMES, load
from pathtracing_amd import flatten
from pathtracing_amd import native as N
from test_reference_parity import _bytes

pytestmark = pytest.mark.gpu


def _same(boxes):
    st = {}
    h = N.bvh4_build(boxes)
    d = N.bvh4_build_device(boxes, stats=st)
    assert _bytes(d[0], 128) == _bytes(h[0], 128), "clusters"
    assert d[1].tobytes()[:3] + d[1].tobytes()[4:] == h[1].tobytes()[:3] + h[1].tobytes()[4:], "root"
    np.testing.assert_array_equal(d[2], h[2])
    np.testing.assert_array_equal(d[3], h[3])
    return st


def _tri_boxes(rng, n, spread=10.0, size=0.05):
    v0 = rng.uniform(-spread, spread, (n, 3)).astype(np.float32)
    v1 = v0 + rng.normal(0, size, (n, 3)).astype(np.float32)
    v2 = v0 + rng.normal(0, size, (n, 3)).astype(np.float32)
    t = np.stack([v0, v1, v2], 1)
    return np.concatenate([t.min(1), t.max(1)], 1).astype(np.float32)


@pytest.mark.parametrize("n", [1, 2, 3, 5, 47, 48, 49, 50, 64, 127, 128, 129, 1000, 4097, 4098])
def test_device_build_small_sizes(n):
    _same(_tri_boxes(np.random.default_rng(n), n))


def test_device_build_empty():
    cl, root, order, bbox = N.bvh4_build_device(np.zeros((0, 6), np.float32))
    assert cl.shape[0] == 0 and order.shape[0] == 0


def test_device_build_degenerate_sets():
    rng = np.random.default_rng(7)
    same = np.tile(np.array([[0.5, 0.5, 0.5, 1.5, 1.5, 1.5]], np.float32), (3000, 1))
    _same(same)                                  # every centroid equal: one big leaf
    flat = _tri_boxes(rng, 20000)
    flat[:, 1] = 2.0
    flat[:, 4] = 2.0                             # a plane: one axis skipped everywhere
    _same(flat)
    line = _tri_boxes(rng, 20000)
    line[:, [1, 2, 4, 5]] = 1.0                  # a line
    _same(line)
    dup = np.repeat(_tri_boxes(rng, 500), 40, axis=0)  # clusters of identical boxes
    _same(dup)


def test_device_build_clustered_and_skewed():
    rng = np.random.default_rng(11)
    parts = [_tri_boxes(rng, 50000, spread=s, size=s * 0.01) + np.float32(o)
             for s, o in ((0.01, 0), (1, 5), (100, -300), (0.5, 1e3))]
    _same(np.concatenate(parts))


def test_device_build_large():
    st = _same(_tri_boxes(np.random.default_rng(3), 1_000_000))
    assert st["levels"] > 5 and st["small_tasks"] > 1000 and st["ms_device"] > 0


@pytest.mark.parametrize("name", NAMES)
def test_device_build_scene_matches_reference_fixture(name):
    """Scenes flattened with the device build: TLAS and BLAS arrays against the
    reference's own (the fixture), the same check as the host build's."""
    from test_reference_parity import test_bvh4_build_is_byte_identical
    flatten.BVH_DEVICE = 0
    try:
        setup, integ, fx = load(name)
        test_bvh4_build_is_byte_identical((name, setup, integ, fx))
    finally:
        flatten.BVH_DEVICE = None
