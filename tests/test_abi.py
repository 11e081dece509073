"""CPU tests of the C-ABI library: it loads without a GPU, exports every entry
point include/pt_api.h declares, reports errors without aborting, and its
host-side BVH builder handles the reference's edge cases."""
import ctypes as C
import re
from pathlib import Path

import numpy as np
import pytest

from pathtracing_amd import native as N

ROOT = Path(__file__).resolve().parents[1]


def declared_functions():
    text = (ROOT / "include" / "pt_api.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(pt_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = N.lib()
    names = declared_functions()
    assert "pt_render" in names and "pt_scene_upload" in names and "pt_bvh4_build" in names
    for name in names:
        assert hasattr(lib, name), f"libpt_hip.so does not export {name}"


def test_version_and_error_paths_without_device():
    lib = N.lib()
    assert lib.pt_version() == 9
    # argument validation never aborts
    assert lib.pt_scene_upload(None, None) == -1
    assert lib.pt_render(None, None, None, None, None) == -1
    assert lib.pt_trace(None, None, 0, 0, None, None) == -1
    assert lib.pt_create(None, 1, None) == -1
    ctx = C.c_void_p()
    assert lib.pt_create(C.byref(ctx), 0, None) == -1  # n_devices out of range
    dup = (C.c_int * 2)(0, 0)
    assert lib.pt_create(C.byref(ctx), 2, dup) == -1  # a device listed twice
    assert not ctx.value
    assert lib.pt_device_count(None) == 0
    assert lib.pt_film_reduce(None, None, 0, 0) == -1
    assert lib.pt_comm_init_rank(None, 1, 0, None) == -1
    assert lib.pt_comm_unique_id(None) == -1
    assert lib.pt_comm_destroy(None) == -1
    assert lib.pt_frame_samples(None, None, None, 0, None) == -1
    lib.pt_destroy(None)
    assert isinstance(lib.pt_last_error(None), (bytes, type(None)))


def test_bvh4_build_edge_cases():
    # empty: an empty root, no clusters (the reference allocates 2*0-1 nodes: UB)
    cl, root, order, bbox = N.bvh4_build(np.zeros((0, 6), np.float32))
    assert cl.shape[0] == 0 and root["active"] == 0 and root["count"] == 0
    # one primitive: a leaf root
    cl, root, order, bbox = N.bvh4_build(np.array([[0, 0, 0, 1, 1, 1]], np.float32))
    assert cl.shape[0] == 0 and root["active"] == 0 and root["count"] == 1
    np.testing.assert_array_equal(order, [0])
    # identical centroids: no split is possible, one leaf holding everything
    boxes = np.tile(np.array([[0, 0, 0, 1, 1, 1]], np.float32), (300, 1))
    cl, root, order, bbox = N.bvh4_build(boxes)
    assert root["active"] == 0 and root["count"] == (300 & 0xFF)  # u8 truncation (BVH.hpp:39,793)
    # random boxes: every primitive appears once in leaf order
    rng = np.random.default_rng(3)
    lo = rng.random((5000, 3)).astype(np.float32)
    boxes = np.concatenate([lo, lo + 0.01], 1)
    cl, root, order, bbox = N.bvh4_build(boxes)
    assert sorted(order.tolist()) == list(range(5000))
    assert cl.shape[0] > 0 and root["active"] != 0
    np.testing.assert_allclose(bbox[:3], boxes[:, :3].min(0))
    np.testing.assert_allclose(bbox[3:], boxes[:, 3:].max(0))


def test_order_table_is_a_permutation_table():
    t = N.order_table()
    assert t.shape == (8, 135)
    for p in np.unique(t):
        slots = {(int(p) >> (2 * s)) & 3 for s in range(4)}
        assert slots == {0, 1, 2, 3}


def test_flat_scene_layout(tmp_path):
    from pathtracing_amd import scenes
    s = scenes.cornell(W=16, H=16, spp=1, config="c3")
    integ = s.make_integrator()
    flat = integ.flat
    # TLAS slots then BLAS slots; the BLAS prim is a PT_PRIM_BLAS slot
    assert flat.prims.shape[0] == len(s.scene.primitives) + 34
    assert (flat.prims["kind"] == N.PT_PRIM_BLAS).sum() == 1
    tri = flat.prims[flat.prims["kind"] == N.PT_PRIM_TRIANGLE]
    assert sorted(tri["index"].tolist()) == list(range(34))
    d = flat.desc()
    assert d.n_prims == flat.prims.shape[0] and d.n_bvhs == 2 and d.n_lights == 1
