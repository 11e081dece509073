"""ctypes binding of libpt_hip.so (include/pt_api.h).

The library is built in-tree by __graft_entry__.build() (hipcc, gfx950) into
pathtracing_amd/_lib/libpt_hip.so.  There is no fallback: if it cannot be
loaded, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

LIB_DIR = Path(__file__).resolve().parent / "_lib"
LIB_PATH = Path(os.environ["PT_HIP_LIB"]) if os.environ.get("PT_HIP_LIB") else LIB_DIR / "libpt_hip.so"  # override: debugging builds

PT_OK = 0
PT_PRIM_TRIANGLE, PT_PRIM_QUAD, PT_PRIM_SPHERE, PT_PRIM_BLAS, PT_PRIM_INSTANCE = 0, 1, 2, 3, 4
PT_TEX_SOLID, PT_TEX_IMAGE, PT_TEX_CHECKER = 0, 1, 2
PT_MAT_DIFFUSE, PT_MAT_DIELECTRIC, PT_MAT_THIN, PT_MAT_CONDUCTOR = 0, 1, 2, 3
PT_LIGHT_AREA, PT_LIGHT_UNIFORM_INF, PT_LIGHT_SKY_INF, PT_LIGHT_DISTANT, PT_LIGHT_POINT, PT_LIGHT_TEX_INF = 0, 1, 2, 3, 4, 5
PT_IMAGE_U8, PT_IMAGE_F32 = 0, 1
PT_TEXINF_X, PT_TEXINF_Y = 1920, 1080
PT_LS_UNIFORM, PT_LS_POWER = 0, 1
PT_INTEGRATOR_PATH, PT_INTEGRATOR_SIMPLE, PT_INTEGRATOR_VOLPATH = 0, 1, 2
PT_FILTER_MITCHELL, PT_FILTER_BOX, PT_FILTER_GAUSSIAN, PT_FILTER_LANCZOS = 0, 1, 2, 3
PT_TONEMAP_REINHARD_JODIE, PT_TONEMAP_ACES = 0, 1
PT_RENDER_COUNT_NODES = 0x1
PT_RENDER_TIMING = 0x2
PT_RENDER_TRAVERSAL_POOL = 0x4
PT_RENDER_TRAVERSAL_SIMPLE = 0x8
PT_RENDER_NODES_FULL = 0x10
PT_RENDER_NODES_QUANTIZED = 0x20
PT_RENDER_ADAPTIVE = 0x40
PT_RENDER_SORT_MATERIAL = 0x80
PT_RENDER_SORT_SPATIAL = 0x100
PT_RENDER_NO_SORT = 0x200
PT_RENDER_SORT_RAYS = 0x400
PT_RENDER_SERIAL_SHADOW = 0x800
PT_RENDER_OVERLAP_SHADOW = 0x1000
PT_RENDER_ANY_STACKLESS = 0x4000
PT_RENDER_NO_TAIL = 0x2000
PT_NODES_AUTO, PT_NODES_FULL, PT_NODES_QUANTIZED = 0, 1, 2

# ---- numpy mirrors of the array element structs (layouts asserted below) ----
REF_NODE = np.dtype([("count", "u1"), ("active", "u1"), ("perm", "u1"), ("pad", "u1"), ("cluster_idx", "<u4")])
REF_CLUSTER = np.dtype([("xmin", "<f4", 4), ("xmax", "<f4", 4), ("ymin", "<f4", 4), ("ymax", "<f4", 4),
                        ("zmin", "<f4", 4), ("zmax", "<f4", 4), ("children", REF_NODE, 4)])
PRIM = np.dtype([("kind", "<u4"), ("index", "<u4"), ("material", "<i4"), ("light", "<i4"), ("medium", "<i4")])
QUAD = np.dtype([("Q", "<f4", 3), ("u", "<f4", 3), ("v", "<f4", 3), ("normal", "<f4", 3), ("D", "<f4"),
                 ("w", "<f4", 3)])
SPHERE = np.dtype([("center", "<f4", 3), ("radius", "<f4")])
TEXTURE = np.dtype([("kind", "<u4"), ("scale", "<f4", 3), ("value", "<f4", 3), ("a", "<i4"), ("b", "<i4"),
                    ("inv_scale", "<f4", 2), ("image", "<i4")])
IMAGE = np.dtype([("offset", "<u8"), ("width", "<i4"), ("height", "<i4"), ("channels", "<i4"), ("format", "<i4")])
MATERIAL = np.dtype([("kind", "<u4"), ("tex", "<i4"), ("norm", "<i4"), ("rough", "<i4"), ("metal", "<i4"),
                     ("alpha", "<i4"), ("alpha_mode", "<u4"), ("alpha_cutoff", "<f4"), ("ri", "<f4"),
                     ("albedo", "<f4", 3)])
LIGHT = np.dtype([("kind", "<u4"), ("prim", "<i4"), ("tex", "<i4"), ("one_sided", "<u4"), ("power", "<f4"),
                  ("pmf", "<f4"), ("color", "<f4", 3), ("vec", "<f4", 3), ("scale", "<f4"), ("instance", "<i4")])
INSTANCE = np.dtype([("transform", "<f4", 16), ("inv", "<f4", 16), ("bvh", "<u4"), ("virt_base", "<u4"),
                     ("motion", "<f4", 3), ("time_bounds", "<f4", 2), ("animated", "<u4"), ("inner", "<i4")])
MEDIUM = np.dtype([("sigma_a", "<f4", 3), ("sigma_s", "<f4", 3), ("sigma_t", "<f4", 3), ("Le", "<f4", 3),
                   ("g", "<f4")])
RAY = np.dtype([("o", "<f4", 3), ("d", "<f4", 3), ("tmax", "<f4"), ("time", "<f4")])
HIT = np.dtype([("t", "<f4"), ("b1", "<f4"), ("b2", "<f4"), ("prim", "<i4")])

assert REF_NODE.itemsize == 8 and REF_CLUSTER.itemsize == 128 and PRIM.itemsize == 20
assert QUAD.itemsize == 64 and SPHERE.itemsize == 16 and TEXTURE.itemsize == 48 and IMAGE.itemsize == 24
assert MATERIAL.itemsize == 48 and LIGHT.itemsize == 56 and RAY.itemsize == 32 and INSTANCE.itemsize == 164 and HIT.itemsize == 16


class RefNode(C.Structure):
    _fields_ = [("count", C.c_uint8), ("active", C.c_uint8), ("perm", C.c_uint8), ("pad", C.c_uint8),
                ("cluster_idx", C.c_uint32)]


class BvhDesc(C.Structure):
    _fields_ = [("clusters", C.c_void_p), ("n_clusters", C.c_uint32), ("root", RefNode),
                ("prim_base", C.c_uint32), ("n_prims", C.c_uint32)]


class SceneDesc(C.Structure):
    _fields_ = [
        ("positions", C.c_void_p), ("normals", C.c_void_p), ("uvs", C.c_void_p), ("tangents", C.c_void_p),
        ("n_vertices", C.c_uint32),
        ("tri_vidx", C.c_void_p), ("tri_flags", C.c_void_p), ("n_triangles", C.c_uint32),
        ("quads", C.c_void_p), ("n_quads", C.c_uint32),
        ("spheres", C.c_void_p), ("n_spheres", C.c_uint32),
        ("prims", C.c_void_p), ("n_prims", C.c_uint32),
        ("bvhs", C.c_void_p), ("n_bvhs", C.c_uint32),
        ("materials", C.c_void_p), ("n_materials", C.c_uint32),
        ("textures", C.c_void_p), ("n_textures", C.c_uint32),
        ("images", C.c_void_p), ("n_images", C.c_uint32),
        ("texels", C.c_void_p), ("n_texel_bytes", C.c_uint64),
        ("lights", C.c_void_p), ("n_lights", C.c_uint32),
        ("light_sampler", C.c_uint32),
        ("sampler_lights", C.c_void_p), ("n_sampler_lights", C.c_uint32),
        ("infinite_lights", C.c_void_p), ("n_infinite_lights", C.c_uint32),
        ("light_dist", C.c_void_p), ("n_light_dist", C.c_uint64),
        ("media", C.c_void_p), ("n_media", C.c_uint32), ("scene_medium", C.c_int32),
        ("instances", C.c_void_p), ("n_instances", C.c_uint32),
    ]


class CameraDesc(C.Structure):
    _fields_ = [("origin", C.c_float * 3), ("u", C.c_float * 3), ("v", C.c_float * 3), ("w", C.c_float * 3),
                ("half_width", C.c_float), ("half_height", C.c_float), ("defocus_radius", C.c_float),
                ("focus_distance", C.c_float), ("focus_angle", C.c_float), ("width", C.c_int32),
                ("height", C.c_int32), ("medium", C.c_int32), ("shutter", C.c_float * 2), ("has_shutter", C.c_int32)]


class RenderDesc(C.Structure):
    _fields_ = [("integrator", C.c_uint32), ("spp", C.c_uint32), ("max_depth", C.c_uint32), ("seed", C.c_uint32),
                ("filter", C.c_uint32), ("filter_radius", C.c_float * 2), ("filter_params", C.c_double * 2),
                ("shard_index", C.c_uint32), ("shard_count", C.c_uint32), ("flags", C.c_uint32),
                ("paths_in_flight", C.c_uint32), ("pixel_begin", C.c_uint32), ("pixel_end", C.c_uint32),
                ("strata", C.c_uint32 * 2)]


class Stats(C.Structure):
    _fields_ = [("paths", C.c_uint64), ("rays_closest", C.c_uint64), ("rays_any", C.c_uint64),
                ("nodes_closest", C.c_uint64), ("tris_closest", C.c_uint64), ("nodes_any", C.c_uint64),
                ("tris_any", C.c_uint64), ("shade_hits", C.c_uint64), ("ms_total", C.c_double),
                ("ms_closest", C.c_double), ("ms_any", C.c_double), ("ms_shade", C.c_double),
                ("launches_closest", C.c_uint64), ("launches_any", C.c_uint64),
                ("stack_overflows", C.c_uint64), ("n_devices", C.c_uint32), ("tie_overflows", C.c_uint32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "pad"}


class BvhBuildStats(C.Structure):
    _fields_ = [("ms_total", C.c_double), ("ms_device", C.c_double), ("ms_collapse", C.c_double),
                ("levels", C.c_uint32), ("small_tasks", C.c_uint32), ("nodes", C.c_uint32), ("pad", C.c_uint32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "pad"}


EXPORTS = [
    "pt_version", "pt_create", "pt_destroy", "pt_last_error", "pt_set_stream", "pt_scene_upload", "pt_render",
    "pt_trace", "pt_scene_device_bytes", "pt_bvh4_build", "pt_bvh4_order_table", "pt_film_resolve",
    "pt_mat4_inverse", "pt_bvh4_build_device", "pt_set_node_format", "pt_render_adaptive", "pt_render_samples",
    "pt_texinf_weights", "pt_device_count", "pt_comm_unique_id", "pt_comm_init_rank", "pt_film_reduce",
    "pt_comm_destroy", "pt_frame_samples", "pt_frame_sample_range",
]
PT_COMM_ID_BYTES = 128

_lib = None


class NativeError(RuntimeError):
    pass


def lib():
    """Load libpt_hip.so (fails loudly: there is no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise NativeError(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
    # One HIP runtime per process: torch bundles its own libamdhip64.so.7.
    # Loaded first, the library binds to it by soname; loaded before torch, it
    # would pull in /opt/rocm's copy and torch's later GPU init fails ("No HIP
    # GPUs are available").  torch stays plumbing (device tensors, streams).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(str(LIB_PATH))
    vp = C.c_void_p
    L.pt_version.restype = C.c_int
    L.pt_create.argtypes = [C.POINTER(vp), C.c_int, C.POINTER(C.c_int)]
    L.pt_create.restype = C.c_int32
    L.pt_device_count.argtypes = [vp]
    L.pt_device_count.restype = C.c_int
    L.pt_comm_unique_id.argtypes = [vp]
    L.pt_comm_unique_id.restype = C.c_int32
    L.pt_comm_init_rank.argtypes = [vp, C.c_int, C.c_int, vp]
    L.pt_comm_init_rank.restype = C.c_int32
    L.pt_film_reduce.argtypes = [vp, vp, C.c_uint64, C.c_int]
    L.pt_film_reduce.restype = C.c_int32
    L.pt_comm_destroy.argtypes = [vp]
    L.pt_comm_destroy.restype = C.c_int32
    L.pt_frame_samples.argtypes = [vp, vp, vp, C.c_uint32, vp]
    L.pt_frame_samples.restype = C.c_int32
    if hasattr(L, "pt_frame_sample_range"):  # an API-5 build loaded for a timing A/B lacks it
        L.pt_frame_sample_range.argtypes = [vp, vp, vp]
        L.pt_frame_sample_range.restype = C.c_int32
    L.pt_destroy.argtypes = [vp]
    L.pt_destroy.restype = None
    L.pt_last_error.argtypes = [vp]
    L.pt_last_error.restype = C.c_char_p
    L.pt_set_stream.argtypes = [vp, vp]
    L.pt_set_stream.restype = C.c_int32
    L.pt_set_node_format.argtypes = [vp, C.c_int]
    L.pt_set_node_format.restype = C.c_int32
    L.pt_scene_upload.argtypes = [vp, C.POINTER(SceneDesc)]
    L.pt_scene_upload.restype = C.c_int32
    L.pt_render.argtypes = [vp, C.POINTER(CameraDesc), C.POINTER(RenderDesc), vp, C.POINTER(Stats)]
    L.pt_render.restype = C.c_int32
    L.pt_render_adaptive.argtypes = [vp, C.POINTER(CameraDesc), C.POINTER(RenderDesc), vp, vp, C.POINTER(Stats)]
    L.pt_render_adaptive.restype = C.c_int32
    L.pt_trace.argtypes = [vp, vp, C.c_uint32, C.c_int, vp, C.POINTER(Stats)]
    L.pt_trace.restype = C.c_int32
    L.pt_mat4_inverse.argtypes = [vp, vp]
    L.pt_mat4_inverse.restype = C.c_int32
    L.pt_film_resolve.argtypes = [vp, vp, C.c_int32, C.c_int32, C.c_uint32, vp]
    L.pt_film_resolve.restype = C.c_int32
    L.pt_interact.argtypes = [vp, vp, C.c_uint32, vp]
    L.pt_interact.restype = C.c_int32
    L.pt_bsdf_cases.argtypes = [vp, C.c_int32, vp, C.c_uint32, vp]
    L.pt_bsdf_cases.restype = C.c_int32
    L.pt_light_cases.argtypes = [vp, vp, C.c_uint32, vp]
    L.pt_light_cases.restype = C.c_int32
    L.pt_light_picks.argtypes = [vp, vp, C.c_uint32, vp]
    L.pt_light_picks.restype = C.c_int32
    L.pt_anim_inverse_cases.argtypes = [vp, vp, C.c_uint32, vp]
    L.pt_anim_inverse_cases.restype = C.c_int32
    L.pt_alpha_coverage.argtypes = [C.POINTER(SceneDesc), vp]
    L.pt_alpha_coverage.restype = C.c_int32
    L.pt_scene_device_bytes.argtypes = [vp]
    L.pt_scene_device_bytes.restype = C.c_uint64
    L.pt_bvh4_build.argtypes = [vp, C.c_uint32, vp, C.POINTER(C.c_uint32), C.POINTER(RefNode), vp, vp]
    L.pt_bvh4_build.restype = C.c_int32
    L.pt_bvh4_build_device.argtypes = [vp, vp, C.c_uint32, vp, C.POINTER(C.c_uint32), C.POINTER(RefNode), vp, vp,
                                       C.POINTER(BvhBuildStats)]
    L.pt_bvh4_build_device.restype = C.c_int32
    L.pt_texinf_weights.argtypes = [vp, C.c_int32, C.c_int32, C.c_int32, vp, C.c_float, vp, C.c_int32]
    L.pt_texinf_weights.restype = C.c_int32
    L.pt_bvh4_order_table.argtypes = [vp]
    L.pt_bvh4_order_table.restype = C.c_int32
    _lib = L
    return L


def texinf_weights(texels: np.ndarray, color_scale, le_scale: float, threads: int = 0) -> np.ndarray:
    """TextureInfiniteLight::PreProcess's 1920 x 1080 cell weights (host
    routine of libpt_hip, pt_texinf_weights); texels HxWxC float32."""
    t = np.ascontiguousarray(texels, np.float32)
    h, w, c = t.shape
    cs = np.ascontiguousarray(color_scale, np.float32).reshape(3)
    out = np.zeros(PT_TEXINF_X * PT_TEXINF_Y, np.float32)
    n = threads or min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1))
    check(lib().pt_texinf_weights(t.ctypes.data, w, h, c, cs.ctypes.data, float(le_scale), out.ctypes.data, int(n)))
    return out


def mat4_inverse(m: np.ndarray) -> np.ndarray:
    """glm::inverse of a column-major float32 mat4 (host routine of libpt_hip)."""
    m = np.ascontiguousarray(m, np.float32).reshape(4, 4)
    out = np.zeros((4, 4), np.float32)
    check(lib().pt_mat4_inverse(m.ctypes.data, out.ctypes.data))
    return out


def check(status: int, ctx=None):
    if status != PT_OK:
        msg = lib().pt_last_error(ctx)
        raise NativeError(f"pt status {status}: {msg.decode() if msg else ''}")


def ptr(a: np.ndarray | None):
    if a is None or a.size == 0:
        return None
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


def bvh4_build(boxes: np.ndarray):
    """Reference BVH4 build (BVH.hpp:95-105, 290-390, 743-1017) over n boxes
    {min.xyz, max.xyz} -> (clusters, root, prim_order, bbox)."""
    boxes = np.ascontiguousarray(boxes, dtype=np.float32).reshape(-1, 6)
    n = boxes.shape[0]
    clusters = np.zeros(max(n, 1), dtype=REF_CLUSTER)
    order = np.zeros(max(n, 1), dtype=np.uint32)
    nc = C.c_uint32(0)
    root = RefNode()
    bbox = np.zeros(6, dtype=np.float32)
    check(lib().pt_bvh4_build(ptr(boxes), n, clusters.ctypes.data, C.byref(nc), C.byref(root), order.ctypes.data,
                              bbox.ctypes.data))
    r = np.zeros(1, dtype=REF_NODE)
    r[0] = (root.count, root.active, root.perm, root.pad, root.cluster_idx)
    return clusters[: nc.value].copy(), r[0], order[:n].copy(), bbox


def bvh4_build_device(boxes: np.ndarray, device: int = 0, stats: dict | None = None):
    """pt_bvh4_build_device: the same build as bvh4_build (byte-identical
    outputs) run on the GPU.  `stats`, if given, receives the timings."""
    boxes = np.ascontiguousarray(boxes, dtype=np.float32).reshape(-1, 6)
    n = boxes.shape[0]
    clusters = np.zeros(max(n, 1), dtype=REF_CLUSTER)
    order = np.zeros(max(n, 1), dtype=np.uint32)
    nc = C.c_uint32(0)
    root = RefNode()
    bbox = np.zeros(6, dtype=np.float32)
    st = BvhBuildStats()
    L = lib()
    ctx = C.c_void_p()
    dev = (C.c_int * 1)(int(device))
    check(L.pt_create(C.byref(ctx), 1, dev))
    try:
        check(L.pt_bvh4_build_device(ctx, ptr(boxes), n, clusters.ctypes.data, C.byref(nc), C.byref(root),
                                     order.ctypes.data, bbox.ctypes.data, C.byref(st)), ctx)
    finally:
        L.pt_destroy(ctx)
    if stats is not None:
        stats.update(st.as_dict())
    r = np.zeros(1, dtype=REF_NODE)
    r[0] = (root.count, root.active, root.perm, root.pad, root.cluster_idx)
    return clusters[: nc.value].copy(), r[0], order[:n].copy(), bbox


def order_table() -> np.ndarray:
    out = np.zeros(8 * 135, dtype=np.uint8)
    check(lib().pt_bvh4_order_table(out.ctypes.data))
    return out.reshape(8, 135)
