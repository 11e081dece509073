"""Scene -> flat, device-ready arrays (pt_scene_desc of include/pt_api.h).

Primitive slots are laid out in BVH leaf order: slots [0, n_top) are the TLAS
primitives (Scene::Add order permuted by the TLAS build), followed by every
Model's BLAS primitives in its own leaf order.  Light order is the reference's:
Scene::GetLights() walks the TLAS primitives in leaf order, descending into
each Model's BLAS leaf order (BVH.hpp:69-81, Model.hpp:33-35), then
Scene::infiniteLights (Scene.cpp:39-43); lights added to the light sampler
afterwards come last.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

from . import native as N
from .scene import (AlphaMode, AreaLight, CheckerTexture, DistantLight, FunctionInfiniteLight, GeometricPrimitive,
                    ImageTexture, LightSampler, Material, MicrofacetDielectric, MicrofacetDiffuse, Model, PointLight,
                    TransformedPrimitive, AnimatedPrimitive, mat4_identity, mat4_translate, _expand_seq,
                    PowerLightSampler, QuadShape, Scene, SolidColor, SpecularConductor, SphereShape, Texture,
                    ThinDielectric, TransformedLight, UniformInfiniteLight, UniformLightSampler,
                    FloatImageTexture, TextureInfiniteLight)


@dataclass
class FlatScene:
    positions: np.ndarray
    normals: np.ndarray
    uvs: np.ndarray
    tangents: np.ndarray
    tri_vidx: np.ndarray
    tri_flags: np.ndarray
    quads: np.ndarray
    spheres: np.ndarray
    prims: np.ndarray
    bvh_clusters: List[np.ndarray]
    bvh_roots: List[np.void]
    bvh_prim_base: List[int]
    bvh_n_prims: List[int]
    materials: np.ndarray
    textures: np.ndarray
    images: np.ndarray
    texels: np.ndarray
    bbox: np.ndarray
    tlas_lights: list                 # AreaLights in TLAS GetLights order
    light_slot: Dict[int, int]        # id(AreaLight) -> prim slot
    material_ids: Dict[int, int]      # id(Material) -> index
    top_order: np.ndarray             # TLAS slot -> Scene.Add index
    blas_orders: List[np.ndarray]     # per model: slot -> model-local triangle
    model_tri_base: List[int]         # per model: first global triangle id
    texture_ids: Dict[int, int]
    # light tables (set by bind_lights)
    lights: Optional[np.ndarray] = None
    light_sampler: int = 0
    sampler_lights: Optional[np.ndarray] = None
    infinite_lights: Optional[np.ndarray] = None
    light_objects: list = field(default_factory=list)
    light_dist: np.ndarray = field(default_factory=lambda: np.zeros(0, np.float32))
    instances: Optional[np.ndarray] = None   # pt_instance records
    # participating media: id(HomogeneusMedium) -> index into `media`
    media: Optional[np.ndarray] = None
    medium_ids: Dict[int, int] = field(default_factory=dict)
    scene_medium: int = -1

    def medium_id(self, md) -> int:
        """Index of medium `md` (registered on first use), -1 for None."""
        if md is None:
            return -1
        if id(md) not in self.medium_ids:
            rec = np.zeros(1, dtype=N.MEDIUM)
            rec["sigma_a"], rec["sigma_s"], rec["sigma_t"] = md.sigma_a, md.sigma_s, md.sigma_t
            rec["Le"], rec["g"] = md.Le(), md.g
            self.medium_ids[id(md)] = len(self.medium_ids)
            self.media = rec if self.media is None else np.concatenate([self.media, rec])
            self._medium_keep = getattr(self, "_medium_keep", []) + [md]
        return self.medium_ids[id(md)]

    @property
    def n_prims(self) -> int:
        return int(self.prims.shape[0])

    def desc(self):
        """pt_scene_desc referencing these arrays (keep self alive while used)."""
        d = N.SceneDesc()
        d.positions = N.ptr(self.positions)
        d.normals = N.ptr(self.normals)
        d.uvs = N.ptr(self.uvs)
        d.tangents = N.ptr(self.tangents)
        d.n_vertices = self.positions.shape[0] if self.positions.size else 0
        d.tri_vidx = N.ptr(self.tri_vidx)
        d.tri_flags = N.ptr(self.tri_flags)
        d.n_triangles = self.tri_flags.shape[0]
        d.quads = N.ptr(self.quads)
        d.n_quads = self.quads.shape[0]
        d.spheres = N.ptr(self.spheres)
        d.n_spheres = self.spheres.shape[0]
        d.prims = N.ptr(self.prims)
        d.n_prims = self.prims.shape[0]
        bv = (N.BvhDesc * len(self.bvh_clusters))()
        for i, (cl, root) in enumerate(zip(self.bvh_clusters, self.bvh_roots)):
            bv[i].clusters = N.ptr(cl)
            bv[i].n_clusters = cl.shape[0]
            bv[i].root = N.RefNode(int(root["count"]), int(root["active"]), int(root["perm"]), 0,
                                   int(root["cluster_idx"]))
            bv[i].prim_base = self.bvh_prim_base[i]
            bv[i].n_prims = self.bvh_n_prims[i]
        self._bvh_keep = bv
        d.bvhs = C.cast(bv, C.c_void_p).value
        d.n_bvhs = len(self.bvh_clusters)
        d.materials = N.ptr(self.materials)
        d.n_materials = self.materials.shape[0]
        d.textures = N.ptr(self.textures)
        d.n_textures = self.textures.shape[0]
        d.images = N.ptr(self.images)
        d.n_images = self.images.shape[0]
        d.texels = N.ptr(self.texels)
        d.n_texel_bytes = self.texels.size
        if self.lights is None:
            raise RuntimeError("lights not bound: use an Integrator (bind_lights)")
        d.lights = N.ptr(self.lights)
        d.n_lights = self.lights.shape[0]
        d.light_sampler = self.light_sampler
        d.sampler_lights = N.ptr(self.sampler_lights)
        d.n_sampler_lights = self.sampler_lights.shape[0]
        d.infinite_lights = N.ptr(self.infinite_lights)
        d.n_infinite_lights = self.infinite_lights.shape[0]
        d.light_dist = N.ptr(self.light_dist) if self.light_dist.size else None
        d.n_light_dist = self.light_dist.shape[0]
        d.instances = N.ptr(self.instances)
        d.n_instances = 0 if self.instances is None else self.instances.shape[0]
        d.media = N.ptr(self.media)
        d.n_media = 0 if self.media is None else self.media.shape[0]
        d.scene_medium = self.scene_medium
        return d


class _Registry:
    def __init__(self):
        self.textures: List[np.void] = []
        self.tex_ids: Dict[int, int] = {}
        self.images: List[tuple] = []
        self.texel_chunks: List[np.ndarray] = []
        self.texel_bytes = 0
        self.materials: List[np.void] = []
        self.mat_ids: Dict[int, int] = {}

    def texture(self, t: Optional[Texture]) -> int:
        if t is None:
            return -1
        if id(t) in self.tex_ids:
            return self.tex_ids[id(t)]
        rec = np.zeros(1, dtype=N.TEXTURE)[0]
        rec["scale"] = t.colorScale
        rec["a"] = -1
        rec["b"] = -1
        rec["image"] = -1
        if isinstance(t, SolidColor):
            rec["kind"] = N.PT_TEX_SOLID
            # SolidColor::Evaluate = colorScale * albedo, precomputed in float32
            rec["value"] = (t.colorScale * t.albedo).astype(np.float32)
        elif isinstance(t, CheckerTexture):
            rec["kind"] = N.PT_TEX_CHECKER
            rec["a"] = self.texture(t.tex1)
            rec["b"] = self.texture(t.tex2)
            rec["inv_scale"] = t.invScale
        elif isinstance(t, ImageTexture):
            rec["kind"] = N.PT_TEX_IMAGE
            h, w, c = t.data.shape
            off = self.texel_bytes
            data = np.ascontiguousarray(t.data.reshape(-1))
            self.texel_chunks.append(data)
            self.texel_bytes += data.size
            pad = (-self.texel_bytes) % 16
            if pad:
                self.texel_chunks.append(np.zeros(pad, dtype=np.uint8))
                self.texel_bytes += pad
            rec["image"] = len(self.images)
            self.images.append((off, w, h, c, 0))
        elif isinstance(t, FloatImageTexture):
            # FloatImage texels (Texture.hpp:70-103): float32 bytes, 4-aligned
            rec["kind"] = N.PT_TEX_IMAGE
            h, w, c = t.data.shape
            off = self.texel_bytes
            data = np.ascontiguousarray(t.data.reshape(-1), np.float32).view(np.uint8)
            self.texel_chunks.append(data)
            self.texel_bytes += data.size
            pad = (-self.texel_bytes) % 16
            if pad:
                self.texel_chunks.append(np.zeros(pad, dtype=np.uint8))
                self.texel_bytes += pad
            rec["image"] = len(self.images)
            self.images.append((off, w, h, c, N.PT_IMAGE_F32))
        else:
            raise TypeError(f"unsupported texture {type(t).__name__}")
        self.tex_ids[id(t)] = len(self.textures)
        self.textures.append(rec)
        return self.tex_ids[id(t)]

    def material(self, m: Optional[Material]) -> int:
        if m is None:
            return -1
        if id(m) in self.mat_ids:
            return self.mat_ids[id(m)]
        rec = np.zeros(1, dtype=N.MATERIAL)[0]
        rec["kind"] = m.kind
        for k in ("tex", "norm", "rough", "metal", "alpha"):
            rec[k] = -1
        if isinstance(m, (MicrofacetDiffuse, MicrofacetDielectric)):
            rec["tex"] = self.texture(m.tex)
            rec["norm"] = self.texture(m.norm)
            rec["rough"] = self.texture(m.roughnessTexture)
            if isinstance(m, MicrofacetDiffuse):
                rec["metal"] = self.texture(m.metallicTexture)
            else:
                rec["ri"] = m.ri
            rec["alpha"] = self.texture(m.alpha)
            rec["alpha_mode"] = m.alphaTester.mode
            rec["alpha_cutoff"] = m.alphaTester.cutoff
        elif isinstance(m, ThinDielectric):
            rec["ri"] = m.ri
            rec["tex"] = self.texture(m.tex)
        elif isinstance(m, SpecularConductor):
            rec["albedo"] = m.albedo
        else:
            raise TypeError(f"unsupported material {type(m).__name__}")
        self.mat_ids[id(m)] = len(self.materials)
        self.materials.append(rec)
        return self.mat_ids[id(m)]


# Where model BLASes and the TLAS are built: the host builder (default) or the
# device build (pt_bvh4_build_device, byte-identical output) on that GPU for
# BVHs of at least BVH_DEVICE_MIN primitives (env PT_BVH_DEVICE=<gpu>, or
# set_bvh_device: bench.py builds C4's 10 M-triangle BLAS on each rank's own
# GPU in ~0.1 s instead of ~5 s of host cores shared by 8 ranks).
BVH_DEVICE: Optional[int] = (int(os.environ["PT_BVH_DEVICE"]) if os.environ.get("PT_BVH_DEVICE", "") != ""
                              else None)
BVH_DEVICE_MIN = 0
_last_build: list[str] = []


def set_bvh_device(device: Optional[int], min_prims: int = 0) -> None:
    global BVH_DEVICE, BVH_DEVICE_MIN
    BVH_DEVICE = device
    BVH_DEVICE_MIN = int(min_prims)


def last_bvh_build() -> str:
    """Where the BVHs of the last flatten were built, e.g. 'device 1 + host 1'."""
    if not _last_build:
        return "none"
    return " + ".join(f"{k} {_last_build.count(k)}" for k in ("device", "host") if k in _last_build)


def bvh_build(boxes: np.ndarray):
    n = np.asarray(boxes).reshape(-1, 6).shape[0]
    if BVH_DEVICE is None or n < BVH_DEVICE_MIN:
        _last_build.append("host")
        return N.bvh4_build(boxes)
    _last_build.append("device")
    return N.bvh4_build_device(boxes, device=BVH_DEVICE)


def _stack(recs, dtype):
    if not recs:
        return np.zeros(0, dtype=dtype)
    a = np.zeros(len(recs), dtype=dtype)
    for i, r in enumerate(recs):
        a[i] = r
    return a


def _fma32(a, b, c):
    return (np.asarray(a, np.float64) * np.asarray(b, np.float64) + np.asarray(c, np.float64)).astype(np.float32)


def mat4_mul_point(m: np.ndarray, p) -> np.ndarray:
    """glm mat4 * vec4(p, 1) (glm/detail/type_mat4x4.inl:561-572) as the
    reference build contracts it: fma(m0, x, m1*y) + fma(m2, z, m3*1)."""
    f = np.float32
    x, y, z = (f(v) for v in p)
    a0 = _fma32(m[0], x, (m[1] * y).astype(f))
    a1 = _fma32(m[2], z, m[3])
    return (a0 + a1).astype(f)[:3]


def instance_bbox(inner: np.ndarray, m: np.ndarray) -> np.ndarray:
    """TransformedPrimitive::BoundingBox (Primitive.cpp:32-40): the 8 corners
    (AABB::Corner, AABB.hpp:133-137) transformed and expanded in order."""
    lo, hi = inner[:3], inner[3:]
    pts = []
    for i in range(8):
        c = (lo[0] if not (i & 1) else hi[0], hi[1] if (i & 2) else lo[1], hi[2] if (i & 4) else lo[2])
        pts.append(mat4_mul_point(m, c))
    from .scene import _expand_seq
    return _expand_seq(pts)


def _chain(p):
    """(wrapper levels outermost first, the Model / GeometricPrimitive they
    wrap) of a TransformedPrimitive / AnimatedPrimitive, possibly nested
    (Primitive.cpp:32-96); ([], p) for anything else."""
    levels = []
    while isinstance(p, TransformedPrimitive):
        levels.append(p)
        p = p.primitive
    return levels, p


def flatten_scene(scene: Scene) -> FlatScene:
    _last_build.clear()
    reg = _Registry()
    top = scene.primitives
    if not top:
        raise ValueError("empty scene")

    # ---- models: BLAS over their triangles (top-level and instanced, once each) ----
    models, model_index = [], {}
    for p in top:
        m = _chain(p)[1]
        if isinstance(m, Model) and id(m) not in model_index:
            model_index[id(m)] = len(models)
            models.append(m)
    # instanced GeometricPrimitives: a one-primitive BLAS each
    gp_inst, gp_index = [], {}
    for p in top:
        m = _chain(p)[1]
        if isinstance(p, TransformedPrimitive) and isinstance(m, GeometricPrimitive):
            if id(m) not in gp_index:
                gp_index[id(m)] = len(gp_inst)
                gp_inst.append(m)
    pos, nrm, uvs, tan, vidx, tflags = [], [], [], [], [], []
    vbase = 0
    tri_base = 0
    model_tri_base = []
    model_tri_mat = []       # per model: material id per local triangle
    model_tri_med = []
    model_blas = []          # (clusters, root, order, bbox)
    for m in models:
        model_tri_base.append(tri_base)
        boxes = []
        mats, meds, med_objs = [], [], []
        for mesh in m.meshes:
            nv = mesh.vertices.shape[0]
            pos.append(mesh.vertices)
            nrm.append(mesh.normals)
            uvs.append(mesh.texCoords)
            tan.append(mesh.tangents if mesh.tangents is not None else np.zeros((nv, 3), np.float32))
            vidx.append(mesh.indices.reshape(-1, 3).astype(np.uint32) + np.uint32(vbase))
            nt = mesh.GetTriangleCount()
            tflags.append(np.full(nt, 1 if mesh.tangents is not None else 0, dtype=np.uint32))
            boxes.append(mesh.tri_bboxes())
            # Model::BuildBlas(material, medium) (Model.hpp:62-80) takes both
            # overrides, a null one included; BuildBlas() the meshes' own
            override = m.override_material is not None or m.override_medium is not None
            mat = m.override_material if override else mesh.material
            mats.append(np.full(nt, reg.material(mat), dtype=np.int32))
            med = m.override_medium if override else mesh.medium
            meds.append(np.full(nt, -1, dtype=np.int32))
            med_objs.append((len(meds) - 1, med))
            vbase += nv
            tri_base += nt
        bx = np.concatenate(boxes) if boxes else np.zeros((0, 6), np.float32)
        model_blas.append(bvh_build(bx))
        model_tri_mat.append(np.concatenate(mats) if mats else np.zeros(0, np.int32))
        model_tri_med.append((meds, med_objs))

    gp_blas = [N.bvh4_build(g.shape.bbox()[None]) for g in gp_inst]

    # ---- TLAS over top-level primitives ----
    quads, spheres = [], []
    top_boxes = np.zeros((len(top), 6), dtype=np.float32)
    model_of_top = {}
    for i, p in enumerate(top):
        if isinstance(p, Model):
            top_boxes[i] = model_blas[model_index[id(p)]][3]
            model_of_top[i] = model_index[id(p)]
        elif isinstance(p, GeometricPrimitive):
            top_boxes[i] = p.shape.bbox()
        elif isinstance(p, TransformedPrimitive):
            levels, m = _chain(p)
            box = model_blas[model_index[id(m)]][3] if isinstance(m, Model) else m.shape.bbox()
            for lv in reversed(levels):  # each wrapper boxes the box of what it wraps
                if isinstance(lv, AnimatedPrimitive):
                    # AnimatedPrimitive::BoundingBox (Primitive.cpp:76-80): the box at
                    # rest expanded by the box translated by the whole direction
                    moved = instance_bbox(box, mat4_translate(mat4_identity(), lv.direction))
                    box = _expand_seq([box[:3], box[3:], moved[:3], moved[3:]])
                else:
                    box = instance_bbox(box, lv.transform)
            top_boxes[i] = box
        else:
            raise TypeError(f"unsupported primitive {type(p).__name__}")
    tl_clusters, tl_root, tl_order, tl_bbox = bvh_build(top_boxes)

    n_top = len(top)
    n_blas_prims = sum(int(b[2].shape[0]) for b in model_blas) + len(gp_blas)
    prims = np.zeros(n_top + n_blas_prims, dtype=N.PRIM)
    prims["light"] = -1
    prims["medium"] = -1
    light_slot: Dict[int, int] = {}
    light_instance: Dict[int, int] = {}  # id(TransformedLight) -> instance index
    inner_area_lights = []               # AreaLights inside instances (hit identity)
    tlas_lights = []
    top_media = []  # (slot, medium object) of top-level primitives
    # BLAS slot ranges
    blas_base = []
    base = n_top
    for b in model_blas + gp_blas:
        blas_base.append(base)
        base += int(b[2].shape[0])
    instances = []  # pt_instance records, TLAS slot order
    # the inner levels of nested wrappers, after every record a TLAS slot names
    level_records = []
    n_top_inst = sum(1 for p in top if isinstance(p, TransformedPrimitive))
    virt_base = n_top + n_blas_prims

    def level_record(lv, b):
        ins = np.zeros(1, dtype=N.INSTANCE)[0]
        ins["transform"] = lv.transform.reshape(16)
        ins["inv"] = lv.invTransform.reshape(16)
        ins["bvh"] = b
        ins["inner"] = -1
        if isinstance(lv, AnimatedPrimitive):  # per-ray translation (Primitive.cpp:82-89)
            ins["motion"] = lv.direction
            ins["time_bounds"] = lv.timeBounds
            ins["animated"] = 1
        return ins

    # TLAS slots
    for slot in range(n_top):
        p = top[int(tl_order[slot])]
        rec = prims[slot]
        if isinstance(p, TransformedPrimitive):
            levels, m = _chain(p)
            b = 1 + (model_index[id(m)] if isinstance(m, Model) else len(model_blas) + gp_index[id(m)])
            ins = level_record(p, b)
            ins["virt_base"] = virt_base
            prev = ins
            for lv in levels[1:]:  # nested wrappers: a level record each, linked outermost first
                prev["inner"] = n_top_inst + len(level_records)
                prev = level_record(lv, b)
                level_records.append(prev)
            virt_base += int((model_blas + gp_blas)[b - 1][2].shape[0])
            rec["kind"] = N.PT_PRIM_INSTANCE
            rec["index"] = len(instances)
            rec["material"] = -1
            # TransformedPrimitive::GetLights: the inner primitive's lights
            # (a Model's in BLAS leaf order) wrapped (Primitive.cpp:66-73)
            inner_lights = []
            if isinstance(m, Model) and m.tri_lights:
                kb = model_index[id(m)]
                order = model_blas[kb][2]
                emissive = np.zeros(m.triangle_count(), dtype=bool)
                emissive[np.fromiter(m.tri_lights.keys(), dtype=np.int64)] = True
                inner_lights = [(m.tri_lights[int(order[j])], blas_base[kb] + int(j))
                                for j in np.nonzero(emissive[order])[0]]
            elif isinstance(m, GeometricPrimitive) and m.areaLight is not None:
                inner_lights = [(m.areaLight, blas_base[len(model_blas) + gp_index[id(m)]])]
            for al, bslot in inner_lights:
                tl = al
                for lv in reversed(levels):  # GetLights of each wrapper wraps the inner one's
                    tl = TransformedLight(tl, lv)
                light_slot[id(tl)] = bslot
                light_instance[id(tl)] = len(instances)
                light_slot[id(al)] = bslot
                inner_area_lights.append(al)
                tlas_lights.append(tl)
            instances.append(ins)
            continue
        if isinstance(p, Model):
            k = model_of_top[int(tl_order[slot])]
            rec["kind"] = N.PT_PRIM_BLAS
            rec["index"] = 1 + k
            rec["material"] = -1
            # lights of this model in BLAS leaf order
            order = model_blas[k][2]
            if p.tri_lights:
                emissive = np.zeros(p.triangle_count(), dtype=bool)
                emissive[np.fromiter(p.tri_lights.keys(), dtype=np.int64)] = True
                for j in np.nonzero(emissive[order])[0]:
                    al = p.tri_lights[int(order[j])]
                    light_slot[id(al)] = blas_base[k] + int(j)
                    tlas_lights.append(al)
        else:
            sh = p.shape
            if isinstance(sh, QuadShape):
                rec["kind"] = N.PT_PRIM_QUAD
                rec["index"] = len(quads)
                q = np.zeros(1, dtype=N.QUAD)[0]
                q["Q"], q["u"], q["v"], q["normal"], q["D"], q["w"] = sh.Q, sh.u, sh.v, sh.normal, sh.D, sh.w
                quads.append(q)
            elif isinstance(sh, SphereShape):
                rec["kind"] = N.PT_PRIM_SPHERE
                rec["index"] = len(spheres)
                s = np.zeros(1, dtype=N.SPHERE)[0]
                s["center"], s["radius"] = sh.center, sh.radius
                spheres.append(s)
            else:
                raise TypeError(f"unsupported shape {type(sh).__name__}")
            rec["material"] = reg.material(p.material)
            top_media.append((slot, p.medium))
            if p.areaLight is not None:
                light_slot[id(p.areaLight)] = slot
                tlas_lights.append(p.areaLight)
    # BLAS slots
    for k, b in enumerate(model_blas):
        order = b[2]
        s0 = blas_base[k]
        n = order.shape[0]
        prims["kind"][s0:s0 + n] = N.PT_PRIM_TRIANGLE
        prims["index"][s0:s0 + n] = order + np.uint32(model_tri_base[k])
        prims["material"][s0:s0 + n] = model_tri_mat[k][order]
        model_tri_med[k] = (order, s0, n, model_tri_med[k])
    # one-primitive BLASes of instanced GeometricPrimitives
    for j, g in enumerate(gp_inst):
        s0 = blas_base[len(model_blas) + j]
        rec = prims[s0]
        sh = g.shape
        if isinstance(sh, QuadShape):
            rec["kind"] = N.PT_PRIM_QUAD
            rec["index"] = len(quads)
            q = np.zeros(1, dtype=N.QUAD)[0]
            q["Q"], q["u"], q["v"], q["normal"], q["D"], q["w"] = sh.Q, sh.u, sh.v, sh.normal, sh.D, sh.w
            quads.append(q)
        else:
            rec["kind"] = N.PT_PRIM_SPHERE
            rec["index"] = len(spheres)
            s = np.zeros(1, dtype=N.SPHERE)[0]
            s["center"], s["radius"] = sh.center, sh.radius
            spheres.append(s)
        rec["material"] = reg.material(g.material)
        top_media.append((s0, g.medium))
    # emissive triangle lights: fill prim light ids later in bind_lights

    clusters = [tl_clusters] + [b[0] for b in model_blas + gp_blas]
    roots = [tl_root] + [b[1] for b in model_blas + gp_blas]
    pbase = [0] + blas_base
    npr = [n_top] + [int(b[2].shape[0]) for b in model_blas + gp_blas]

    cat = lambda xs, shape, dt: (np.ascontiguousarray(np.concatenate(xs), dtype=dt) if xs
                                 else np.zeros(shape, dtype=dt))
    flat = FlatScene(
        positions=cat(pos, (0, 3), np.float32), normals=cat(nrm, (0, 3), np.float32),
        uvs=cat(uvs, (0, 2), np.float32), tangents=cat(tan, (0, 3), np.float32),
        tri_vidx=cat(vidx, (0, 3), np.uint32), tri_flags=cat(tflags, (0,), np.uint32),
        quads=_stack(quads, N.QUAD), spheres=_stack(spheres, N.SPHERE), prims=prims,
        bvh_clusters=clusters, bvh_roots=roots, bvh_prim_base=pbase, bvh_n_prims=npr,
        materials=_stack(reg.materials, N.MATERIAL), textures=_stack(reg.textures, N.TEXTURE),
        images=np.array(reg.images, dtype=N.IMAGE) if reg.images else np.zeros(0, dtype=N.IMAGE),
        texels=(np.ascontiguousarray(np.concatenate(reg.texel_chunks)) if reg.texel_chunks
                else np.zeros(0, dtype=np.uint8)),
        bbox=tl_bbox, tlas_lights=tlas_lights, light_slot=light_slot, material_ids=dict(reg.mat_ids),
        top_order=tl_order, blas_orders=[b[2] for b in model_blas], model_tri_base=model_tri_base,
        texture_ids=dict(reg.tex_ids))
    flat._reg = reg
    flat.instances = _stack(instances + level_records, N.INSTANCE)
    flat.light_instance = light_instance
    flat.inner_area_lights = inner_area_lights
    # media: the scene's first, then primitives in slot order, then meshes
    flat.scene_medium = flat.medium_id(scene.GetMedium())
    for slot, md in top_media:
        prims["medium"][slot] = flat.medium_id(md)
    for order, s0, n, (meds, med_objs) in model_tri_med:
        for j, md in med_objs:
            meds[j][:] = flat.medium_id(md)
        tri_med = np.concatenate(meds) if meds else np.zeros(0, np.int32)
        prims["medium"][s0:s0 + n] = tri_med[order]
    return flat


def bind_lights(flat: FlatScene, scene: Scene, sampler: Optional[LightSampler]):
    """Light table = Scene::GetLights() + lights added only to the sampler;
    power/pmf as the sampler's PreProcess left them (LightSampler.cpp)."""
    reg = flat._reg
    lights = list(flat.tlas_lights) + list(scene.infiniteLights)
    seen = {id(l) for l in lights}
    if sampler is not None:
        for l in sampler.all_lights:
            if id(l) not in seen:
                lights.append(l)
                seen.add(id(l))
    # the inner AreaLight of an emitter inside an instance: what a path that
    # hits it sees (interaction.AreaLight, Primitive.cpp:58), not in the sampler
    for l in getattr(flat, "inner_area_lights", []):
        if id(l) not in seen:
            lights.append(l)
            seen.add(id(l))
    idx = {id(l): i for i, l in enumerate(lights)}
    table = np.zeros(len(lights), dtype=N.LIGHT)
    table["prim"] = -1
    table["tex"] = -1
    table["instance"] = -1
    dists = []  # TEX_INF running sums, concatenated
    for i, l in enumerate(lights):
        r = table[i]
        r["power"] = l.Power()
        r["pmf"] = sampler.PMF(l) if sampler is not None else 0.0
        if isinstance(l, TransformedLight):
            r["kind"] = N.PT_LIGHT_AREA
            r["prim"] = flat.light_slot[id(l)]
            r["tex"] = reg.texture(l.area.emissiveTexture)
            r["one_sided"] = 1 if l.area.oneSided else 0
            r["instance"] = flat.light_instance[id(l)]
        elif isinstance(l, AreaLight):
            r["kind"] = N.PT_LIGHT_AREA
            r["prim"] = flat.light_slot[id(l)]
            r["tex"] = reg.texture(l.emissiveTexture)
            r["one_sided"] = 1 if l.oneSided else 0
        elif isinstance(l, UniformInfiniteLight):
            r["kind"] = N.PT_LIGHT_UNIFORM_INF
            r["color"] = l.color
        elif isinstance(l, FunctionInfiniteLight):
            r["kind"] = N.PT_LIGHT_SKY_INF
            r["color"] = l.c0
            r["vec"] = l.c1
            r["scale"] = l.scale
        elif isinstance(l, TextureInfiniteLight):
            if l.accWeights is None:  # no light sampler ran PreProcess (SimplePath): Le only
                l.PreProcess(flat.bbox)
            r["kind"] = N.PT_LIGHT_TEX_INF
            r["tex"] = reg.texture(l.tex)
            r["scale"] = l.LeScale
            r["prim"] = sum(a.shape[0] for a in dists)
            dists.append(l.accWeights)
        elif isinstance(l, DistantLight):
            r["kind"] = N.PT_LIGHT_DISTANT
            r["color"] = l.color
            r["vec"] = l.dir
        elif isinstance(l, PointLight):
            r["kind"] = N.PT_LIGHT_POINT
            r["color"] = l.color
            r["vec"] = l.p
        else:
            raise TypeError(f"unsupported light {type(l).__name__}")
    # prim -> area light id
    flat.prims["light"] = -1
    for i, l in enumerate(lights):
        if isinstance(l, AreaLight):
            flat.prims["light"][flat.light_slot[id(l)]] = i
    # textures may have grown (emissive textures)
    flat.textures = _stack(reg.textures, N.TEXTURE)
    flat.images = np.array(reg.images, dtype=N.IMAGE) if reg.images else np.zeros(0, dtype=N.IMAGE)
    flat.texels = (np.ascontiguousarray(np.concatenate(reg.texel_chunks)) if reg.texel_chunks
                   else np.zeros(0, dtype=np.uint8))
    flat.lights = table
    flat.light_dist = np.ascontiguousarray(np.concatenate(dists) if dists else np.zeros(0, np.float32), np.float32)
    flat.light_objects = lights
    flat.light_sampler = sampler.kind if sampler is not None else N.PT_LS_UNIFORM
    flat.sampler_lights = np.array([idx[id(l)] for l in (sampler.lights if sampler is not None else [])],
                                   dtype=np.uint32)
    flat.infinite_lights = np.array([idx[id(l)] for l in scene.infiniteLights], dtype=np.uint32)
    return flat


def camera_desc(cam, flat: Optional[FlatScene] = None) -> N.CameraDesc:
    d = N.CameraDesc()
    md = cam.GetMedium() if hasattr(cam, "GetMedium") else None
    if md is not None and (flat is None or id(md) not in flat.medium_ids):
        raise ValueError("camera medium not registered with the flat scene (use an Integrator)")
    d.medium = -1 if md is None else flat.medium_ids[id(md)]
    d.origin[:] = [float(x) for x in cam.lookFrom]
    d.u[:] = [float(x) for x in cam.u]
    d.v[:] = [float(x) for x in cam.v]
    d.w[:] = [float(x) for x in cam.w]
    d.half_width = float(cam.halfWidth)
    d.half_height = float(cam.halfHeight)
    d.defocus_radius = float(cam.defocusRadius)
    d.focus_distance = float(cam.FocusDistance)
    d.focus_angle = float(cam.FocusAngle)
    sh = getattr(cam, "shutter", None)
    d.has_shutter = 0 if sh is None else 1
    if sh is not None:
        d.shutter[:] = [float(sh[0]), float(sh[1])]
    W, H = cam.film.Resolution()
    d.width = W
    d.height = H
    return d
