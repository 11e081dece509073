"""Scene library: the BASELINE.json configurations and the parity scenes.

  example_1     C1 — examples/example_1.cpp:20-75 (checker floor, green sphere,
                red 600x quad light, HG medium sphere, uniform sky)
  cornell       C2 (diffuse, SimplePath) / C3 (+ rough glass sphere, mirror and
                metallic boxes, PathIntegrator NEE+MIS+RR) — SURVEY.md §8(d)
  material_zoo  parity scene exercising every material/texture/light kind
  heightfield   procedural triangle mesh (BVH stress; SURVEY.md §6 probe)
  sanmiguel     C4 — San-Miguel-class procedural scene (see function doc)

Every constructor returns (scene, camera, integrator_name, light_sampler,
max_depth, extra_lights) in the reference's own vocabulary; nothing here
touches a GPU.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from .scene import (AlphaMode, AlphaTester, AreaLight, Camera, CheckerTexture, DistantLight, Film,
                    FloatImageTexture, TextureInfiniteLight,
                    FunctionInfiniteLight, GeometricPrimitive, HenyeyGreenstein, HomogeneusMedium, ImageTexture,
                    Mesh,
                    MicrofacetDielectric, MicrofacetDiffuse, MitchellFilter, Model, PointLight, PowerLightSampler,
                    QuadShape, Scene, SolidColor, SpecularConductor, SphereShape, ThinDielectric,
                    UniformInfiniteLight, UniformLightSampler)


@dataclass
class SceneSetup:
    scene: Scene
    camera: Camera
    integrator: str            # "path" | "simple" | "volpath"
    light_sampler: object
    max_depth: int
    seed: int
    spp: int
    extra_lights: list = field(default_factory=list)
    strata: Optional[tuple] = None  # (xSamples, ySamples): a StratifiedSampler host

    def finish(self):
        """BuildTlas + LightSampler::Add/PreProcess, as main.cpp:300-306."""
        self.scene.BuildTlas()
        if self.light_sampler is not None:
            self.light_sampler.Add(self.scene.GetLights())
            for l in self.extra_lights:
                self.light_sampler.Add(l)
            self.light_sampler.PreProcess(self.scene.BoundingBox())
        return self

    def make_integrator(self):
        from .integrator import PathIntegrator, PCGSampler, SimplePathIntegrator, StratifiedSampler, VolPathIntegrator
        if self.strata:
            sampler = StratifiedSampler(self.strata[0], self.strata[1], self.seed)
            assert sampler.SamplesPerPixel() == self.spp
        else:
            sampler = PCGSampler(self.spp, self.seed)
        if self.integrator == "simple":
            return SimplePathIntegrator(self.scene, self.camera, sampler, self.max_depth)
        if self.integrator == "volpath":
            return VolPathIntegrator(self.scene, self.camera, sampler, self.light_sampler, self.max_depth)
        return PathIntegrator(self.scene, self.camera, sampler, self.light_sampler, self.max_depth)


# --------------------------------------------------------------------------
def example_1(W: int = 256, H: int = 256, spp: int = 16, integrator: str = "path", max_depth: int = 8,
              seed: int = 0x5EED0001, medium: bool = True, filt=None, lens=None) -> SceneSetup:
    """C1: examples/example_1.cpp:17-104 (UniformLightSampler, Mitchell 1.5).
    `filt` replaces the film's filter, `lens` = (FocusAngle, FocusDistance)
    turns on the thin lens (Camera.hpp:27-33)."""
    scene = Scene()
    white = SolidColor((0.9, 0.9, 0.9))
    green = SolidColor((0.2, 0.3, 0.1))
    checker_mat = MicrofacetDiffuse(CheckerTexture(white, green, (0.001, 0.001)))
    sphere_mat = MicrofacetDiffuse(green)
    floor = QuadShape((-100, -0.3, -100), (1000, 0, 0), (0, 0, 1000))
    sphere = SphereShape((0, 0.1, -1.2), 0.5)
    medium_sphere = SphereShape((1, 0, -1), 0.5)
    light_shape = QuadShape((-1, -0.28, -1), (0.2, 0, -0.2), (0, 0.2, 0))
    light_color = np.array([1, 0, 0], np.float32) * np.float32(600)
    area = AreaLight(light_shape, light_color, False)
    scene.Add(GeometricPrimitive(floor, checker_mat, None, None))
    scene.Add(GeometricPrimitive(sphere, sphere_mat, None))
    scene.Add(GeometricPrimitive(area.getShape(), MicrofacetDiffuse((0, 0, 0)), area, None))
    if medium:
        med = HomogeneusMedium((0.01, 0.9, 0.9), (1.0, 0.1, 0.1), 0.8, 5.0)
        scene.Add(GeometricPrimitive(medium_sphere, None, None, med))
    scene.infiniteLights.append(UniformInfiniteLight((0.45, 0.65, 1)))
    film = Film((W, H), filt or MitchellFilter())
    camera = Camera((0.3, 0.4, 1), (0, 0, 0), 1.7, film, *(lens or (0.0, 0.0)))
    return SceneSetup(scene, camera, integrator, UniformLightSampler(), max_depth, seed, spp).finish()


# --------------------------------------------------------------------------
def _quad_tris(p0, p1, p2, p3):
    """Two triangles (p0,p1,p2),(p0,p2,p3) with a flat normal and unit uvs."""
    v = np.array([p0, p1, p2, p3], np.float32)
    n = np.cross(v[1] - v[0], v[2] - v[0])
    n = (n / np.linalg.norm(n)).astype(np.float32)
    nrm = np.repeat(n[None], 4, 0)
    uv = np.array([[0, 0], [1, 0], [1, 1], [0, 1]], np.float32)
    idx = np.array([0, 1, 2, 0, 2, 3], np.uint32)
    return idx, v, nrm, uv


def _merge(parts):
    idx, vs, ns, uvs = [], [], [], []
    base = 0
    for i, v, n, uv in parts:
        idx.append(i + base)
        vs.append(v)
        ns.append(n)
        uvs.append(uv)
        base += v.shape[0]
    return (np.concatenate(idx).astype(np.uint32), np.concatenate(vs).astype(np.float32),
            np.concatenate(ns).astype(np.float32), np.concatenate(uvs).astype(np.float32))


def _box(center, size, angle):
    cx, cy, cz = center
    sx, sy, sz = size
    c, s = math.cos(angle), math.sin(angle)

    def P(x, y, z):
        x, z = x - cx, z - cz
        return (cx + c * x - s * z, y, cz + s * x + c * z)
    x0, x1, y0, y1, z0, z1 = cx - sx / 2, cx + sx / 2, cy - sy / 2, cy + sy / 2, cz - sz / 2, cz + sz / 2
    faces = [
        (P(x0, y1, z0), P(x0, y1, z1), P(x1, y1, z1), P(x1, y1, z0)),  # top
        (P(x0, y0, z1), P(x1, y0, z1), P(x1, y1, z1), P(x0, y1, z1)),  # +z
        (P(x1, y0, z0), P(x0, y0, z0), P(x0, y1, z0), P(x1, y1, z0)),  # -z
        (P(x1, y0, z1), P(x1, y0, z0), P(x1, y1, z0), P(x1, y1, z1)),  # +x
        (P(x0, y0, z0), P(x0, y0, z1), P(x0, y1, z1), P(x0, y1, z0)),  # -x
        (P(x0, y0, z0), P(x1, y0, z0), P(x1, y0, z1), P(x0, y0, z1)),  # bottom
    ]
    return _merge([_quad_tris(*f) for f in faces])


def tie_models(W: int = 32, H: int = 32, spp: int = 4, max_depth: int = 8, seed: int = 0x5EED0035) -> SceneSetup:
    """Exact-t ties across BLAS hops: the Cornell walls as two identical
    Models with different materials, plus a third copy of the floor beside a
    quad light in the TLAS.  Identical boxes cannot be split, so the TLAS
    holds the Models in one leaf; every wall hit is a tie, which the
    reference breaks by visit order: it recurses into each Model inside its
    leaf loop (Model::Intersect, BVH.hpp:1206) and a tie accepts the later
    hit (Primitive.cpp:6-26).  A traversal that visits a leaf's BLAS after
    the rest of the leaf picks the other Model."""
    scene = Scene()
    walls = [
        _quad_tris((-1, -1, 1), (1, -1, 1), (1, -1, -1), (-1, -1, -1)),   # floor
        _quad_tris((-1, -1, -1), (1, -1, -1), (1, 1, -1), (-1, 1, -1)),   # back
        _quad_tris((-1, -1, 1), (-1, -1, -1), (-1, 1, -1), (-1, 1, 1)),   # left
        _quad_tris((1, -1, -1), (1, -1, 1), (1, 1, 1), (1, 1, -1)),       # right
    ]
    mats = [MicrofacetDiffuse((0.73, 0.73, 0.73)), MicrofacetDiffuse((0.65, 0.05, 0.05)),
            MicrofacetDiffuse((0.12, 0.45, 0.15))]
    for m in mats:
        scene.Add(Model([Mesh(i, v, None, n, uv, m) for (i, v, n, uv) in walls]))
    light = AreaLight(QuadShape((-0.25, 0.999, -0.25), (0.5, 0, 0), (0, 0, 0.5)), (17.0, 12.0, 4.0), False)
    scene.Add(GeometricPrimitive(light.getShape(), MicrofacetDiffuse((0.78, 0.78, 0.78)), light))
    camera = Camera((0, 0, 3.7), (0, 0, 0), 0.75, Film((W, H), MitchellFilter()))
    return SceneSetup(scene, camera, "path", UniformLightSampler(), max_depth, seed, spp).finish()


def tie_instances(W: int = 32, H: int = 32, spp: int = 4, max_depth: int = 8,
                  seed: int = 0x5EED0036) -> SceneSetup:
    """Exact-t ties inside instances: tie_models' three wall Models (same
    geometry, three materials), each instanced under the same rotation and
    scale (TransformedPrimitive, Primitive.cpp:42-64).  The three instances
    have identical boxes, so the TLAS holds them in one leaf, and every wall
    hit is a tie met again inside each instance: the exact re-trace must list
    such a ray once (pt_pool.h OCT_TIE across instance enter / exit) and pick
    the instance the reference's recursion order picks."""
    from .scene import TransformedPrimitive, mat4_identity, mat4_rotate, mat4_scale
    scene = Scene()
    walls = [
        _quad_tris((-1, -1, 1), (1, -1, 1), (1, -1, -1), (-1, -1, -1)),   # floor
        _quad_tris((-1, -1, -1), (1, -1, -1), (1, 1, -1), (-1, 1, -1)),   # back
        _quad_tris((-1, -1, 1), (-1, -1, -1), (-1, 1, -1), (-1, 1, 1)),   # left
        _quad_tris((1, -1, -1), (1, -1, 1), (1, 1, 1), (1, 1, -1)),       # right
    ]
    mats = [MicrofacetDiffuse((0.73, 0.73, 0.73)), MicrofacetDiffuse((0.65, 0.05, 0.05)),
            MicrofacetDiffuse((0.12, 0.45, 0.15))]
    xf = mat4_scale(mat4_rotate(mat4_identity(), 0.15, (0, 1, 0)), (1.05, 1.0, 0.95))
    for m in mats:
        scene.Add(TransformedPrimitive(Model([Mesh(i, v, None, n, uv, m) for (i, v, n, uv) in walls]), xf))
    light = AreaLight(QuadShape((-0.25, 0.95, -0.25), (0.5, 0, 0), (0, 0, 0.5)), (17.0, 12.0, 4.0), False)
    scene.Add(GeometricPrimitive(light.getShape(), MicrofacetDiffuse((0.78, 0.78, 0.78)), light))
    camera = Camera((0, 0, 3.7), (0, 0, 0), 0.75, Film((W, H), MitchellFilter()))
    return SceneSetup(scene, camera, "path", UniformLightSampler(), max_depth, seed, spp).finish()


def cornell(W: int = 1024, H: int = 1024, spp: int = 256, config: str = "c2", max_depth: int = 8,
            seed: Optional[int] = None, fog: bool = False, filt=None, lens=None) -> SceneSetup:
    """C2/C3 Cornell box: 5 walls + 2 boxes as one triangle Model (34 tris) and
    a quad area light under the ceiling.  C2: MicrofacetDiffuse(albedo)
    (roughness 1, metallic 0), SimplePathIntegrator.  C3: + rough glass sphere
    MicrofacetDielectric(1.5, 0.15), mirror SpecularConductor tall box,
    metallic MicrofacetDiffuse(metallic 1, rough 0.3) short box,
    PathIntegrator with UniformLightSampler.  maxDepth 8."""
    c3 = config == "c3" or fog
    if seed is None:
        seed = 0x5EED0005 if fog else (0x5EED0003 if c3 else 0x5EED0002)
    # fog: the C3 box filled with a thin forward-scattering medium (scene and
    # camera medium, main.cpp:150-153, 264-266), an emissive medium inside the
    # glass sphere (main.cpp:208) and a medium-only sphere boundary, lit also
    # by a point light: VolPathIntegrator
    fog_md = HomogeneusMedium((0.05, 0.05, 0.08), (0.6, 0.6, 0.5), HenyeyGreenstein(0.6), 0.35) if fog else None
    scene = Scene(fog_md)
    white = MicrofacetDiffuse((0.73, 0.73, 0.73))
    red = MicrofacetDiffuse((0.65, 0.05, 0.05))
    green = MicrofacetDiffuse((0.12, 0.45, 0.15))
    walls = [
        (_quad_tris((-1, -1, 1), (1, -1, 1), (1, -1, -1), (-1, -1, -1)), white),   # floor
        (_quad_tris((-1, 1, -1), (1, 1, -1), (1, 1, 1), (-1, 1, 1)), white),       # ceiling
        (_quad_tris((-1, -1, -1), (1, -1, -1), (1, 1, -1), (-1, 1, -1)), white),   # back
        (_quad_tris((-1, -1, 1), (-1, -1, -1), (-1, 1, -1), (-1, 1, 1)), red),     # left
        (_quad_tris((1, -1, -1), (1, -1, 1), (1, 1, 1), (1, 1, -1)), green),       # right
    ]
    meshes = [Mesh(i, v, None, n, uv, m) for (i, v, n, uv), m in walls]
    tall = _box((-0.35, -0.4, -0.35), (0.6, 1.2, 0.6), 0.3)
    short = _box((0.4, -0.7, 0.3), (0.6, 0.6, 0.6), -0.3)
    if c3:
        tall_mat = SpecularConductor((0.95, 0.93, 0.88))
        short_mat = MicrofacetDiffuse(SolidColor((1.0, 0.78, 0.34)), None, SolidColor((0.3, 0.3, 0.3)),
                                      SolidColor((1, 1, 1)))
    else:
        tall_mat = white
        short_mat = white
    meshes.append(Mesh(*tall[:1], tall[1], None, tall[2], tall[3], tall_mat))
    meshes.append(Mesh(*short[:1], short[1], None, short[2], short[3], short_mat))
    scene.Add(Model(meshes))
    light = AreaLight(QuadShape((-0.25, 0.999, -0.25), (0.5, 0, 0), (0, 0, 0.5)), (17.0, 12.0, 4.0), False)
    scene.Add(GeometricPrimitive(light.getShape(), MicrofacetDiffuse((0.78, 0.78, 0.78)), light))
    extra = []
    if c3:
        inner = (HomogeneusMedium((0.2, 0.4, 0.6), (1.5, 1.0, 0.5), HenyeyGreenstein(-0.3), 2.0, (0.4, 0.6, 1.0), 1.5)
                 if fog else None)
        scene.Add(GeometricPrimitive(SphereShape((0.35, 0.05, 0.35), 0.3),
                                     MicrofacetDielectric(1.5, 0.15, (1, 1, 1)), None, inner))
    if fog:
        # medium-only boundary: a sphere (a mesh without material would crash
        # the reference's TriangleShape::Intersect, Shape.cpp:237-241)
        dense = HomogeneusMedium((0.9, 0.3, 0.1), (2.0, 3.0, 4.0), 0.0, 1.0)
        scene.Add(GeometricPrimitive(SphereShape((-0.55, 0.45, 0.45), 0.22), None, None, dense))
        extra.append(PointLight((0.5, 0.6, 0.6), (0.8, 0.8, 1.2)))
    film = Film((W, H), filt or MitchellFilter())
    camera = Camera((0, 0, 3.7), (0, 0, 0), 0.75, film, *(lens or (0.0, 0.0)), medium=fog_md)
    kind = "volpath" if fog else ("path" if c3 else "simple")
    ls = PowerLightSampler() if fog else (UniformLightSampler() if c3 else None)
    return SceneSetup(scene, camera, kind, ls, max_depth, seed, spp, extra).finish()


def lit_instances(W: int = 1024, H: int = 1024, spp: int = 256, max_depth: int = 8,
                  seed: int = 0x5EED0061) -> SceneSetup:
    """Emitters inside instances (§8f f2): an emissive lamp Model (a box mesh,
    one AreaLight per triangle) at the top level and instanced twice under
    rotate / non-uniform scale / translate (TransformedLight: Power x det),
    an instanced one-sided quad light and an AnimatedPrimitive emissive sphere
    (AnimatedLight), in the C2 room under its ceiling light;
    PathIntegrator, PowerLightSampler (Light.cpp:300-364, Primitive.cpp:66-96)."""
    from .scene import (AnimatedPrimitive, TransformedPrimitive, mat4_identity, mat4_rotate, mat4_scale,
                        mat4_translate)
    scene = Scene()
    white = MicrofacetDiffuse((0.73, 0.73, 0.73))
    red = MicrofacetDiffuse((0.65, 0.05, 0.05))
    green = MicrofacetDiffuse((0.12, 0.45, 0.15))
    walls = [
        (_quad_tris((-1, -1, 1), (1, -1, 1), (1, -1, -1), (-1, -1, -1)), white),
        (_quad_tris((-1, 1, -1), (1, 1, -1), (1, 1, 1), (-1, 1, 1)), white),
        (_quad_tris((-1, -1, -1), (1, -1, -1), (1, 1, -1), (-1, 1, -1)), white),
        (_quad_tris((-1, -1, 1), (-1, -1, -1), (-1, 1, -1), (-1, 1, 1)), red),
        (_quad_tris((1, -1, -1), (1, -1, 1), (1, 1, 1), (1, 1, -1)), green),
    ]
    scene.Add(Model([Mesh(i, v, None, n, uv, m) for (i, v, n, uv), m in walls]))
    light = AreaLight(QuadShape((-0.25, 0.999, -0.25), (0.5, 0, 0), (0, 0, 0.5)), (6.0, 5.0, 4.0), False)
    scene.Add(GeometricPrimitive(light.getShape(), MicrofacetDiffuse((0.78, 0.78, 0.78)), light))
    bi, bv, bn, buv = _box((0, 0, 0), (0.16, 0.1, 0.16), 0.2)
    lamp = Model([Mesh(bi, bv, None, bn, buv, MicrofacetDiffuse((0.8, 0.8, 0.8)), SolidColor((3.0, 2.2, 1.2)))])
    scene.Add(lamp)  # top level: its AreaLights directly
    for pos, ang, ax, sc in [((-0.55, -0.7, -0.2), 0.7, (0, 1, 0), (1.5, 0.8, 1.2)),
                             ((0.5, 0.45, -0.45), -1.1, (1, 0, 1), (0.9, 1.6, 0.9))]:
        m = mat4_scale(mat4_rotate(mat4_translate(mat4_identity(), pos), ang, ax), sc)
        scene.Add(TransformedPrimitive(lamp, m))
    ql = AreaLight(QuadShape((-0.5, 0, -0.5), (1, 0, 0), (0, 0, 1)), (2.0, 3.0, 4.0), True)
    panel = GeometricPrimitive(ql.getShape(), MicrofacetDiffuse((0.5, 0.5, 0.5)), ql)
    scene.Add(TransformedPrimitive(panel, mat4_rotate(mat4_scale(mat4_translate(mat4_identity(), (0.6, -0.3, 0.3)),
                                                                  (0.3, 1, 0.2)), 2.0, (1, 0, 0.2))))
    sl = AreaLight(SphereShape((-0.3, -0.8, 0.5), 0.1), (5.0, 1.5, 1.0), False)
    scene.Add(AnimatedPrimitive(GeometricPrimitive(sl.getShape(), MicrofacetDiffuse((0.9, 0.9, 0.9)), sl),
                                (0.3, 0.2, 0), (0.25, 1.0)))
    film = Film((W, H), MitchellFilter())
    camera = Camera((0, 0, 3.7), (0, 0, 0), 0.75, film)
    return SceneSetup(scene, camera, "path", PowerLightSampler(), max_depth, seed, spp).finish()


def env_texels(rng, w: int = 64, h: int = 32) -> np.ndarray:
    """A procedural HDR sky (sky gradient + a bright sun blob + noise) whose
    float values are exact Radiance RGBE decodes (m * 2^(e - 136)), so the
    .hdr file a recipe writes decodes (stbi_loadf) to the very same floats."""
    y = (np.arange(h, dtype=np.float64) + 0.5) / h
    x = (np.arange(w, dtype=np.float64) + 0.5) / w
    X, Y = np.meshgrid(x, y)
    base = np.stack([0.4 + 0.6 * Y, 0.55 + 0.4 * Y, 0.9 + 0.2 * (1 - Y)], -1)
    sun = 40.0 * np.exp(-(((X - 0.3) / 0.05) ** 2 + ((Y - 0.35) / 0.08) ** 2))[..., None] * np.array([1.0, 0.9, 0.7])
    v = base * (0.8 + 0.4 * rng.random((h, w, 1))) + sun
    e = np.ceil(np.log2(np.maximum(v.max(-1), 1e-30))).astype(np.int64)  # shared exponent: max < 2^e
    m = np.clip(np.floor(v / np.exp2(e - 8)[..., None]), 0, 255).astype(np.int64)
    rgbe = np.concatenate([m, (e + 128)[..., None]], -1).astype(np.uint8)
    rgbe[0, 0, 0] = max(3, int(rgbe[0, 0, 0]))  # a flat (not run-length) file: first byte != 2
    return rgbe


def rgbe_decode(rgbe: np.ndarray) -> np.ndarray:
    """stbi__hdr_convert: m * ldexp(1, e - 136) in float, 0 for e = 0."""
    f = np.ldexp(np.float32(1.0), rgbe[..., 3].astype(np.int32) - 136).astype(np.float32)
    out = (rgbe[..., :3].astype(np.float32) * f[..., None]).astype(np.float32)
    out[rgbe[..., 3] == 0] = 0.0
    return out


def envmap(W: int = 256, H: int = 256, spp: int = 16, max_depth: int = 8, seed: int = 0x5EED0071,
           le_scale: float = 1.5, integrator: str = "path") -> SceneSetup:
    """C1's floor and spheres under a TextureInfiniteLight (Light.cpp:110-200)
    over a FloatImageTexture HDR sky (main.cpp:115-116, 222-224 use one),
    PowerLightSampler (main.cpp's) with the red quad light."""
    rng = np.random.default_rng(71)
    rgbe = env_texels(rng)
    sky = FloatImageTexture(rgbe_decode(rgbe))
    sky.rgbe = rgbe
    s = example_1(W=W, H=H, spp=spp, integrator=integrator, max_depth=max_depth, seed=seed, medium=False)
    scene = s.scene
    scene.infiniteLights = [TextureInfiniteLight(sky, le_scale)]
    return SceneSetup(scene, s.camera, integrator, PowerLightSampler(), max_depth, seed, spp).finish()


def textured_emitters(W: int = 32, H: int = 32, spp: int = 4, seed: int = 0x5EED0081) -> SceneSetup:
    """Area lights with textured emission (AreaLight::PreProcess averages the
    emissive texture over its shape, Light.cpp:277-287): an image-textured
    quad, a checker-emission sphere and an image-textured emissive mesh in the
    C2 room; PowerLightSampler."""
    rng = np.random.default_rng(81)
    s = cornell(W=W, H=H, spp=spp, config="c2", seed=seed)
    scene = s.scene
    img = _noise_img(rng, 16, 16, 3, lo=40, hi=255, smooth=2)
    ql = AreaLight(QuadShape((-0.6, -0.9, -0.6), (0.3, 0, 0), (0, 0.2, 0.1)), ImageTexture(img, True, (6, 5, 4)), True)
    scene.Add(GeometricPrimitive(ql.getShape(), MicrofacetDiffuse((0.5, 0.5, 0.5)), ql))
    sl = AreaLight(SphereShape((0.5, -0.2, 0.4), 0.12),
                   CheckerTexture(SolidColor((4, 4, 3)), SolidColor((0.5, 0.5, 2)), (0.1, 0.2)), False)
    scene.Add(GeometricPrimitive(sl.getShape(), MicrofacetDiffuse((0.9, 0.9, 0.9)), sl))
    bi, bv, bn, buv = _box((-0.3, 0.5, -0.4), (0.2, 0.2, 0.2), 0.4)
    scene.Add(Model([Mesh(bi, bv, None, bn, buv, MicrofacetDiffuse((0.8, 0.8, 0.8)),
                          ImageTexture(_noise_img(rng, 8, 8, 3, lo=100, hi=255, smooth=1), False, (3, 3, 3)))]))
    return SceneSetup(scene, s.camera, "path", PowerLightSampler(), 8, seed, spp).finish()


def blend_box(W: int = 64, H: int = 64, spp: int = 16, max_depth: int = 8, alpha: float = 0.35,
              seed: int = 0x5EED0041) -> SceneSetup:
    """C3 Cornell box behind a see-through panel: a two-triangle mesh with a
    constant alpha texture under AlphaTester Blend (Material.hpp:181-198), so
    every ray crossing it passes with probability 1 - alpha (the reference's
    hidden random_float() < a, Material.hpp:189)."""
    setup = cornell(W=W, H=H, spp=spp, config="c3", max_depth=max_depth, seed=seed)
    scene = setup.scene
    panel = _quad_tris((-0.55, -0.6, 1.2), (0.55, -0.6, 1.2), (0.55, 0.5, 1.2), (-0.55, 0.5, 1.2))
    mat = MicrofacetDiffuse(SolidColor((0.1, 0.6, 0.2)), None, None, None, SolidColor((alpha, alpha, alpha)))
    mat.setAlphaTester(AlphaTester(AlphaMode.Blend))
    idx, v, n, uv = panel
    scene.Add(Model([Mesh(idx, v, None, n, uv, mat)]))
    return SceneSetup(scene, setup.camera, setup.integrator, UniformLightSampler(), max_depth, seed, spp).finish()


def alpha_maps(W: int = 32, H: int = 32, spp: int = 4, max_depth: int = 8, seed: int = 0x5EED0042) -> SceneSetup:
    """C3 Cornell box behind panels cut by every deterministic alpha source
    (AlphaTester Mask, Material.hpp:181-198): an RGB alpha texture with a
    colorScale (Evaluate(uv).x * scale), a one-channel alpha texture, a solid
    alpha below the cutoff (never passes), an RGBA albedo's fourth channel
    (Texture::alpha), and a rough dielectric with an alpha texture."""
    rng = np.random.default_rng(4242)
    setup = cornell(W=W, H=H, spp=spp, config="c3", max_depth=max_depth, seed=seed)
    scene = setup.scene
    Mask = AlphaTester(AlphaMode.Mask, 0.5)
    rgb_alpha = ImageTexture(_noise_img(rng, 24, 24, 3, 0, 255, smooth=3), colorScale=(1.25, 1, 1))
    one_alpha = ImageTexture(_noise_img(rng, 16, 16, 1, 0, 255, smooth=2))
    rgba = ImageTexture(_noise_img(rng, 16, 16, 4, 0, 255, smooth=2), gammaCorrection=True)
    mats = []
    m = MicrofacetDiffuse(SolidColor((0.2, 0.5, 0.8)), None, None, None, rgb_alpha)
    m.setAlphaTester(Mask)
    mats.append(m)
    m = MicrofacetDiffuse(SolidColor((0.8, 0.3, 0.2)), None, None, None, one_alpha)
    m.setAlphaTester(AlphaTester(AlphaMode.Mask, 0.4))
    mats.append(m)
    m = MicrofacetDiffuse(SolidColor((0.9, 0.9, 0.1)), None, None, None, SolidColor((0.3, 0.3, 0.3)))
    m.setAlphaTester(Mask)
    mats.append(m)
    m = MicrofacetDiffuse(rgba)
    m.setAlphaTester(AlphaTester(AlphaMode.Mask, 0.55))
    mats.append(m)
    m = MicrofacetDielectric(1.5, SolidColor((1, 1, 1)), None, SolidColor((0.3, 0.3, 0.3)), one_alpha)
    m.setAlphaTester(Mask)
    mats.append(m)
    meshes = []
    for k, mat in enumerate(mats):
        x0 = -0.9 + 0.36 * k
        z = 0.9 - 0.25 * (k % 2)
        idx, v, n, uv = _quad_tris((x0, -0.8, z), (x0 + 0.34, -0.8, z), (x0 + 0.34, 0.3, z + 0.1),
                                   (x0, 0.3, z + 0.1))
        meshes.append(Mesh(idx, v, None, n, uv * 1.7, mat))
    scene.Add(Model(meshes))
    return SceneSetup(scene, setup.camera, setup.integrator, UniformLightSampler(), max_depth, seed, spp).finish()


# --------------------------------------------------------------------------
def _grid_mesh(nx: int, nz: int, size: float, y_fn, rng, tangents: bool, uv_scale: float = 1.0):
    xs = np.linspace(-size, size, nx + 1, dtype=np.float32)
    zs = np.linspace(-size, size, nz + 1, dtype=np.float32)
    X, Z = np.meshgrid(xs, zs)
    Y = y_fn(X, Z).astype(np.float32)
    v = np.stack([X, Y, Z], -1).reshape(-1, 3).astype(np.float32)
    # normals from finite differences
    dydx = np.gradient(Y, axis=1) / (xs[1] - xs[0])
    dydz = np.gradient(Y, axis=0) / (zs[1] - zs[0])
    n = np.stack([-dydx, np.ones_like(Y), -dydz], -1).reshape(-1, 3)
    n = (n / np.linalg.norm(n, axis=1, keepdims=True)).astype(np.float32)
    uu, vv = np.meshgrid(np.linspace(0, uv_scale, nx + 1), np.linspace(0, uv_scale, nz + 1))
    uv = np.stack([uu, vv], -1).reshape(-1, 2).astype(np.float32)
    i = np.arange((nx + 1) * (nz + 1)).reshape(nz + 1, nx + 1)
    a, b, c, d = i[:-1, :-1], i[:-1, 1:], i[1:, 1:], i[1:, :-1]
    idx = np.stack([a, d, c, a, c, b], -1).reshape(-1).astype(np.uint32)
    t = None
    if tangents:
        t = np.stack([np.ones_like(Y), dydx, np.zeros_like(Y)], -1).reshape(-1, 3)
        t = (t / np.linalg.norm(t, axis=1, keepdims=True)).astype(np.float32)
    return idx, v, t, n, uv


def heightfield(n: int = 100, W: int = 128, H: int = 128, spp: int = 8, max_depth: int = 8,
                seed: int = 0x5EED0005, integrator: str = "path") -> SceneSetup:
    """N x N heightfield mesh (2 N^2 triangles) + quad light, PowerLightSampler
    (the SURVEY.md §6 'procedural heightfield' probe)."""
    rng = np.random.default_rng(1234)
    scene = Scene()
    f = lambda X, Z: 0.15 * np.sin(3.1 * X) * np.cos(2.7 * Z) + 0.05 * np.sin(11 * X + 7 * Z)
    idx, v, t, nr, uv = _grid_mesh(n, n, 2.0, f, rng, False)
    mat = MicrofacetDiffuse(SolidColor((0.6, 0.55, 0.5)), None, SolidColor((0.6, 0.6, 0.6)), SolidColor((0, 0, 0)))
    scene.Add(Model([Mesh(idx, v, None, nr, uv, mat)]))
    light = AreaLight(QuadShape((-0.5, 1.5, -0.5), (1, 0, 0), (0, 0, 1)), (20, 20, 20), False)
    scene.Add(GeometricPrimitive(light.getShape(), MicrofacetDiffuse((0, 0, 0)), light))
    scene.infiniteLights.append(UniformInfiniteLight((0.1, 0.12, 0.15)))
    film = Film((W, H), MitchellFilter())
    camera = Camera((0, 1.6, 3.2), (0, 0, 0), 1.0, film)
    return SceneSetup(scene, camera, integrator, PowerLightSampler(), max_depth, seed, spp).finish()


# --------------------------------------------------------------------------
def _noise_img(rng, h, w, c, lo=0, hi=255, smooth=4):
    base = rng.integers(lo, hi + 1, size=(h // smooth + 2, w // smooth + 2, c)).astype(np.float32)
    ys = np.linspace(0, base.shape[0] - 1.001, h)
    xs = np.linspace(0, base.shape[1] - 1.001, w)
    y0, x0 = ys.astype(int), xs.astype(int)
    fy, fx = (ys - y0)[:, None, None], (xs - x0)[None, :, None]
    a = base[y0][:, x0]
    b = base[y0][:, x0 + 1]
    cc = base[y0 + 1][:, x0]
    d = base[y0 + 1][:, x0 + 1]
    out = (1 - fy) * ((1 - fx) * a + fx * b) + fy * ((1 - fx) * cc + fx * d)
    return np.clip(out + 0.5, 0, 255).astype(np.uint8)


def material_zoo(W: int = 48, H: int = 48, spp: int = 4, max_depth: int = 8, seed: int = 0x5EED0007,
                 integrator: str = "path") -> SceneSetup:
    """Parity scene: every material kind, image textures (albedo with sRGB
    linearisation, tangent-space normal map, roughness/metallic maps, RGBA
    alpha in Mask mode), checker, one-sided quad light, sphere light, emissive
    triangles, sky gradient + distant + point lights, PowerLightSampler."""
    rng = np.random.default_rng(77)
    scene = Scene()
    albedo_img = ImageTexture(_noise_img(rng, 32, 32, 3, 40, 230), gammaCorrection=True)
    normal_img = ImageTexture(np.concatenate([_noise_img(rng, 16, 16, 2, 90, 165), np.full((16, 16, 1), 230, np.uint8)],
                                             axis=2))
    rough_img = ImageTexture(_noise_img(rng, 16, 16, 3, 20, 250))
    metal_img = ImageTexture(_noise_img(rng, 16, 16, 3, 0, 255))
    rgba = _noise_img(rng, 16, 16, 4, 0, 255)
    leaf_img = ImageTexture(rgba, gammaCorrection=True)
    checker = CheckerTexture(SolidColor((0.8, 0.8, 0.8)), albedo_img, (0.25, 0.25))

    # ground: textured, normal mapped, tangents (exercises onb(si) + normal map)
    idx, v, t, nr, uv = _grid_mesh(8, 8, 3.0, lambda X, Z: 0.05 * np.sin(2 * X) * np.cos(3 * Z), rng, True, 2.0)
    ground_mat = MicrofacetDiffuse(checker, normal_img, rough_img, metal_img)
    ground = Mesh(idx, v, t, nr, uv, ground_mat)
    # alpha-masked foliage card (Mask mode is deterministic)
    leaf_mat = MicrofacetDiffuse(leaf_img)
    leaf_mat.setAlphaTester(AlphaTester(AlphaMode.Mask, 0.5))
    i2, v2, n2, uv2 = _quad_tris((-0.8, -0.2, 0.2), (0.2, -0.2, 0.2), (0.2, 0.8, -0.1), (-0.8, 0.8, -0.1))
    leaf = Mesh(i2, v2, None, n2, uv2, leaf_mat)
    # emissive triangle strip
    i3, v3, n3, uv3 = _quad_tris((1.2, 0.1, -1.0), (1.6, 0.1, -1.0), (1.6, 0.6, -1.2), (1.2, 0.6, -1.2))
    emis = Mesh(i3, v3, None, n3, uv3, MicrofacetDiffuse((0.1, 0.1, 0.1)), SolidColor((4.0, 3.0, 2.0)))
    # glossy metal box, thin glass pane
    bi, bv, bn, buv = _box((0.9, 0.05, 0.5), (0.5, 0.5, 0.5), 0.6)
    metal = MicrofacetDiffuse(SolidColor((0.9, 0.6, 0.3)), None, SolidColor((0.25, 0.25, 0.25)), SolidColor((1, 1, 1)))
    box = Mesh(bi, bv, None, bn, buv, metal)
    pi_, pv, pn, puv = _quad_tris((-1.6, -0.2, -0.6), (-1.0, -0.2, -0.9), (-1.0, 0.6, -0.9), (-1.6, 0.6, -0.6))
    pane = Mesh(pi_, pv, None, pn, puv, ThinDielectric(1.5, SolidColor((0.9, 1.0, 0.95))))
    scene.Add(Model([ground, leaf, emis, box, pane]))
    # spheres: rough glass, smooth glass, mirror; a sphere light
    scene.Add(GeometricPrimitive(SphereShape((-0.3, 0.25, -0.9), 0.35), MicrofacetDielectric(1.5, 0.2, (1, 1, 1))))
    scene.Add(GeometricPrimitive(SphereShape((0.4, 0.2, -1.6), 0.3), MicrofacetDielectric(1.33, (0.95, 1, 1))))
    scene.Add(GeometricPrimitive(SphereShape((-1.3, 0.3, 0.6), 0.3), SpecularConductor((0.9, 0.9, 0.95))))
    sl = AreaLight(SphereShape((0.0, 1.6, 0.8), 0.15), (6, 6, 5), False)
    scene.Add(GeometricPrimitive(sl.getShape(), MicrofacetDiffuse((0, 0, 0)), sl))
    ql = AreaLight(QuadShape((-0.5, 2.0, -0.5), (1.0, 0, 0), (0, 0, 1.0)), (5, 5, 5), True)
    scene.Add(GeometricPrimitive(ql.getShape(), MicrofacetDiffuse((0.5, 0.5, 0.5)), ql))
    scene.infiniteLights.append(FunctionInfiniteLight((1, 0.85, 0.55), (0.45, 0.65, 1), 0.5))
    film = Film((W, H), MitchellFilter())
    camera = Camera((0.2, 1.4, 3.4), (0, 0, -0.3), 1.1, film)
    extra = [DistantLight((-1, 6, 1), (2.5, 2.3, 2.1)), PointLight((1.5, 1.2, 1.0), (1.5, 1.5, 1.5))]
    return SceneSetup(scene, camera, integrator, PowerLightSampler(), max_depth, seed, spp, extra).finish()


# --------------------------------------------------------------------------
# C4: San-Miguel-class procedural courtyard
# --------------------------------------------------------------------------
def _grid_idx(rows: int, cols: int) -> np.ndarray:
    i = np.arange((rows + 1) * (cols + 1), dtype=np.uint32).reshape(rows + 1, cols + 1)
    a, b, c, d = i[:-1, :-1], i[:-1, 1:], i[1:, 1:], i[1:, :-1]
    return np.stack([a, d, c, a, c, b], -1).reshape(-1)


def _unit(v):
    return (v / np.linalg.norm(v, axis=-1, keepdims=True)).astype(np.float32)


def _patch(p0, eu, ev, ku: int, kv: int, uv_scale=(1.0, 1.0), disp=None):
    """ku x kv grid over p0 + s*eu + t*ev (s, t in [0,1]); flat normal
    cross(eu, ev), tangent eu; optional displacement along the normal."""
    p0, eu, ev = (np.asarray(x, np.float32) for x in (p0, eu, ev))
    S, T = np.meshgrid(np.linspace(0, 1, ku + 1, dtype=np.float32), np.linspace(0, 1, kv + 1, dtype=np.float32))
    n = _unit(np.cross(eu, ev))
    v = p0 + S[..., None] * eu + T[..., None] * ev
    if disp is not None:
        v = v + disp(S, T)[..., None] * n
    v = v.reshape(-1, 3).astype(np.float32)
    nr = np.repeat(n[None], v.shape[0], 0)
    tg = np.repeat(_unit(eu)[None], v.shape[0], 0)
    uv = np.stack([S * uv_scale[0], T * uv_scale[1]], -1).reshape(-1, 2).astype(np.float32)
    return _grid_idx(kv, ku), v, tg, nr, uv


def _merge_t(parts):
    """_merge for (idx, v, t, n, uv) parts."""
    idx, vs, ts, ns, uvs = [], [], [], [], []
    base = 0
    for i, v, t, n, uv in parts:
        idx.append(i + np.uint32(base))
        vs.append(v)
        ts.append(t)
        ns.append(n)
        uvs.append(uv)
        base += v.shape[0]
    cat = lambda x: np.ascontiguousarray(np.concatenate(x), dtype=np.float32)
    return np.concatenate(idx).astype(np.uint32), cat(vs), cat(ts), cat(ns), cat(uvs)


def _sbox(center, size, angle: float, k: int):
    """Box with every face subdivided k x k, rotated about y."""
    cx, cy, cz = center
    sx, sy, sz = (s / 2 for s in size)
    c, s_ = math.cos(angle), math.sin(angle)
    R = np.array([[c, 0, -s_], [0, 1, 0], [s_, 0, c]], np.float32)
    faces = [((-sx, sy, -sz), (2 * sx, 0, 0), (0, 0, 2 * sz)),    # top (+y)
             ((-sx, -sy, sz), (2 * sx, 0, 0), (0, 2 * sy, 0)),    # +z
             ((sx, -sy, -sz), (-2 * sx, 0, 0), (0, 2 * sy, 0)),   # -z
             ((sx, -sy, sz), (0, 0, -2 * sz), (0, 2 * sy, 0)),    # +x
             ((-sx, -sy, -sz), (0, 0, 2 * sz), (0, 2 * sy, 0)),   # -x
             ((-sx, -sy, sz), (2 * sx, 0, 0), (0, 0, -2 * sz))]   # bottom (-y)
    parts = []
    for p0, eu, ev in faces:
        p0 = R @ np.array(p0, np.float32) + np.array([cx, cy, cz], np.float32)
        parts.append(_patch(p0, R @ np.array(eu, np.float32), R @ np.array(ev, np.float32), k, k))
    return _merge_t(parts)


def _cylinder(cx, cz, y0, y1, r, nseg: int, nring: int, uv_scale=(1.0, 1.0), radius_fn=None):
    th = np.linspace(0, 2 * math.pi, nseg + 1, dtype=np.float32)
    ys = np.linspace(y0, y1, nring + 1, dtype=np.float32)
    T, Y = np.meshgrid(th, ys)
    R = r if radius_fn is None else radius_fn(T, (Y - y0) / (y1 - y0))
    ct, st = np.cos(T), np.sin(T)
    v = np.stack([cx + R * ct, Y, cz + R * st], -1).reshape(-1, 3).astype(np.float32)
    n = np.stack([ct, np.zeros_like(T), st], -1).reshape(-1, 3).astype(np.float32)
    t = np.stack([-st, np.zeros_like(T), ct], -1).reshape(-1, 3).astype(np.float32)
    uv = np.stack([T / (2 * math.pi) * uv_scale[0], (Y - y0) / (y1 - y0) * uv_scale[1]], -1)
    return _grid_idx(nring, nseg), v, t, n, uv.reshape(-1, 2).astype(np.float32)


def _uv_sphere(c, r, nlat: int, nlon: int, radius_fn=None):
    ph = np.linspace(0.02, math.pi - 0.02, nlat + 1, dtype=np.float32)
    th = np.linspace(0, 2 * math.pi, nlon + 1, dtype=np.float32)
    TH, PH = np.meshgrid(th, ph)
    d = np.stack([np.sin(PH) * np.cos(TH), np.cos(PH), np.sin(PH) * np.sin(TH)], -1)
    R = r if radius_fn is None else radius_fn(TH, PH)
    v = (np.asarray(c, np.float32) + (R[..., None] if np.ndim(R) else R) * d).reshape(-1, 3).astype(np.float32)
    n = d.reshape(-1, 3).astype(np.float32)
    t = _unit(np.stack([-np.sin(TH), np.zeros_like(TH), np.cos(TH)], -1).reshape(-1, 3) + 1e-7)
    uv = np.stack([TH / (2 * math.pi), PH / math.pi], -1).reshape(-1, 2).astype(np.float32)
    return _grid_idx(nlat, nlon), v, t, n, uv


def _leaf_cards(rng, center, radius: float, n: int, size: float):
    """n alpha-masked leaf quads scattered in a crown (2 triangles each)."""
    p = rng.normal(size=(n, 3)).astype(np.float32)
    p = p / np.linalg.norm(p, axis=1, keepdims=True) * (radius * rng.random((n, 1)) ** 0.33)
    p = p * np.array([1.0, 0.7, 1.0], np.float32) + np.asarray(center, np.float32)
    a = _unit(rng.normal(size=(n, 3)).astype(np.float32))
    b = np.cross(a, _unit(rng.normal(size=(n, 3)).astype(np.float32)))
    b = _unit(b + 1e-6)
    a, b = a * size, b * size * 0.6
    v = np.stack([p - a - b, p + a - b, p + a + b, p - a + b], 1).reshape(-1, 3).astype(np.float32)
    nr = np.repeat(_unit(np.cross(a, b)), 4, 0)
    uv = np.tile(np.array([[0, 0], [1, 0], [1, 1], [0, 1]], np.float32), (n, 1))
    base = (np.arange(n, dtype=np.uint32) * 4)[:, None]
    idx = (base + np.array([0, 1, 2, 0, 2, 3], np.uint32)).reshape(-1)
    return idx, v, None, nr, uv


def _leaf_image(rng, size: int) -> np.ndarray:
    rgb = _noise_img(rng, size, size, 3, 0, 255, smooth=max(2, size // 64))
    g = np.array([40, 110, 35], np.float32) + (rgb.astype(np.float32) - 128) * np.array([0.15, 0.35, 0.12])
    y, x = np.mgrid[0:size, 0:size].astype(np.float32) / size
    mask = ((x - 0.5) / 0.47) ** 2 + ((y - 0.5) / 0.3) ** 2 < 1.0
    a = np.where(mask, 255, 0).astype(np.uint8)
    return np.concatenate([np.clip(g, 0, 255).astype(np.uint8), a[..., None]], axis=2)


def _normal_image(rng, size: int, strength: int = 40) -> np.ndarray:
    xy = _noise_img(rng, size, size, 2, 128 - strength, 128 + strength, smooth=max(2, size // 128))
    return np.concatenate([xy, np.full((size, size, 1), 235, np.uint8)], axis=2)


def _tinted(rng, size: int, base, spread: float = 40, smooth: int = 8) -> np.ndarray:
    n = _noise_img(rng, size, size, 1, 0, 255, smooth=smooth).astype(np.float32) - 128
    out = np.asarray(base, np.float32)[None, None, :] + n * (spread / 128.0)
    return np.clip(out, 0, 255).astype(np.uint8)


def sanmiguel(W: int = 1920, H: int = 1080, spp: int = 1024, max_depth: int = 128, seed: int = 0x5EED0004,
              detail: float = 1.0, tex_size: int = 1024, integrator: str = "path") -> SceneSetup:
    """C4: San-Miguel-class procedural courtyard, generator
    seed 0x5EED0004.  At detail=1: ~10 M triangles in one Model (BLAS4 under a
    TLAS4 with the lamp globes), 58 u8 textures (tex_size², the ground
    2·tex_size²), ~20 % of the triangles alpha-masked foliage cards (Mask
    mode, deterministic), diffuse / textured / normal-mapped / metallic /
    mirror / rough and smooth glass / thin glass materials, ~3000 emissive
    lamp triangles, sky gradient x1.5 (main.cpp:292-295) + DistantLight
    ((-1,6,1), 25*(1,.93,.83)) (main.cpp:304), PowerLightSampler, Mitchell,
    camera (17.3,1.2,7.2) -> (0,0,0), fov 1.7 (main.cpp:308-315)."""
    rng = np.random.default_rng(seed)
    # `detail` scales tessellation and leaf-card counts (triangles ~ detail);
    # the instance layout (8 trees, 40 bushes, 30 table sets, 12 lamps, ...)
    # is the same at every detail
    d = float(detail)
    g = lambda n: max(2, int(round(n * math.sqrt(d))))   # per-axis tessellation
    cnt = lambda n: max(1, int(round(n * d)))            # element counts (leaf cards)
    ts = int(tex_size)
    Opaque = AlphaTester(AlphaMode.Opaque)

    def diffuse(tex, norm=None, rough=None, metal=None):
        m = MicrofacetDiffuse(tex, norm, rough, metal)
        m.setAlphaTester(Opaque)
        return m

    def img(a, srgb=True):
        return ImageTexture(a, gammaCorrection=srgb)

    # ---- textures (58) ----
    ground_alb = img(_tinted(rng, 2 * ts, (150, 135, 115), 60, smooth=4))
    ground_nrm = img(_normal_image(rng, 2 * ts, 50), False)
    ground_rgh = img(_noise_img(rng, ts, ts, 3, 150, 255), False)
    wall_alb = [img(_tinted(rng, ts, c, 35)) for c in ((205, 175, 140), (220, 200, 170), (190, 120, 90),
                                                        (200, 190, 160))]
    wall_nrm = [img(_normal_image(rng, ts, 30), False) for _ in range(4)]
    stone_alb, stone_nrm = img(_tinted(rng, ts, (185, 180, 170), 30)), img(_normal_image(rng, ts, 25), False)
    bark_alb = [img(_tinted(rng, ts, (90, 65, 45), 40, smooth=3)) for _ in range(2)]
    bark_nrm = [img(_normal_image(rng, ts, 60), False) for _ in range(2)]
    leaf_tex = [img(_leaf_image(rng, ts)) for _ in range(6)]
    bush_alb = [img(_tinted(rng, ts, c, 45, smooth=2)) for c in ((50, 110, 40), (70, 120, 45), (40, 90, 50),
                                                                 (90, 130, 50), (60, 100, 30), (110, 60, 90))]
    wood_alb = [img(_tinted(rng, ts, (120 + 12 * i, 80 + 6 * i, 50 + 4 * i), 30, smooth=2)) for i in range(8)]
    wood_rgh = img(_noise_img(rng, ts, ts, 3, 120, 230), False)
    frame_alb = [img(_tinted(rng, ts, c, 15)) for c in ((60, 60, 62), (150, 150, 155), (190, 160, 90),
                                                          (120, 70, 40))]
    frame_rgh = img(_noise_img(rng, ts, ts, 3, 40, 120), False)
    fabric_alb = [img(_tinted(rng, ts, c, 25, smooth=1)) for c in ((160, 40, 40), (40, 60, 140), (200, 180, 90),
                                                                     (60, 120, 90), (180, 180, 180),
                                                                     (120, 60, 140))]
    fabric_nrm = img(_normal_image(rng, ts, 20), False)
    tile_alb = [img(_tinted(rng, ts, c, 30)) for c in ((170, 90, 60), (200, 200, 190), (60, 90, 140),
                                                        (150, 150, 140))]
    pot_alb = [img(_tinted(rng, ts, c, 25)) for c in ((180, 95, 60), (160, 85, 55), (140, 120, 100),
                                                       (90, 110, 130))]

    # ---- materials ----
    ground_m = diffuse(ground_alb, ground_nrm, ground_rgh)
    wall_m = [diffuse(a, n) for a, n in zip(wall_alb, wall_nrm)]
    stone_m = diffuse(stone_alb, stone_nrm)
    bark_m = [diffuse(a, n) for a, n in zip(bark_alb, bark_nrm)]
    leaf_m = []
    for t in leaf_tex:
        m = MicrofacetDiffuse(t)
        m.setAlphaTester(AlphaTester(AlphaMode.Mask, 0.5))
        leaf_m.append(m)
    bush_m = [diffuse(a) for a in bush_alb]
    wood_m = [diffuse(a, None, wood_rgh) for a in wood_alb]
    frame_m = [diffuse(a, None, frame_rgh, SolidColor((1, 1, 1))) for a in frame_alb]
    fabric_m = [diffuse(a, fabric_nrm) for a in fabric_alb]
    tile_m = [diffuse(a) for a in tile_alb]
    pot_m = [diffuse(a) for a in pot_alb]
    mirror = SpecularConductor((0.9, 0.9, 0.88))
    # dielectric roughness >= 0.15: below that the GGX lobe is so narrow that
    # evaluating it is ill-conditioned in fp32 (1-ulp changes of the half
    # vector move D by >10 %), so no two implementations agree sample-wise;
    # the water is smooth (the specular branch, Material.hpp:402-435)
    glass_rough = MicrofacetDielectric(1.5, 0.2, (1, 1, 1))
    water = MicrofacetDielectric(1.33, (0.85, 0.95, 1.0))
    pane = ThinDielectric(1.5, SolidColor((0.92, 0.96, 0.95)))
    bulb_m = diffuse(SolidColor((0.9, 0.9, 0.9)))

    meshes: List[Mesh] = []

    def add(part, mat, emission=None):
        i, v, t, n, uv = part
        meshes.append(Mesh(i, v, t, n, uv, mat, emission))

    X0, X1, Z0, Z1, WALL_H = -20.0, 25.0, -15.0, 15.0, 9.0
    # ground: cobblestone heightfield
    gx, gz = g(1600), g(1100)

    def cobble(S, T):
        u, v = S * (X1 - X0), T * (Z1 - Z0)
        return 0.015 * (np.sin(u * 9.0) * np.sin(v * 9.0)) ** 2 + 0.004 * np.sin(u * 31 + v * 17)
    add(_patch((X0, 0.0, Z1), (X1 - X0, 0, 0), (0, 0, Z0 - Z1), gx, gz, ((X1 - X0) / 4, (Z1 - Z0) / 4), cobble),
        ground_m)
    # tiled path across the courtyard (slightly raised)
    add(_patch((-18.0, 0.03, 1.2), (40.0, 0, 0), (0, 0, -2.4), g(300), g(20), (20, 1.2)), tile_m[0])
    # buildings: four stone walls with a displaced ashlar pattern
    walls = [((X0, 0, Z0), (0, 0, Z1 - Z0), (0, WALL_H, 0)),   # back wall (faces +x)
             ((X0, 0, Z1), (X1 - X0, 0, 0), (0, WALL_H, 0)),   # +z wall
             ((X1, 0, Z0), (X0 - X1, 0, 0), (0, WALL_H, 0)),   # -z wall
             ((X1, 0, Z1), (0, 0, Z0 - Z1), (0, WALL_H, 0))]   # behind the camera

    def ashlar(S, T):
        return -0.03 * ((np.sin(S * 120) > 0.95) | (np.sin(T * 36) > 0.95)) + 0.006 * np.sin(S * 410) * np.sin(T * 97)
    for k, (p0, eu, ev) in enumerate(walls):
        add(_patch(p0, eu, ev, g(400), g(100), (12, 3), ashlar), wall_m[k])
    # windows: thin glass panes set into the walls, one-sided mirrors as shutters
    for k in range(40):
        w = k % 4
        p0, eu, ev = (np.asarray(x, np.float32) for x in walls[w])
        s, t = 0.08 + 0.84 * ((k // 4) % 10) / 9.0, 0.45 + 0.3 * ((k // 40) % 2)
        n = _unit(np.cross(eu, ev))
        q0 = p0 + s * eu + t * ev + 0.02 * n
        add(_patch(q0, _unit(eu) * 1.1, _unit(ev) * 1.6, 1, 1), pane)
    # arcade: columns with a capital and an entablature beam
    cols = [(-17.0, z) for z in np.linspace(-12, 12, 9)] + [(x, -12.5) for x in np.linspace(-14, 22, 13)]
    for k, (cx, cz) in enumerate(cols[:22]):
        fl = lambda T, V: 0.28 * (1 + 0.04 * np.cos(16 * T)) * (1 - 0.12 * V)   # fluted, tapering shaft
        add(_cylinder(cx, cz, 0.0, 4.0, 0.28, g(64), g(200), (2, 4), fl), stone_m)
        add(_sbox((cx, 4.1, cz), (0.8, 0.2, 0.8), 0.0, g(10)), stone_m)
    add(_sbox((-17.0, 4.45, 0.0), (0.9, 0.5, 25.0), 0.0, g(40)), stone_m)
    add(_sbox((4.0, 4.45, -12.5), (37.0, 0.5, 0.9), 0.0, g(40)), stone_m)
    # trees: bark trunk + crown of alpha-masked leaf cards
    trees = [(-10.0, -7.0), (-4.0, 9.0), (6.0, -8.0), (12.0, 10.0), (-13.0, 4.0), (2.0, 3.0), (15.0, -4.0),
             (-6.0, -2.0)]
    for k, (cx, cz) in enumerate(trees):
        h = 3.5 + 1.5 * rng.random()
        tr = lambda T, V: 0.3 * (1.0 - 0.5 * V) * (1 + 0.08 * np.sin(5 * T + 13 * V))
        add(_cylinder(cx, cz, 0.0, h, 0.3, g(48), g(96), (2, 3), tr), bark_m[k % 2])
        add(_leaf_cards(rng, (cx, h + 1.2, cz), 2.4, cnt(120_000), 0.16), leaf_m[k % 6])
    # bushes in pots along the walls
    for k in range(40):
        side = k % 3
        if side == 0:
            cx, cz = -18.6, -13.0 + 26.0 * (k / 40.0)
        elif side == 1:
            cx, cz = -16.0 + 38.0 * (k / 40.0), 13.6
        else:
            cx, cz = -16.0 + 38.0 * (k / 40.0), -13.8
        r = 0.45 + 0.25 * rng.random()
        ph = rng.random(3) * 6.0
        bl = lambda TH, PH, r=r, ph=ph: r * (1 + 0.12 * np.sin(7 * TH + ph[0]) * np.sin(5 * PH + ph[1])
                                             + 0.05 * np.sin(23 * TH + 17 * PH + ph[2]))
        add(_uv_sphere((cx, 0.55 + r, cz), r, g(100), g(200), bl), bush_m[k % 6])
        pot = lambda T, V: 0.42 + 0.12 * V
        add(_cylinder(cx, cz, 0.0, 0.6, 0.45, g(64), g(32), (3, 1), pot), pot_m[k % 4])
    # tables with four chairs: wooden tops, metallic frames, fabric seats
    placed = 0
    for k in range(200):
        if placed >= 30:
            break
        cx, cz = rng.uniform(-14, 20), rng.uniform(-10, 11)
        if (cx - 17.3) ** 2 + (cz - 7.2) ** 2 < 9 or min((cx - tx) ** 2 + (cz - tz) ** 2 for tx, tz in trees) < 6:
            continue
        placed += 1
        a = rng.uniform(0, math.pi)
        kk = g(12)
        wm, fm, cm = wood_m[placed % 8], frame_m[placed % 4], fabric_m[placed % 6]
        parts = [_sbox((cx, 0.74, cz), (1.1, 0.05, 1.1), a, kk)]
        for sx, sz in ((-0.45, -0.45), (0.45, -0.45), (0.45, 0.45), (-0.45, 0.45)):
            lx, lz = cx + sx * math.cos(a) - sz * math.sin(a), cz + sx * math.sin(a) + sz * math.cos(a)
            parts.append(_sbox((lx, 0.36, lz), (0.06, 0.72, 0.06), a, kk))
        add(_merge_t(parts[:1]), wm)
        add(_merge_t(parts[1:]), fm)
        for j in range(4):
            ca = a + j * math.pi / 2
            ox, oz = cx + 0.95 * math.cos(ca), cz + 0.95 * math.sin(ca)
            add(_sbox((ox, 0.45, oz), (0.45, 0.06, 0.45), ca, kk), cm)
            bx, bz = ox + 0.22 * math.cos(ca), oz + 0.22 * math.sin(ca)
            add(_sbox((bx, 0.75, bz), (0.04, 0.55, 0.45), ca, kk), cm)
            legs = []
            for sx, sz in ((-0.2, -0.2), (0.2, -0.2), (0.2, 0.2), (-0.2, 0.2)):
                lx = ox + sx * math.cos(ca) - sz * math.sin(ca)
                lz = oz + sx * math.sin(ca) + sz * math.cos(ca)
                legs.append(_sbox((lx, 0.21, lz), (0.035, 0.42, 0.035), ca, kk))
            add(_merge_t(legs), fm)
        # a glass on the table
        add(_cylinder(cx + 0.2, cz + 0.1, 0.77, 0.9, 0.035, g(32), g(8)), glass_rough)
    # fountain: stone basin, rough water surface, mirror spout
    add(_cylinder(3.0, -1.0, 0.0, 0.55, 1.8, g(256), g(32), (8, 1)), stone_m)
    add(_cylinder(3.0, -1.0, 0.0, 0.55, 1.65, g(256), g(32), (8, 1)), stone_m)
    add(_patch((1.4, 0.45, 0.6), (3.2, 0, 0), (0, 0, -3.2), g(64), g(64), (1, 1),
               lambda S, T: 0.01 * np.sin(S * 40) * np.sin(T * 37)), water)
    add(_cylinder(3.0, -1.0, 0.45, 1.6, 0.12, g(64), g(64)), mirror)
    # lamp posts: mirror-metal posts, emissive bulbs (triangle area lights)
    lamps = [(-15.0, -10.0), (-15.0, 10.0), (0.0, -11.0), (0.0, 11.5), (10.0, -11.0), (10.0, 11.5), (20.0, -11.0),
             (20.0, 11.5), (-8.0, 4.0), (8.0, 4.0), (-8.0, -4.5), (14.0, 0.0)]
    bulb_light = SolidColor((40.0, 34.0, 24.0))
    for k, (cx, cz) in enumerate(lamps):
        add(_cylinder(cx, cz, 0.0, 3.0, 0.06, g(32), g(64)), mirror)
        add(_uv_sphere((cx, 3.25, cz), 0.1, 8, 16), bulb_m, bulb_light)

    scene = Scene()
    scene.Add(Model(meshes))
    # glass lamp globes around the bulbs (analytic spheres, TLAS primitives)
    for cx, cz in lamps:
        scene.Add(GeometricPrimitive(SphereShape((cx, 3.25, cz), 0.25), MicrofacetDielectric(1.5, (1, 1, 1))))
    scene.infiniteLights.append(FunctionInfiniteLight((1, 0.85, 0.55), (0.45, 0.65, 1), 1.5))
    film = Film((W, H), MitchellFilter())
    camera = Camera((17.3, 1.2, 7.2), (0, 0, 0), 1.7, film)
    sun = DistantLight((-1, 6, 1), np.float32(25.0) * np.array([1, 0.93, 0.83], np.float32))
    return SceneSetup(scene, camera, integrator, PowerLightSampler(), max_depth, seed, spp, [sun]).finish()


CONFIGS = {
    "c1": lambda **kw: example_1(**kw),
    "c2": lambda **kw: cornell(config="c2", **kw),
    "c3": lambda **kw: cornell(config="c3", **kw),
    "c4": lambda **kw: sanmiguel(**kw),
}


# --------------------------------------------------------------------------
def _smooth_sphere(nu: int, nv: int, tangents: bool = True):
    """A smooth-shaded sphere mesh (unit radius) with uvs and tangents."""
    th = np.linspace(0, np.pi, nv + 1)
    ph = np.linspace(0, 2 * np.pi, nu + 1)
    T, P = np.meshgrid(th, ph, indexing="ij")
    n = np.stack([np.sin(T) * np.cos(P), np.cos(T), np.sin(T) * np.sin(P)], -1).reshape(-1, 3)
    v = (n * np.array([1.0, 0.8, 1.0])).astype(np.float32)  # squashed: the normal matrix matters
    uv = np.stack([P / (2 * np.pi), T / np.pi], -1).reshape(-1, 2).astype(np.float32)
    i = np.arange((nv + 1) * (nu + 1)).reshape(nv + 1, nu + 1)
    a, b, c, d = i[:-1, :-1], i[:-1, 1:], i[1:, 1:], i[1:, :-1]
    idx = np.stack([a, b, c, a, c, d], -1).reshape(-1).astype(np.uint32)
    nrm = (n / np.linalg.norm(n, axis=1, keepdims=True)).astype(np.float32)
    t = None
    if tangents:
        t = np.stack([-np.sin(P), np.zeros_like(P), np.cos(P)], -1).reshape(-1, 3).astype(np.float32)
    return idx, v, t, nrm, uv


def instances(W: int = 1024, H: int = 1024, spp: int = 256, max_depth: int = 8,
              seed: int = 0x5EED0006) -> SceneSetup:
    """Instancing (§8f): the C2 room (a top-level Model) with one glossy model
    (a squashed smooth sphere mesh with tangents and a normal-mapped checker)
    instanced three times under rotate / scale / translate
    (TransformedPrimitive), a glass sphere and a metal quad as instanced
    GeometricPrimitives, and an AnimatedPrimitive sphere (main.cpp:186-190);
    PathIntegrator, PowerLightSampler."""
    from .scene import (AnimatedPrimitive, TransformedPrimitive, mat4_identity, mat4_rotate, mat4_scale,
                        mat4_translate)
    scene = Scene()
    white = MicrofacetDiffuse((0.73, 0.73, 0.73))
    red = MicrofacetDiffuse((0.65, 0.05, 0.05))
    green = MicrofacetDiffuse((0.12, 0.45, 0.15))
    walls = [
        (_quad_tris((-1, -1, 1), (1, -1, 1), (1, -1, -1), (-1, -1, -1)), white),
        (_quad_tris((-1, 1, -1), (1, 1, -1), (1, 1, 1), (-1, 1, 1)), white),
        (_quad_tris((-1, -1, -1), (1, -1, -1), (1, 1, -1), (-1, 1, -1)), white),
        (_quad_tris((-1, -1, 1), (-1, -1, -1), (-1, 1, -1), (-1, 1, 1)), red),
        (_quad_tris((1, -1, -1), (1, -1, 1), (1, 1, 1), (1, 1, -1)), green),
    ]
    scene.Add(Model([Mesh(i, v, None, n, uv, m) for (i, v, n, uv), m in walls]))
    light = AreaLight(QuadShape((-0.25, 0.999, -0.25), (0.5, 0, 0), (0, 0, 0.5)), (17.0, 12.0, 4.0), False)
    scene.Add(GeometricPrimitive(light.getShape(), MicrofacetDiffuse((0.78, 0.78, 0.78)), light))
    idx, v, t, n, uv = _smooth_sphere(24, 12)
    glossy = MicrofacetDiffuse(CheckerTexture(SolidColor((0.9, 0.6, 0.2)), SolidColor((0.2, 0.3, 0.8)), (0.125, 0.25)),
                               None, SolidColor((0.35, 0.35, 0.35)), SolidColor((0.0, 0.0, 0.0)))
    rock = Model([Mesh(idx, v, t, n, uv, glossy)])
    placements = [((-0.5, -0.72, -0.3), 0.6, (0, 1, 0), (0.28, 0.28, 0.28)),
                  ((0.45, -0.6, 0.2), -0.9, (1, 1, 0), (0.25, 0.4, 0.25)),
                  ((0.0, 0.1, -0.5), 1.7, (0, 0, 1), (0.35, 0.2, 0.2))]
    for pos, ang, ax, sc in placements:
        m = mat4_scale(mat4_rotate(mat4_translate(mat4_identity(), pos), ang, ax), sc)
        scene.Add(TransformedPrimitive(rock, m))
    glass = GeometricPrimitive(SphereShape((0, 0, 0), 1.0), MicrofacetDielectric(1.5, 0.05, (1, 1, 1)))
    scene.Add(TransformedPrimitive(glass, mat4_scale(mat4_translate(mat4_identity(), (-0.45, -0.1, 0.45)),
                                                      (0.22, 0.22, 0.22))))
    plate = GeometricPrimitive(QuadShape((-0.5, 0, -0.5), (1, 0, 0), (0, 0, 1)), SpecularConductor((0.9, 0.85, 0.8)))
    scene.Add(TransformedPrimitive(plate, mat4_rotate(mat4_scale(mat4_translate(mat4_identity(), (0.55, 0.3, -0.6)),
                                                                  (0.5, 1, 0.5)), 1.1, (1, 0, 0.3))))
    ball = GeometricPrimitive(SphereShape((0.3, -0.85, 0.55), 0.15), MicrofacetDiffuse((0.1, 0.2, 0.5)))
    scene.Add(AnimatedPrimitive(ball, (0, 0.2, 0), (0.25, 1.0)))
    film = Film((W, H), MitchellFilter())
    camera = Camera((0, 0, 3.7), (0, 0, 0), 0.75, film)
    return SceneSetup(scene, camera, "path", PowerLightSampler(), max_depth, seed, spp).finish()


# --------------------------------------------------------------------------
def motion_blur(W: int = 32, H: int = 32, spp: int = 4, max_depth: int = 16,
                seed: int = 0x5EED0071) -> SceneSetup:
    """Motion blur, NoModel-lite (main.cpp:164-270): a shutter camera
    Camera(lookFrom, lookAt, fov, film, vec2(0, 1)) (Camera.hpp:16-19) inside
    a thin forward-scattering medium (camera and scene medium), the animated
    sphere of main.cpp:186-190 (AnimatedPrimitive, direction (0, 0.2, 0),
    time bounds (0, 1)), an emissive sphere under an AnimatedPrimitive (its
    AnimatedLight, Light.cpp:338-364), the quad light, the rough glass and
    metallic spheres, a medium-only sphere and the checker floor and dome;
    VolPathIntegrator with the PowerLightSampler.  Every ray carries the time
    its camera sample drew (Camera.hpp:25), through scatter (Material.hpp:264),
    shadow rays (Integrators.cpp:433, 447) and medium steps (314, 361)."""
    from .scene import AnimatedPrimitive
    outside = HomogeneusMedium((0.01, 0.9, 0.9), (1.0, 0.1, 0.1), HenyeyGreenstein(0.75), 0.1)
    scene = Scene(outside)
    white = SolidColor((0.9, 0.9, 0.9))
    green = SolidColor((0.2, 0.3, 0.1))
    area = AreaLight(QuadShape((0.3, 2.5, 0), (-0.15, 0, 0), (0, 0, -0.15)), (1000.0, 1000.0, 1000.0), False)
    scene.Add(GeometricPrimitive(area.getShape(), MicrofacetDiffuse((0, 0, 0)), area, None))
    scene.Add(GeometricPrimitive(QuadShape((-100, -0.3, -100), (1000, 0, 0), (0, 0, 1000)),
                                 MicrofacetDiffuse(CheckerTexture(white, green, (0.001, 0.001))), None, None))
    ball = GeometricPrimitive(SphereShape((0, 0.1, -1.2), 0.5), MicrofacetDiffuse((0.1, 0.2, 0.5)), None)
    scene.Add(AnimatedPrimitive(ball, (0, 0.2, 0), (0, 1)))
    lamp = AreaLight(SphereShape((0.55, 0.45, -0.5), 0.12), (10.0, 6.0, 3.0), False)
    scene.Add(AnimatedPrimitive(GeometricPrimitive(lamp.getShape(), MicrofacetDiffuse((0.8, 0.8, 0.8)), lamp),
                                (-0.6, 0.1, 0.3), (0, 1)))
    scene.Add(GeometricPrimitive(SphereShape((-1, 0.3, -1), 0.5), MicrofacetDielectric(1.5, 0.15, (1, 1, 1)), None))
    met = MicrofacetDiffuse(SolidColor((0.8, 0.6, 0.2)), None, SolidColor((0, 0, 0)), SolidColor((1, 1, 1)))
    scene.Add(GeometricPrimitive(SphereShape((-1, 0, 0.2), 0.5), met, None))
    scene.Add(GeometricPrimitive(SphereShape((1, 0, -1), 0.5), None, None,
                                 HomogeneusMedium((0.01, 0.9, 0.9), (1.0, 0.1, 0.1), HenyeyGreenstein(0.8), 5.0)))
    scene.Add(GeometricPrimitive(SphereShape((0, 0, 0), 10),
                                 MicrofacetDiffuse(CheckerTexture(white, green, (0.02, 0.02))), None))
    camera = Camera((0.3, 0.4, 1), (0, 0, 0), 1.7, Film((W, H), MitchellFilter()), (0.0, 1.0))
    camera.SetMedium(outside)
    return SceneSetup(scene, camera, "volpath", PowerLightSampler(), max_depth, seed, spp).finish()


def motion_path(W: int = 32, H: int = 32, spp: int = 4, max_depth: int = 8, integrator: str = "path",
                seed: int = 0x5EED0072, shutter=(0.1, 0.9)) -> SceneSetup:
    """Motion blur on triangles and the pool of lights (PathIntegrator / SimplePathIntegrator):
    the C2 room, an AnimatedPrimitive Model (a box mesh whose BLAS the rays
    enter at their own translation), an emissive box Model under an
    AnimatedPrimitive (one AnimatedLight per emissive triangle), an animated
    metal sphere whose time bounds (0.25, 1) exercise the clamp of
    Primitive.cpp:83 (clamp(time - t0, t0, t1)), under a shutter (0.1, 0.9)
    camera."""
    from .scene import AnimatedPrimitive
    scene = Scene()
    white = MicrofacetDiffuse((0.73, 0.73, 0.73))
    red = MicrofacetDiffuse((0.65, 0.05, 0.05))
    green = MicrofacetDiffuse((0.12, 0.45, 0.15))
    walls = [
        (_quad_tris((-1, -1, 1), (1, -1, 1), (1, -1, -1), (-1, -1, -1)), white),
        (_quad_tris((-1, 1, -1), (1, 1, -1), (1, 1, 1), (-1, 1, 1)), white),
        (_quad_tris((-1, -1, -1), (1, -1, -1), (1, 1, -1), (-1, 1, -1)), white),
        (_quad_tris((-1, -1, 1), (-1, -1, -1), (-1, 1, -1), (-1, 1, 1)), red),
        (_quad_tris((1, -1, -1), (1, -1, 1), (1, 1, 1), (1, 1, -1)), green),
    ]
    scene.Add(Model([Mesh(i, v, None, n, uv, m) for (i, v, n, uv), m in walls]))
    light = AreaLight(QuadShape((-0.25, 0.999, -0.25), (0.5, 0, 0), (0, 0, 0.5)), (12.0, 10.0, 8.0), False)
    scene.Add(GeometricPrimitive(light.getShape(), MicrofacetDiffuse((0.78, 0.78, 0.78)), light))
    bi, bv, bn, buv = _box((-0.35, -0.55, -0.2), (0.4, 0.9, 0.4), 0.3)
    crate = Model([Mesh(bi, bv, None, bn, buv, MicrofacetDiffuse(SolidColor((0.9, 0.5, 0.2)), None,
                                                                 SolidColor((0.4, 0.4, 0.4)), SolidColor((0, 0, 0))))])
    scene.Add(AnimatedPrimitive(crate, (0.5, 0.0, 0.15), (0, 1)))
    li, lv, ln, luv = _box((0.4, 0.3, -0.3), (0.12, 0.12, 0.12), -0.4)
    lamp = Model([Mesh(li, lv, None, ln, luv, MicrofacetDiffuse((0.8, 0.8, 0.8)), SolidColor((4.0, 3.0, 1.5)))])
    scene.Add(AnimatedPrimitive(lamp, (-0.3, -0.5, 0.2), (0, 1)))
    ball = GeometricPrimitive(SphereShape((0.35, -0.8, 0.4), 0.2), SpecularConductor((0.9, 0.85, 0.8)))
    scene.Add(AnimatedPrimitive(ball, (0, 0.35, -0.2), (0.25, 1.0)))
    camera = Camera((0, 0, 3.7), (0, 0, 0), 0.75, Film((W, H), MitchellFilter()), shutterBounds=shutter)
    ls = None if integrator == "simple" else PowerLightSampler()
    return SceneSetup(scene, camera, integrator, ls, max_depth, seed, spp).finish()


def nested_instances(W: int = 32, H: int = 32, spp: int = 4, max_depth: int = 8, integrator: str = "path",
                     seed: int = 0x5EED0091, shutter=(0.0, 1.0)) -> SceneSetup:
    """Nested wrappers (TransformedPrimitive of a TransformedPrimitive,
    Primitive.cpp:32-96; their lights TransformedLight of a TransformedLight,
    Light.cpp:300-364): a crate Model under two and under three static
    levels (rotate / non-uniform scale / translate), an emissive lamp Model
    under a TransformedPrimitive of an AnimatedPrimitive (a moving emitter
    inside a static frame), an emissive sphere under an AnimatedPrimitive of
    a TransformedPrimitive, and a glass quad under four levels, in the C2 room
    with its ceiling light; shutter camera, PowerLightSampler."""
    from .scene import (AnimatedPrimitive, TransformedPrimitive, mat4_identity, mat4_rotate, mat4_scale,
                        mat4_translate)
    I = mat4_identity()
    scene = Scene()
    white = MicrofacetDiffuse((0.73, 0.73, 0.73))
    red = MicrofacetDiffuse((0.65, 0.05, 0.05))
    green = MicrofacetDiffuse((0.12, 0.45, 0.15))
    walls = [
        (_quad_tris((-1, -1, 1), (1, -1, 1), (1, -1, -1), (-1, -1, -1)), white),
        (_quad_tris((-1, 1, -1), (1, 1, -1), (1, 1, 1), (-1, 1, 1)), white),
        (_quad_tris((-1, -1, -1), (1, -1, -1), (1, 1, -1), (-1, 1, -1)), white),
        (_quad_tris((-1, -1, 1), (-1, -1, -1), (-1, 1, -1), (-1, 1, 1)), red),
        (_quad_tris((1, -1, -1), (1, -1, 1), (1, 1, 1), (1, 1, -1)), green),
    ]
    scene.Add(Model([Mesh(i, v, None, n, uv, m) for (i, v, n, uv), m in walls]))
    light = AreaLight(QuadShape((-0.25, 0.999, -0.25), (0.5, 0, 0), (0, 0, 0.5)), (8.0, 7.0, 6.0), False)
    scene.Add(GeometricPrimitive(light.getShape(), MicrofacetDiffuse((0.78, 0.78, 0.78)), light))
    bi, bv, bn, buv = _box((0, 0, 0), (0.3, 0.3, 0.3), 0.0)
    crate = Model([Mesh(bi, bv, None, bn, buv, MicrofacetDiffuse(SolidColor((0.9, 0.5, 0.2)), None,
                                                                 SolidColor((0.4, 0.4, 0.4)), SolidColor((0, 0, 0))))])
    inner = TransformedPrimitive(crate, mat4_scale(mat4_rotate(I, 0.6, (0, 1, 0)), (1.4, 0.7, 1.1)))
    scene.Add(TransformedPrimitive(inner, mat4_translate(I, (-0.45, -0.75, -0.25))))
    mid = TransformedPrimitive(TransformedPrimitive(crate, mat4_rotate(I, -0.4, (1, 0, 0))),
                               mat4_scale(I, (0.8, 1.3, 0.8)))
    scene.Add(TransformedPrimitive(mid, mat4_rotate(mat4_translate(I, (0.45, -0.6, 0.2)), 0.3, (0, 0, 1))))
    li, lv, ln, luv = _box((0, 0, 0), (0.1, 0.1, 0.1), -0.4)
    lamp = Model([Mesh(li, lv, None, ln, luv, MicrofacetDiffuse((0.8, 0.8, 0.8)), SolidColor((4.0, 3.0, 1.5)))])
    scene.Add(TransformedPrimitive(AnimatedPrimitive(lamp, (0.0, -0.3, 0.2), (0, 1)),
                                   mat4_scale(mat4_translate(I, (0.3, 0.4, -0.3)), (1.5, 1.0, 1.2))))
    sl = AreaLight(SphereShape((0, 0, 0), 0.08), (5.0, 1.5, 1.0), False)
    ball = GeometricPrimitive(sl.getShape(), MicrofacetDiffuse((0.9, 0.9, 0.9)), sl)
    scene.Add(AnimatedPrimitive(TransformedPrimitive(ball, mat4_scale(mat4_translate(I, (-0.5, 0.3, 0.3)),
                                                                       (1.2, 0.9, 1.0))),
                                (0.25, -0.1, 0.0), (0.25, 1.0)))
    pane = GeometricPrimitive(QuadShape((-0.5, 0, -0.5), (1, 0, 0), (0, 0, 1)), MicrofacetDielectric(1.5, 0.1, (1, 1, 1)))
    chain = pane
    for m in (mat4_scale(I, (0.5, 1, 0.4)), mat4_rotate(I, 1.2, (1, 0, 0)), mat4_rotate(I, 0.5, (0, 1, 0)),
              mat4_translate(I, (0.1, -0.1, 0.5))):
        chain = TransformedPrimitive(chain, m)
    scene.Add(chain)
    camera = Camera((0, 0, 3.7), (0, 0, 0), 0.75, Film((W, H), MitchellFilter()), shutterBounds=shutter)
    ls = None if integrator == "simple" else PowerLightSampler()
    return SceneSetup(scene, camera, integrator, ls, max_depth, seed, spp).finish()


# --------------------------------------------------------------------------
def ref_models(W: int = 32, H: int = 32, spp: int = 4, max_depth: int = 8, seed: int = 0x5EED0091) -> SceneSetup:
    """What every main.cpp scene holds: ResourceManager::CacheModel<BLAS4>
    results in the TLAS (main.cpp:290) -- the C2 room as one Model, an
    emissive lamp Model (its BuildBlas makes one AreaLight per triangle,
    Model.hpp:43-60) and a sphere mesh Model built with a material override,
    BuildBlas<BLAS4>(glass, nullptr) (Model.hpp:62-80, the extra CacheModel
    arguments of main.cpp:376), beside a quad light; PathIntegrator,
    PowerLightSampler.  The reference harness builds these as the reference's
    own Model objects (scene.ref_models, oracle/ref_model.cpp), so the
    drop-in's Model unwrap (integration/HipIntegrator.cpp, PT_WITH_MODEL)
    runs on them."""
    scene = Scene()
    scene.ref_models = True
    white = MicrofacetDiffuse((0.73, 0.73, 0.73))
    red = MicrofacetDiffuse((0.65, 0.05, 0.05))
    green = MicrofacetDiffuse((0.12, 0.45, 0.15))
    walls = [
        (_quad_tris((-1, -1, 1), (1, -1, 1), (1, -1, -1), (-1, -1, -1)), white),
        (_quad_tris((-1, 1, -1), (1, 1, -1), (1, 1, 1), (-1, 1, 1)), white),
        (_quad_tris((-1, -1, -1), (1, -1, -1), (1, 1, -1), (-1, 1, -1)), white),
        (_quad_tris((-1, -1, 1), (-1, -1, -1), (-1, 1, -1), (-1, 1, 1)), red),
        (_quad_tris((1, -1, -1), (1, -1, 1), (1, 1, 1), (1, 1, -1)), green),
    ]
    scene.Add(Model([Mesh(i, v, None, n, uv, m) for (i, v, n, uv), m in walls]))
    light = AreaLight(QuadShape((-0.25, 0.999, -0.25), (0.5, 0, 0), (0, 0, 0.5)), (9.0, 7.0, 4.0), False)
    scene.Add(GeometricPrimitive(light.getShape(), MicrofacetDiffuse((0.78, 0.78, 0.78)), light))
    bi, bv, bn, buv = _box((0.45, -0.85, -0.35), (0.3, 0.3, 0.3), 0.4)
    scene.Add(Model([Mesh(bi, bv, None, bn, buv, MicrofacetDiffuse((0.8, 0.8, 0.8)), SolidColor((2.5, 1.8, 1.0)))]))
    idx, v, t, n, uv = _smooth_sphere(20, 10)
    v = v * np.float32(0.3) + np.asarray((-0.3, -0.55, 0.2), np.float32)
    scene.Add(Model([Mesh(idx, v, t, n, uv, white)], material=MicrofacetDielectric(1.5, 0.1, (1, 1, 1))))
    camera = Camera((0, 0, 3.7), (0, 0, 0), 0.75, Film((W, H), MitchellFilter()))
    return SceneSetup(scene, camera, "path", PowerLightSampler(), max_depth, seed, spp).finish()


def ref_transformed_models(W: int = 32, H: int = 32, spp: int = 4, max_depth: int = 16,
                           seed: int = 0x5EED0092) -> SceneSetup:
    """TransformedPrimitive of a Model, as main.cpp:376 / 483 place their
    models: a glass "dragon" (a sphere mesh) built by
    CacheModel<BLAS4>(name, path, glass, HomogeneusMedium) -- the
    BuildBlas(material, medium) form -- placed twice under rotate / scale /
    translate (the cache returns the same Model), a plain Model under one
    transform and an emissive lamp Model under another (its lights become
    TransformedLights, Primitive.cpp:66-73), in the C2 room (itself a Model);
    VolPathIntegrator (the dragon's medium), UniformLightSampler.  The harness
    holds the reference's own Model objects (scene.ref_models)."""
    from .scene import TransformedPrimitive, mat4_identity, mat4_rotate, mat4_scale, mat4_translate
    scene = Scene()
    scene.ref_models = True
    white = MicrofacetDiffuse((0.73, 0.73, 0.73))
    red = MicrofacetDiffuse((0.65, 0.05, 0.05))
    green = MicrofacetDiffuse((0.12, 0.45, 0.15))
    walls = [
        (_quad_tris((-1, -1, 1), (1, -1, 1), (1, -1, -1), (-1, -1, -1)), white),
        (_quad_tris((-1, 1, -1), (1, 1, -1), (1, 1, 1), (-1, 1, 1)), white),
        (_quad_tris((-1, -1, -1), (1, -1, -1), (1, 1, -1), (-1, 1, -1)), white),
        (_quad_tris((-1, -1, 1), (-1, -1, -1), (-1, 1, -1), (-1, 1, 1)), red),
        (_quad_tris((1, -1, -1), (1, -1, 1), (1, 1, 1), (1, 1, -1)), green),
    ]
    scene.Add(Model([Mesh(i, v, None, n, uv, m) for (i, v, n, uv), m in walls]))
    light = AreaLight(QuadShape((-0.25, 0.999, -0.25), (0.5, 0, 0), (0, 0, 0.5)), (12.0, 9.0, 5.0), False)
    scene.Add(GeometricPrimitive(light.getShape(), MicrofacetDiffuse((0.78, 0.78, 0.78)), light))
    idx, v, t, n, uv = _smooth_sphere(20, 10)
    fill = HomogeneusMedium((0.01, 0.9, 0.9), (1.0, 0.1, 0.1), HenyeyGreenstein(0.8), 5.0)
    dragon = Model([Mesh(idx, v, t, n, uv, white)], material=MicrofacetDielectric(1.5, 0.05, (1, 1, 1)),
                   medium=fill)
    for pos, ang, ax, sc in [((-0.45, -0.6, 0.1), 0.5, (0, 1, 0), (0.3, 0.35, 0.3)),
                             ((0.35, -0.1, -0.4), -0.8, (1, 0, 1), (0.25, 0.2, 0.3))]:
        scene.Add(TransformedPrimitive(dragon, mat4_scale(mat4_rotate(mat4_translate(mat4_identity(), pos), ang, ax),
                                                          sc)))
    rock = Model([Mesh(idx, v, t, n, uv, MicrofacetDiffuse((0.3, 0.5, 0.8)))])
    scene.Add(TransformedPrimitive(rock, mat4_scale(mat4_translate(mat4_identity(), (0.5, -0.8, 0.5)),
                                                    (0.18, 0.18, 0.18))))
    bi, bv, bn, buv = _box((0, 0, 0), (0.2, 0.12, 0.2), 0.0)
    lamp = Model([Mesh(bi, bv, None, bn, buv, MicrofacetDiffuse((0.8, 0.8, 0.8)), SolidColor((3.0, 2.0, 1.2)))])
    scene.Add(TransformedPrimitive(lamp, mat4_rotate(mat4_translate(mat4_identity(), (-0.55, 0.55, -0.5)), 0.7,
                                                     (1, 1, 0))))
    camera = Camera((0, 0, 3.7), (0, 0, 0), 0.75, Film((W, H), MitchellFilter()))
    return SceneSetup(scene, camera, "volpath", UniformLightSampler(), max_depth, seed, spp).finish()
