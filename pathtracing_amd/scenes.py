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
                    FunctionInfiniteLight, GeometricPrimitive, HomogeneusMedium, ImageTexture, Mesh,
                    MicrofacetDielectric, MicrofacetDiffuse, MitchellFilter, Model, PointLight, PowerLightSampler,
                    QuadShape, Scene, SolidColor, SpecularConductor, SphereShape, ThinDielectric,
                    UniformInfiniteLight, UniformLightSampler)


@dataclass
class SceneSetup:
    scene: Scene
    camera: Camera
    integrator: str            # "path" | "simple"
    light_sampler: object
    max_depth: int
    seed: int
    spp: int
    extra_lights: list = field(default_factory=list)

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
        from .integrator import PathIntegrator, PCGSampler, SimplePathIntegrator
        sampler = PCGSampler(self.spp, self.seed)
        if self.integrator == "simple":
            return SimplePathIntegrator(self.scene, self.camera, sampler, self.max_depth)
        return PathIntegrator(self.scene, self.camera, sampler, self.light_sampler, self.max_depth)


# --------------------------------------------------------------------------
def example_1(W: int = 256, H: int = 256, spp: int = 16, integrator: str = "path", max_depth: int = 8,
              seed: int = 0x5EED0001, medium: bool = True) -> SceneSetup:
    """C1: examples/example_1.cpp:17-104 (UniformLightSampler, Mitchell 1.5)."""
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
    film = Film((W, H), MitchellFilter())
    camera = Camera((0.3, 0.4, 1), (0, 0, 0), 1.7, film)
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


def cornell(W: int = 1024, H: int = 1024, spp: int = 256, config: str = "c2", max_depth: int = 8,
            seed: Optional[int] = None) -> SceneSetup:
    """C2/C3 Cornell box: 5 walls + 2 boxes as one triangle Model (34 tris) and
    a quad area light under the ceiling.  C2: MicrofacetDiffuse(albedo)
    (roughness 1, metallic 0), SimplePathIntegrator.  C3: + rough glass sphere
    MicrofacetDielectric(1.5, 0.15), mirror SpecularConductor tall box,
    metallic MicrofacetDiffuse(metallic 1, rough 0.3) short box,
    PathIntegrator with UniformLightSampler.  maxDepth 8."""
    c3 = config == "c3"
    if seed is None:
        seed = 0x5EED0003 if c3 else 0x5EED0002
    scene = Scene()
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
    if c3:
        scene.Add(GeometricPrimitive(SphereShape((0.35, 0.05, 0.35), 0.3),
                                     MicrofacetDielectric(1.5, 0.15, (1, 1, 1))))
    film = Film((W, H), MitchellFilter())
    camera = Camera((0, 0, 3.7), (0, 0, 0), 0.75, film)
    return SceneSetup(scene, camera, "path" if c3 else "simple", UniformLightSampler() if c3 else None, max_depth,
                      seed, spp).finish()


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


CONFIGS = {
    "c1": lambda **kw: example_1(**kw),
    "c2": lambda **kw: cornell(config="c2", **kw),
    "c3": lambda **kw: cornell(config="c3", **kw),
}
