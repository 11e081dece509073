"""Host-side scene API mirroring the reference's classes (marko176/PathTracing).

Names, constructor arguments and defaults follow the reference so scene recipes
read like its main.cpp / examples/example_1.cpp:

  Textures   SolidColor, ImageTexture, CheckerTexture          (Texture.hpp:122-213)
  Materials  MicrofacetDiffuse, MicrofacetDielectric,
             ThinDielectric, SpecularConductor, AlphaTester     (Material.hpp:176-673)
  Shapes     QuadShape, SphereShape, Mesh (triangles)           (Shape.hpp, Mesh.hpp)
  Prims      GeometricPrimitive, Model (a BLAS4 over meshes)    (Primitive.hpp:17-31, Model.hpp)
  Lights     AreaLight, UniformInfiniteLight, FunctionInfiniteLight (sky gradient),
             DistantLight, PointLight                           (Light.hpp/.cpp)
  Samplers   UniformLightSampler, PowerLightSampler             (LightSampler.hpp)
  Scene      Add / BuildTlas / GetLights / BoundingBox / infiniteLights (Scene.hpp)
  Sensor     Film, MitchellFilter, BoxFilter, GaussianFilter, Camera  (Film.hpp, Filter.hpp, Camera.hpp)

Geometry is held as float32 numpy arrays; every derived quantity the reference
computes in a constructor (quad normal/D/w, camera basis, light power) is
computed in float32 in the same operand order.  Rendering goes through the
native HIP library (pathtracing_amd.integrator); nothing here touches a GPU.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence, Dict

import numpy as np

f32 = np.float32


def _v3(x) -> np.ndarray:
    a = np.asarray(x, dtype=np.float32).reshape(-1)
    if a.size == 1:
        a = np.repeat(a, 3)
    if a.size != 3:
        raise ValueError(f"expected a 3-vector, got {x!r}")
    return a.astype(np.float32)


def _fma32(a, b, c) -> np.float32:
    """fmaf(a, b, c): the exact a*b + c rounded once to float32."""
    from fractions import Fraction
    exact = Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c))
    r = np.float32(float(exact))
    best = r
    for cand in (np.nextafter(r, np.float32(-np.inf)), np.nextafter(r, np.float32(np.inf))):
        dc, db = abs(Fraction(float(cand)) - exact), abs(Fraction(float(best)) - exact)
        if dc < db or (dc == db and (int(cand.view(np.uint32)) & 1) == 0):
            best = cand
    return np.float32(best)


def _dot_c(a, b) -> np.float32:
    """glm::dot as the reference build contracts it: x product rounded, then
    fma(y), fma(z) (DESIGN.md "Numerics")."""
    a = np.asarray(a, dtype=np.float32)
    b = np.asarray(b, dtype=np.float32)
    return _fma32(a[2], b[2], _fma32(a[1], b[1], f32(a[0] * b[0])))


def _normalize_c(v) -> np.ndarray:
    v = np.asarray(v, dtype=np.float32)
    return (v * (f32(1.0) / f32(np.sqrt(_dot_c(v, v))))).astype(np.float32)


def _normalize(v: np.ndarray) -> np.ndarray:
    """glm::normalize = v * (1 / sqrt(dot(v, v))) (glm/detail/func_geometric.inl:88)."""
    v = v.astype(np.float32)
    d = _dot(v, v)
    return (v * (f32(1.0) / f32(np.sqrt(d)))).astype(np.float32)


def _cross(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    a = a.astype(np.float32)
    b = b.astype(np.float32)
    return np.array([a[1] * b[2] - b[1] * a[2],
                     a[2] * b[0] - b[2] * a[0],
                     a[0] * b[1] - b[0] * a[1]], dtype=np.float32)


def _cross_c(a, b) -> np.ndarray:
    """glm::cross as the reference build contracts it in Shape::Area: each
    lane's first product fused, the second rounded."""
    a = np.asarray(a, dtype=np.float32)
    b = np.asarray(b, dtype=np.float32)
    return np.array([_fma32(a[1], b[2], -f32(b[1] * a[2])), _fma32(a[2], b[0], -f32(b[2] * a[0])),
                     _fma32(a[0], b[1], -f32(b[0] * a[1]))], dtype=np.float32)


def _dot(a, b) -> np.float32:
    a = np.asarray(a, dtype=np.float32)
    b = np.asarray(b, dtype=np.float32)
    return f32(f32(a[0] * b[0]) + f32(a[1] * b[1])) + f32(a[2] * b[2])


def _expand_seq(points) -> np.ndarray:
    """AABB().Expand(p0).Expand(p1)... with glm::min/max's operand order
    (AABB.hpp:62-70): keeps the earlier value on ties, so signed zeros match."""
    pts = [np.asarray(p, dtype=np.float32) for p in points]
    mn = np.full(pts[0].shape, np.inf, np.float32)
    mx = np.full(pts[0].shape, -np.inf, np.float32)
    for p in pts:
        mn = np.where(p < mn, p, mn)
        mx = np.where(mx < p, p, mx)
    return np.concatenate([mn, mx], axis=-1).astype(np.float32)


def _fma64(a, b, c) -> float:
    """fma(a, b, c) in double: the exact a*b + c rounded once."""
    from fractions import Fraction
    return float(Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c)))


def luminance(c) -> float:
    """Util.hpp:3-5 (double), as the reference build contracts it: the x
    product rounded, then fma(y), fma(z) (AreaLight::PreProcess's GIMPLE)."""
    c = np.asarray(c, dtype=np.float64)
    return _fma64(c[2], 0.0722, _fma64(c[1], 0.7152, c[0] * 0.2126))


# --------------------------------------------------------------------------
# Textures (Texture.hpp:108-213)
# --------------------------------------------------------------------------
class Texture:
    def __init__(self, colorScale=(1, 1, 1)):
        self.colorScale = _v3(colorScale)

    def Channels(self) -> int:
        return 3


class SolidColor(Texture):
    def __init__(self, color, colorScale=(1, 1, 1)):
        super().__init__(colorScale)
        self.albedo = _v3(color)


class ImageTexture(Texture):
    """u8 image, bilinear, repeat wrap.  `data` is HxWxC uint8 already
    linearised if the reference would have loaded it with gammaCorrection
    (Texture.cpp:4-19 re-quantises through sRGBLUT)."""

    def __init__(self, data: np.ndarray, gammaCorrection: bool = False, colorScale=(1, 1, 1), path: str = ""):
        super().__init__(colorScale)
        data = np.ascontiguousarray(data, dtype=np.uint8)
        if data.ndim == 2:
            data = data[:, :, None]
        self.raw = data                      # as stored in a file (for recipes)
        self.gammaCorrection = bool(gammaCorrection)
        self.path = path
        self.data = srgb_linearize_u8(data) if gammaCorrection else data

    def Channels(self) -> int:
        return int(self.data.shape[2])


class FloatImageTexture(Texture):
    """FloatImageTexture (Texture.hpp:167-194): float texels (an HDR image as
    stbi_loadf returns it, HxWxC, row 0 first), bilinear, repeat wrap, no
    sRGB step.  `data` is the decoded float array; `path` names the file a
    recipe writes it to (tests: Radiance .hdr, whose decode is exact)."""

    def __init__(self, data: np.ndarray, colorScale=(1, 1, 1), path: str = ""):
        super().__init__(colorScale)
        data = np.ascontiguousarray(data, dtype=np.float32)
        if data.ndim == 2:
            data = data[:, :, None]
        self.data = data
        self.path = path

    def Channels(self) -> int:
        return int(self.data.shape[2])


class CheckerTexture(Texture):
    def __init__(self, textureA: Texture, textureB: Texture, uvscale, colorScale=(1, 1, 1)):
        super().__init__(colorScale)
        self.tex1 = textureA
        self.tex2 = textureB
        s = np.asarray(uvscale, dtype=np.float32).reshape(-1)
        if s.size == 1:
            s = np.repeat(s, 2)
        self.uvscale = s.astype(np.float32)
        self.invScale = (f32(1.0) / self.uvscale).astype(np.float32)

    def Channels(self) -> int:
        return self.tex1.Channels()


def _srgb_lut() -> np.ndarray:
    """sRGBLUT (Texture.hpp:26-34): lround(sRGB_to_linear(i/255) * 255), in double."""
    out = np.zeros(256, dtype=np.uint8)
    for i in range(256):
        s = i / 255.0
        lin = s / 12.92 if s <= 0.04045 else ((s + 0.055) / 1.055) ** 2.4
        lin = min(max(lin, 0.0), 1.0)
        out[i] = int(math.floor(lin * 255.0 + 0.5))
    return out


SRGB_LUT = _srgb_lut()


def srgb_linearize_u8(data: np.ndarray) -> np.ndarray:
    out = data.copy()
    c = min(out.shape[2], 3)
    out[:, :, :c] = SRGB_LUT[out[:, :, :c]]
    return out


# --------------------------------------------------------------------------
# Materials (Material.hpp:147-673)
# --------------------------------------------------------------------------
class AlphaMode:
    Opaque = 0
    Blend = 1
    Mask = 2


@dataclass
class AlphaTester:
    mode: int = AlphaMode.Blend   # default Blend (Material.hpp:196)
    cutoff: float = 0.5


class Material:
    kind = -1
    alpha_tester: Optional[AlphaTester] = None  # None = never set (default Blend)


class MicrofacetDiffuse(Material):
    kind = 0

    def __init__(self, tex, norm: Optional[Texture] = None, roughnessTexture: Optional[Texture] = None,
                 metallicTexture: Optional[Texture] = None, alpha_mask: Optional[Texture] = None):
        if not isinstance(tex, Texture):
            tex = SolidColor(tex)
        self.tex = tex
        self.norm = norm
        self.roughnessTexture = roughnessTexture if roughnessTexture is not None else SolidColor((1, 1, 1))
        self.metallicTexture = metallicTexture if metallicTexture is not None else SolidColor((0, 0, 0))
        self.alpha = alpha_mask
        self.alphaTester = AlphaTester()
        self.tester_set = False

    def setAlphaTester(self, tester: AlphaTester):
        """Material.hpp:350-353."""
        self.alphaTester = AlphaTester(tester.mode, tester.cutoff)
        self.tester_set = True
        if self.alpha is None and self.tex.Channels() != 4:
            self.alphaTester.mode = AlphaMode.Opaque


class MicrofacetDielectric(Material):
    kind = 1

    def __init__(self, refIndex: float, *args):
        """(ri, albedo) | (ri, roughness, albedo) | (ri, tex, norm, roughTex, alpha) (Material.hpp:366-368)."""
        self.ri = float(refIndex)
        self.norm = None
        self.alpha = None
        if len(args) == 1 and not isinstance(args[0], Texture):
            self.tex = SolidColor(args[0])
            self.roughnessTexture = SolidColor((0, 0, 0))
        elif len(args) == 2 and not isinstance(args[1], (Texture, type(None))) and np.isscalar(args[0]):
            self.tex = SolidColor(args[1])
            self.roughnessTexture = SolidColor((float(args[0]),) * 3)
        else:
            self.tex = args[0]
            self.norm = args[1] if len(args) > 1 else None
            rt = args[2] if len(args) > 2 else None
            self.roughnessTexture = rt if rt is not None else SolidColor((0, 0, 0))
            self.alpha = args[3] if len(args) > 3 else None
        self.alphaTester = AlphaTester()
        self.tester_set = False

    def setAlphaTester(self, tester: AlphaTester):
        self.alphaTester = AlphaTester(tester.mode, tester.cutoff)
        self.tester_set = True
        if self.alpha is None and self.tex.Channels() != 4:
            self.alphaTester.mode = AlphaMode.Opaque


class ThinDielectric(Material):
    kind = 2

    def __init__(self, eta: float, tex: Optional[Texture] = None):
        self.ri = float(eta)
        self.tex = tex if tex is not None else SolidColor((1, 1, 1))


class SpecularConductor(Material):
    kind = 3

    def __init__(self, albedo):
        self.albedo = _v3(albedo)


# --------------------------------------------------------------------------
# Shapes (Shape.hpp)
# --------------------------------------------------------------------------
class Shape:
    pass


class QuadShape(Shape):
    """Shape.hpp:118-171; ctor-derived normal, D, w in float32."""

    def __init__(self, origin, u, v):
        self.Q = _v3(origin)
        self.u = _v3(u)
        self.v = _v3(v)
        n = _cross(self.u, self.v)
        self.normal = _normalize(n)
        self.D = _dot(self.normal, self.Q)
        self.w = (n / _dot(n, n)).astype(np.float32)

    def bbox(self) -> np.ndarray:
        qu = (self.Q + self.u).astype(np.float32)
        quv = (qu + self.v).astype(np.float32)
        qv = (self.Q + self.v).astype(np.float32)
        return _expand_seq([self.Q, quv, qu, qv])  # QuadShape ctor (Shape.hpp:120-129)

    def Area(self) -> float:
        c = _cross_c(self.u, self.v)  # QuadShape::Area (Shape.hpp:143-145) as built
        return float(f32(np.sqrt(_dot_c(c, c))))


class SphereShape(Shape):
    def __init__(self, sphereCenter, sphereRadius: float):
        self.center = _v3(sphereCenter)
        self.radius = f32(sphereRadius)

    def bbox(self) -> np.ndarray:
        r = np.full(3, self.radius, dtype=np.float32)
        return _expand_seq([self.center - r, self.center + r])  # SphereShape ctor (Shape.hpp:22-26)

    def Area(self) -> float:
        return float(f32(f32(f32(4.0) * f32(math.pi)) * self.radius) * self.radius)


class Mesh:
    """Mesh.hpp:11-93: SoA triangle data + material / emissive texture / medium."""

    def __init__(self, indices, vertices, tangents, normals, texCoords, mat: Optional[Material],
                 emissiveTex: Optional[Texture] = None, meshMedium=None):
        self.indices = np.ascontiguousarray(indices, dtype=np.uint32).reshape(-1)
        self.vertices = np.ascontiguousarray(vertices, dtype=np.float32).reshape(-1, 3)
        self.normals = np.ascontiguousarray(normals, dtype=np.float32).reshape(-1, 3)
        self.texCoords = np.ascontiguousarray(texCoords, dtype=np.float32).reshape(-1, 2)
        t = None if tangents is None or len(tangents) == 0 else np.ascontiguousarray(tangents, dtype=np.float32).reshape(-1, 3)
        self.tangents = t
        self.material = mat
        self.emissiveTexture = emissiveTex
        self.medium = meshMedium
        if self.indices.size % 3:
            raise ValueError("indices must be a multiple of 3")
        nv = self.vertices.shape[0]
        if self.normals.shape[0] != nv or self.texCoords.shape[0] != nv or (t is not None and t.shape[0] != nv):
            raise ValueError("vertex attribute arrays must have equal length")
        if self.indices.size and int(self.indices.max()) >= nv:
            raise ValueError("index out of range")

    def GetTriangleCount(self) -> int:
        return self.indices.size // 3

    def tri_bboxes(self) -> np.ndarray:
        idx = self.indices.reshape(-1, 3)
        p = self.vertices[idx]                  # (n,3,3)
        # AABB(v0).Expand(v1).Expand(v2) (Shape.cpp:270-275)
        return _expand_seq([p[:, 0], p[:, 1], p[:, 2]])


# --------------------------------------------------------------------------
# Media (Medium.hpp, PhaseFunction.hpp): VolPathIntegrator's participating media
# --------------------------------------------------------------------------
class HenyeyGreenstein:
    """PhaseFunction.hpp:17-27: g clamped to [-0.99, 0.99] by the ctor."""

    def __init__(self, G: float):
        self.G = float(np.float32(G))
        self.g = float(np.clip(np.float32(G), np.float32(-0.99), np.float32(0.99)))


class HomogeneusMedium:
    """HomogeneusMedium (Medium.hpp:14-61).  The ctor's products are kept in
    float32 as glm computes them: sigma_a = d*sa, sigma_s = d*ss,
    sigma_t = d*(sa + ss), Le = Le*LeDensity.  `phaseFunction` is a
    HenyeyGreenstein or its g (the reference takes a shared_ptr<PhaseFunction>)."""

    def __init__(self, sigma_a, sigma_s, phaseFunction=0.0, density: float = 1.0, Le=(0.0, 0.0, 0.0),
                 LeDensity: float = 1.0):
        self.sigma_a_in = _v3(sigma_a)
        self.sigma_s_in = _v3(sigma_s)
        self.phaseFunction = (phaseFunction if isinstance(phaseFunction, HenyeyGreenstein)
                              else HenyeyGreenstein(float(phaseFunction)))
        self.density = float(np.float32(density))
        self.Le_in = _v3(Le)
        self.LeDensity = float(np.float32(LeDensity))
        d = np.float32(density)
        self.sigma_a = (d * self.sigma_a_in).astype(np.float32)
        self.sigma_s = (d * self.sigma_s_in).astype(np.float32)
        self.sigma_t = (d * (self.sigma_a_in + self.sigma_s_in).astype(np.float32)).astype(np.float32)
        self.emission = (self.Le_in * np.float32(LeDensity)).astype(np.float32)

    @property
    def g(self) -> float:
        return self.phaseFunction.g

    def Le(self) -> np.ndarray:
        return self.emission

    def IsEmmisive(self) -> bool:
        return bool(np.any(self.emission != 0))


# --------------------------------------------------------------------------
# Lights (Light.hpp / Light.cpp)
# --------------------------------------------------------------------------
class Light:
    def isDelta(self) -> bool:
        return False

    def PreProcess(self, bbox):
        pass

    def Power(self) -> float:
        return 0.0


def _scene_radius(bbox) -> float:
    """glm::distance(bbox.max, center) in float (Light.cpp:9-12)."""
    mn = np.asarray(bbox[:3], dtype=np.float32)
    mx = np.asarray(bbox[3:], dtype=np.float32)
    c = ((mx + mn) * f32(0.5)).astype(np.float32)
    d = (mx - c).astype(np.float32)
    return float(f32(np.sqrt(_dot(d, d))))


class AreaLight(Light):
    def __init__(self, light_shape: Shape, light_color, oneSided: bool = False):
        self.shape = light_shape
        self.emissiveTexture = light_color if isinstance(light_color, Texture) else SolidColor(light_color)
        self.oneSided = bool(oneSided)
        self.cachedPower = 0.0
        self.tri = None  # (mesh, local triangle) for mesh lights

    def getShape(self):
        return self.shape

    def PreProcess(self, bbox):
        """AreaLight::PreProcess (Light.cpp:277-287): (1|2) * Area *
        luminance(mean emission over 16 x 16 samples of the shape).  A solid
        emission is that colour exactly; a textured one is averaged at
        stratified points with a fixed jitter hash (the reference's sampler
        there is a fresh, never-started StratifiedSampler with unseeded
        jitter: its estimate is random, this one deterministic)."""
        tex = self.emissiveTexture
        if isinstance(tex, SolidColor):
            e = (tex.colorScale * tex.albedo).astype(np.float32)
        else:
            e = self._mean_emission(tex)
        area = self.shape_area()
        self.cachedPower = float(f32((1 if self.oneSided else 2) * area * luminance(e)))

    def _mean_emission(self, tex) -> np.ndarray:
        # the reference's fresh StratifiedSampler(16, 16): never started, so
        # call k draws stratum PermutationElement(0, 256, Hash(0u, 0u, 2k))
        # (Sampler.hpp:98-110, Util.hpp:44-175) -- a fixed set of strata,
        # with repeats -- plus unseeded jitter, here a fixed hash
        k = np.arange(256)
        strata = np.array([_permutation_element(0, 256, _ref_hash_u32x2_u64(0, 0, 2 * i) & 0xFFFFFFFF)
                           for i in range(256)])
        h = (k * 2654435761 + 0x5EED) & 0xFFFFFFFF
        jx = ((h * 747796405 + 2891336453) & 0xFFFFFF) / 16777216.0
        jy = ((h * 277803737 + 1442695041) & 0xFFFFFF) / 16777216.0
        u0 = ((strata % 16) + jx) / 16.0
        u1 = ((strata // 16) + jy) / 16.0
        u, v = self._sample_uv(u0.astype(np.float32), u1.astype(np.float32))
        return _tex_eval_np(tex, u, v).mean(0)

    def _sample_uv(self, u0, u1):
        """uv of Shape::Sample(u) (Shape.cpp:74-81, 277-297; Shape.hpp:139-141)."""
        if self.tri is not None:
            mesh, t = self.tri
            i0, i1, i2 = (int(x) for x in mesh.indices[3 * t:3 * t + 3])
            uv = mesh.texCoords
            w = 1.0 - u0 - u1  # not folded
            uu = u0 * uv[i1, 0] + u1 * uv[i2, 0] + w * uv[i0, 0]
            vv = u0 * uv[i1, 1] + u1 * uv[i2, 1] + w * uv[i0, 1]
            return uu, vv
        if isinstance(self.shape, SphereShape):
            z = 1.0 - 2.0 * u0
            r = np.sqrt(np.maximum(0.0, 1.0 - z * z))
            phi = 2.0 * np.pi * u1
            d = np.stack([r * np.cos(phi), r * np.sin(phi), z], 1)
            p = self.shape.center + self.shape.radius * d  # GetSphereUV of the point itself (Shape.cpp:80)
            d = p / np.linalg.norm(p, axis=1, keepdims=True)
            theta = np.arccos(np.clip(d[:, 1], -1, 1))
            ph = np.arctan2(d[:, 2], d[:, 0])
            ph = np.where(ph < 0, ph + 2 * np.pi, ph)
            return ph / (2 * np.pi), theta / np.pi
        return np.zeros_like(u0), np.zeros_like(u0)  # QuadShape::Sample leaves uv at 0

    def shape_area(self) -> float:
        if self.tri is not None:
            mesh, k = self.tri
            i0, i1, i2 = (int(x) for x in mesh.indices[3 * k:3 * k + 3])
            a = mesh.vertices[i0] - mesh.vertices[i2]
            b = mesh.vertices[i1] - mesh.vertices[i2]
            c = _cross_c(a, b)  # TriangleShape::Area (Shape.cpp:298-301) as built
            return float(f32(f32(np.sqrt(_dot_c(c, c))) * f32(0.5)))
        return self.shape.Area()

    def Power(self) -> float:
        return self.cachedPower


_M64 = 0xFFFFFFFFFFFFFFFF


def _ref_hash_u32x2_u64(a: int, b: int, c: int) -> int:
    """Hash(unsigned, unsigned, uint64_t) (Util.hpp:162-170): MurmurHash64A
    over the 16 packed bytes, seed 0."""
    m, r = 0xC6A4A7935BD1E995, 47
    h = (0 ^ (16 * m)) & _M64
    for k in (a | (b << 32), c):
        k = (k * m) & _M64
        k ^= k >> r
        k = (k * m) & _M64
        h ^= k
        h = (h * m) & _M64
    h ^= h >> r
    h = (h * m) & _M64
    h ^= h >> r
    return h


def _permutation_element(i: int, l: int, p: int) -> int:
    """PermutationElement (Util.hpp:44-72), uint32 arithmetic."""
    M = 0xFFFFFFFF
    w = l - 1
    for sh in (1, 2, 4, 8, 16):
        w |= w >> sh
    while True:
        i ^= p; i = (i * 0xE170893D) & M; i ^= p >> 16; i ^= (i & w) >> 4; i ^= p >> 8
        i = (i * 0x0929EB3F) & M; i ^= p >> 23; i ^= (i & w) >> 1; i = (i * (1 | p >> 27)) & M
        i = (i * 0x6935FA69) & M; i ^= (i & w) >> 11; i = (i * 0x74DCB303) & M; i ^= (i & w) >> 2
        i = (i * 0x9E501CC3) & M; i ^= (i & w) >> 2; i = (i * 0xC860A3DF) & M; i &= w; i ^= i >> 5
        if i < l:
            break
    return (i + p) % l


def _tex_eval_np(tex, u, v) -> np.ndarray:
    """Texture::Evaluate at arrays of uv (host estimate for PreProcess):
    SolidColor, CheckerTexture, ImageTexture (u8 / 255), FloatImageTexture,
    bilinear with repeat wrap (Texture.hpp:128-207)."""
    u = np.asarray(u, np.float64)
    v = np.asarray(v, np.float64)
    cs = np.asarray(tex.colorScale, np.float64)
    if isinstance(tex, SolidColor):
        return np.broadcast_to(cs * tex.albedo, (u.shape[0], 3)).astype(np.float64)
    if isinstance(tex, CheckerTexture):
        ux = np.floor(u * tex.invScale[0]).astype(np.int64)
        uy = np.floor(v * tex.invScale[1]).astype(np.int64)
        a, b = _tex_eval_np(tex.tex1, u, v), _tex_eval_np(tex.tex2, u, v)
        return cs * np.where(((ux + uy) % 2 == 0)[:, None], a, b)
    data = tex.data.astype(np.float64)
    if isinstance(tex, ImageTexture):
        data = data / 255.0
    h, w = data.shape[:2]
    x, y = u * w - 0.5, v * h - 0.5
    xi, yi = np.floor(x).astype(np.int64), np.floor(y).astype(np.int64)
    dx, dy = (x - xi)[:, None], (y - yi)[:, None]

    def tx(a, b):
        px = data[np.mod(b, h), np.mod(a, w)]
        return px[:, :3] if px.shape[1] >= 3 else np.repeat(px[:, :1], 3, 1)
    r = ((1 - dx) * (1 - dy) * tx(xi, yi) + dx * (1 - dy) * tx(xi + 1, yi) + (1 - dx) * dy * tx(xi, yi + 1) +
         dx * dy * tx(xi + 1, yi + 1))
    return cs * r


class InfiniteLight(Light):
    sceneRadius = 0.0

    def PreProcess(self, bbox):
        self.sceneRadius = _scene_radius(bbox)


class UniformInfiniteLight(InfiniteLight):
    def __init__(self, light_color):
        self.color = _v3(light_color)

    def Power(self) -> float:
        c = self.color
        return float(f32(f32(f32(c[0] + c[1]) + c[2]) * f32(math.sqrt(self.sceneRadius))))


class FunctionInfiniteLight(InfiniteLight):
    """The sky gradient of main.cpp:292-295, parameterised:
    Le(dir) = scale * ((1-a) * horizon + a * zenith), a = 0.5 * (dir.y + 1).
    Power(): the reference estimates it by stratified jittered sampling
    (Light.cpp:79-107, nondeterministic); we integrate the same luminance
    deterministically (the PMF only enters MIS weights and light selection)."""

    def __init__(self, horizon=(1, 0.85, 0.55), zenith=(0.45, 0.65, 1), scale: float = 1.5):
        self.c0 = _v3(horizon)
        self.c1 = _v3(zenith)
        self.scale = f32(scale)
        self.cachedPower = 0.0
        self.power_override: Optional[float] = None

    def Le(self, d) -> np.ndarray:
        a = f32(0.5) * (f32(d[1]) + f32(1.0))
        return (self.scale * ((f32(1.0) - a) * self.c0 + a * self.c1)).astype(np.float32)

    def PreProcess(self, bbox):
        super().PreProcess(bbox)
        if self.power_override is not None:
            self.cachedPower = float(self.power_override)
            return
        # uniform-sphere integral of luminance: dir.y = z? Le uses dir.y; under
        # the sampling of Light.cpp:88-99 y = r sin(theta) is symmetric, so
        # E[a] = 0.5 and the mean luminance is that of the mean colour.
        mean = (self.scale * (f32(0.5) * self.c0 + f32(0.5) * self.c1)).astype(np.float64)
        self.cachedPower = float(f32(luminance(mean) * math.sqrt(self.sceneRadius)))

    def Power(self) -> float:
        return self.cachedPower


class TextureInfiniteLight(InfiniteLight):
    """TextureInfiniteLight (Light.hpp:94-123, Light.cpp:110-200): an
    environment map, Le(dir) = LeScale * tex(GetSphereUV(dir)), sampled by a
    1920 x 1080 grid of cells weighted by their mean luminance.  PreProcess
    runs the native host restatement of the reference's cell estimate
    (pt_texinf_weights: its unseeded jitter becomes a fixed hash) and keeps
    the float running sums (std::partial_sum) for the device."""
    NX, NY = 1920, 1080

    def __init__(self, tex: "FloatImageTexture", LeScale: float = 1.0):
        if not isinstance(tex, FloatImageTexture):
            raise TypeError("TextureInfiniteLight takes a FloatImageTexture (main.cpp:115-116, 222-224)")
        self.tex = tex
        self.LeScale = f32(LeScale)
        self.cachedPower = 0.0
        self.accWeights: Optional[np.ndarray] = None
        self.weights_override: Optional[np.ndarray] = None

    def PreProcess(self, bbox):
        super().PreProcess(bbox)
        from . import native as N
        if self.weights_override is not None:
            w = np.ascontiguousarray(self.weights_override, np.float32)
        else:
            w = N.texinf_weights(self.tex.data, self.tex.colorScale, float(self.LeScale))
        # std::partial_sum in float (sequential), totalWeight = back()
        self.accWeights = np.cumsum(w, dtype=np.float32)
        total = float(self.accWeights[-1])
        # totalWeight / samples * sqrt(sceneRadius) (Light.cpp:195)
        self.cachedPower = float(f32(total / (self.NX * self.NY) * float(f32(math.sqrt(self.sceneRadius)))))

    def Power(self) -> float:
        return self.cachedPower


class DistantLight(Light):
    def __init__(self, light_dir, light_color):
        self.dir = _v3(light_dir)
        self.color = _v3(light_color)
        self.sceneRadius = 0.0

    def isDelta(self) -> bool:
        return True

    def PreProcess(self, bbox):
        self.sceneRadius = _scene_radius(bbox)

    def Power(self) -> float:
        c = self.color
        return float(f32(f32(f32(c[0] + c[1]) + c[2]) * f32(math.sqrt(self.sceneRadius))))


class PointLight(Light):
    def __init__(self, p, light_color):
        self.p = _v3(p)
        self.color = _v3(light_color)
        self.sceneRadius = 0.0

    def isDelta(self) -> bool:
        return True

    def PreProcess(self, bbox):
        self.sceneRadius = _scene_radius(bbox)

    def Power(self) -> float:
        c = self.color
        return float(f32(f32(f32(c[0] + c[1]) + c[2]) * f32(4.0 * self.sceneRadius)))


class TransformedLight(Light):
    """TransformedLight / AnimatedLight (Light.cpp:300-364): what
    TransformedPrimitive::GetLights / AnimatedPrimitive::GetLights
    (Primitive.cpp:66-73, 91-96) hand the light sampler for an emitter inside
    an instance.  The inner AreaLight keeps its object-space shape; sample()
    moves the point by the instance transform and the normal by its normal
    matrix, PDF() takes point, normal and ray back to object space, L() sees
    a fresh interaction (normal matrix applied, uv = (0, 0)).  Power() is the
    inner power times det(transform) (TransformedLight) or the inner power
    (AnimatedLight).  A path that hits the emitter sees the inner AreaLight
    itself (Primitive.cpp:58).  Nested wrappers wrap the inner wrapper's
    light: `light` is then a TransformedLight, `area` the AreaLight inside."""

    def __init__(self, light: Light, instance: "TransformedPrimitive"):
        self.light = light
        self.instance = instance
        self.animated = isinstance(instance, AnimatedPrimitive)

    @property
    def area(self) -> "AreaLight":
        l = self.light
        while isinstance(l, TransformedLight):
            l = l.light
        return l

    def isDelta(self) -> bool:
        return self.light.isDelta()

    def PreProcess(self, bbox):
        self.light.PreProcess(bbox)

    def Power(self) -> float:
        if self.animated:
            return self.light.Power()
        # glm::determinant(mat4) in float; evaluated in double and rounded
        # (a last-bit difference only moves the PMF by an ulp)
        return float(f32(f32(self.light.Power()) * f32(np.linalg.det(self.instance.transform.astype(np.float64)))))


# --------------------------------------------------------------------------
# Light samplers (LightSampler.cpp)
# --------------------------------------------------------------------------
class LightSampler:
    kind = 0

    def __init__(self):
        self.lights: List[Light] = []
        self.all_lights: List[Light] = []

    def Add(self, light):
        if isinstance(light, (list, tuple)):
            for l in light:
                self.Add(l)
            return
        self.lights.append(light)
        self.all_lights.append(light)

    def PreProcess(self, bbox):
        valid = []
        for l in self.lights:
            l.PreProcess(bbox)
            if l.Power() < 0.01:
                continue
            valid.append(l)
        self.lights = valid

    def PMF(self, light) -> float:
        raise NotImplementedError


class UniformLightSampler(LightSampler):
    kind = 0

    def PMF(self, light) -> float:
        if not self.lights:
            return 0.0
        return float(f32(1.0) / f32(len(self.lights)))


class PowerLightSampler(LightSampler):
    kind = 1

    def __init__(self):
        super().__init__()
        self.totalPower = 0.0

    def PreProcess(self, bbox):
        super().PreProcess(bbox)
        tot = f32(0.0)
        for l in self.lights:
            tot = f32(tot + f32(l.Power()))
        self.totalPower = float(tot)

    def PMF(self, light) -> float:
        if self.totalPower == 0:
            return 1.0
        return float(f32(light.Power()) / f32(self.totalPower))


# --------------------------------------------------------------------------
# Primitives
# --------------------------------------------------------------------------
class Primitive:
    pass


class GeometricPrimitive(Primitive):
    def __init__(self, primitive_shape: Shape, material: Optional[Material], areaLight: Optional[AreaLight] = None,
                 medium=None):
        self.shape = primitive_shape
        self.material = material
        self.areaLight = areaLight
        self.medium = medium


# glm::mat4 helpers.  Matrices are float32 arrays m[col][row] (glm's layout);
# the products are glm's, rounded per operation.
def mat4_identity() -> np.ndarray:
    return np.eye(4, dtype=np.float32)


def mat4_translate(m, v) -> np.ndarray:
    """glm::translate (glm/ext/matrix_transform.inl): m[3] = m0*v0 + m1*v1 + m2*v2 + m3."""
    m = np.asarray(m, np.float32)
    v = _v3(v)
    r = m.copy()
    r[3] = ((m[0] * v[0] + m[1] * v[1]).astype(np.float32) + (m[2] * v[2]).astype(np.float32)).astype(np.float32)
    r[3] = (r[3] + m[3]).astype(np.float32)
    return r


def mat4_scale(m, v) -> np.ndarray:
    m = np.asarray(m, np.float32)
    v = _v3(v)
    r = m.copy()
    for i in range(3):
        r[i] = (m[i] * v[i]).astype(np.float32)
    return r


def mat4_rotate(m, angle: float, axis) -> np.ndarray:
    """glm::rotate(m, angle, axis) (glm/ext/matrix_transform.inl)."""
    m = np.asarray(m, np.float32)
    a = np.float32(angle)
    c, s = np.float32(math.cos(a)), np.float32(math.sin(a))
    ax = _v3(axis)
    ax = (ax / np.float32(np.sqrt(np.float32(_dot(ax, ax))))).astype(np.float32)
    t = ((np.float32(1) - c) * ax).astype(np.float32)
    R = np.zeros((3, 3), np.float32)
    R[0, 0] = c + t[0] * ax[0]
    R[0, 1] = t[0] * ax[1] + s * ax[2]
    R[0, 2] = t[0] * ax[2] - s * ax[1]
    R[1, 0] = t[1] * ax[0] - s * ax[2]
    R[1, 1] = c + t[1] * ax[1]
    R[1, 2] = t[1] * ax[2] + s * ax[0]
    R[2, 0] = t[2] * ax[0] + s * ax[1]
    R[2, 1] = t[2] * ax[1] - s * ax[0]
    R[2, 2] = c + t[2] * ax[2]
    r = m.copy()
    for i in range(3):
        r[i] = ((m[0] * R[i, 0] + m[1] * R[i, 1]).astype(np.float32) + (m[2] * R[i, 2]).astype(np.float32))
    return r.astype(np.float32)


def mat4_inverse(m) -> np.ndarray:
    """glm::inverse(mat4) (glm/detail/func_matrix.inl compute_inverse<4,4>),
    float32 per operation."""
    m = np.asarray(m, np.float32)
    f = np.float32
    def d(a, b, c, e):
        return f(f(a * b) - f(c * e))
    C00 = d(m[2][2], m[3][3], m[3][2], m[2][3]); C02 = d(m[1][2], m[3][3], m[3][2], m[1][3])
    C03 = d(m[1][2], m[2][3], m[2][2], m[1][3]); C04 = d(m[2][1], m[3][3], m[3][1], m[2][3])
    C06 = d(m[1][1], m[3][3], m[3][1], m[1][3]); C07 = d(m[1][1], m[2][3], m[2][1], m[1][3])
    C08 = d(m[2][1], m[3][2], m[3][1], m[2][2]); C10 = d(m[1][1], m[3][2], m[3][1], m[1][2])
    C11 = d(m[1][1], m[2][2], m[2][1], m[1][2]); C12 = d(m[2][0], m[3][3], m[3][0], m[2][3])
    C14 = d(m[1][0], m[3][3], m[3][0], m[1][3]); C15 = d(m[1][0], m[2][3], m[2][0], m[1][3])
    C16 = d(m[2][0], m[3][2], m[3][0], m[2][2]); C18 = d(m[1][0], m[3][2], m[3][0], m[1][2])
    C19 = d(m[1][0], m[2][2], m[2][0], m[1][2]); C20 = d(m[2][0], m[3][1], m[3][0], m[2][1])
    C22 = d(m[1][0], m[3][1], m[3][0], m[1][1]); C23 = d(m[1][0], m[2][1], m[2][0], m[1][1])
    F = [np.array(x, np.float32) for x in ([C00, C00, C02, C03], [C04, C04, C06, C07], [C08, C08, C10, C11],
                                          [C12, C12, C14, C15], [C16, C16, C18, C19], [C20, C20, C22, C23])]
    V = [np.array([m[1][k], m[0][k], m[0][k], m[0][k]], np.float32) for k in range(4)]
    def comb(a, fa, b, fb, c, fc):
        return (((a * fa).astype(f) - (b * fb).astype(f)).astype(f) + (c * fc).astype(f)).astype(f)
    I0 = comb(V[1], F[0], V[2], F[1], V[3], F[2])
    I1 = comb(V[0], F[0], V[2], F[3], V[3], F[4])
    I2 = comb(V[0], F[1], V[1], F[3], V[3], F[5])
    I3 = comb(V[0], F[2], V[1], F[4], V[2], F[5])
    SA = np.array([1, -1, 1, -1], np.float32)
    SB = -SA
    inv = np.stack([I0 * SA, I1 * SB, I2 * SA, I3 * SB]).astype(np.float32)
    row0 = np.array([inv[0][0], inv[1][0], inv[2][0], inv[3][0]], np.float32)
    dot0 = (m[0] * row0).astype(np.float32)
    det = f(f(dot0[0] + dot0[1]) + f(dot0[2] + dot0[3]))
    return (inv * f(f(1) / det)).astype(np.float32)


MAX_INSTANCE_DEPTH = 4  # pt_api.h PT_MAX_INSTANCE_DEPTH


class TransformedPrimitive(Primitive):
    """TransformedPrimitive (Primitive.hpp:34-48, Primitive.cpp:32-72): an
    instance of a Model (BLAS), of a GeometricPrimitive, or of another
    TransformedPrimitive / AnimatedPrimitive (nested, up to
    MAX_INSTANCE_DEPTH levels) under an affine glm::mat4 (float32
    [col][row]).  Rays are taken to object space with the inverse, the hit
    back with the transform and its normal matrix, level by level."""

    def __init__(self, primitive: Primitive, transform):
        depth, base = 1, primitive
        while isinstance(base, TransformedPrimitive):
            depth, base = depth + 1, base.primitive
        if not isinstance(base, (Model, GeometricPrimitive)):
            raise TypeError("instances of a Model, a GeometricPrimitive or another instance only")
        if depth > MAX_INSTANCE_DEPTH:
            raise ValueError(f"{depth} nested instance levels (at most {MAX_INSTANCE_DEPTH})")
        self.primitive = primitive
        self.transform = np.ascontiguousarray(transform, np.float32).reshape(4, 4)
        # glm::inverse as the reference build contracts it: the native host
        # routine (pt_mat4_inverse, compiled like the reference); mat4_inverse
        # is its per-operation-rounded twin
        from . import native as N
        self.invTransform = N.mat4_inverse(self.transform)


class AnimatedPrimitive(TransformedPrimitive):
    """AnimatedPrimitive (Primitive.hpp:52-66, Primitive.cpp:76-96): a
    translation by direction * t, t = clamp(time - t0, t0, t1) / (t1 - t0),
    evaluated per ray at the ray's time (the device and the oracle rebuild
    the translation and its glm::inverse per ray).  `transform` holds the
    time-0 translation: what rays see under a camera without a shutter (time
    0)."""

    def __init__(self, primitive: Primitive, direction, timeBounds):
        self.direction = _v3(direction)
        self.timeBounds = np.asarray(timeBounds, np.float32).reshape(2)
        t0, t1 = self.timeBounds
        t = f32(f32(np.clip(f32(f32(0.0) - t0), t0, t1)) / f32(t1 - t0))
        super().__init__(primitive, mat4_translate(mat4_identity(), (self.direction * t).astype(np.float32)))


class Model(Primitive):
    """A BLAS4 over meshes: Model::BuildBlas<BLAS4> (Model.hpp:43-60) without Assimp.
    Emissive meshes get one AreaLight per triangle, culled if Power <= FLT_EPSILON.
    material / medium: BuildBlas<BLAS4>(material, medium) (Model.hpp:62-80,
    ResourceManager::CacheModel's extra arguments, main.cpp:376): every
    triangle takes both, a None one included."""

    def __init__(self, meshes: Sequence[Mesh], material: Optional[Material] = None, medium=None):
        self.meshes = list(meshes)
        self.override_material = material
        self.override_medium = medium
        # model-local triangle index -> AreaLight (emissive triangles only)
        self.tri_lights: Dict[int, AreaLight] = {}
        base = 0
        for m in self.meshes:
            if m.emissiveTexture is not None:
                for k in range(m.GetTriangleCount()):
                    area = AreaLight(None, m.emissiveTexture)
                    area.tri = (m, k)
                    area.PreProcess(None)
                    if area.Power() > float(np.finfo(np.float32).eps):
                        self.tri_lights[base + k] = area
            base += m.GetTriangleCount()

    def triangle_count(self) -> int:
        return sum(m.GetTriangleCount() for m in self.meshes)


class Scene:
    """Scene.hpp:5-37."""

    def __init__(self, medium: Optional[HomogeneusMedium] = None):
        self.primitives: List[Primitive] = []
        self.infiniteLights: List[InfiniteLight] = []
        self.sceneMedium = medium
        self.flat = None  # set by BuildTlas
        # test recipes only (pathtracing_amd.recipe): the reference harness
        # builds this scene's Models as the reference's own Model objects
        self.ref_models = False

    def GetMedium(self) -> Optional[HomogeneusMedium]:
        return self.sceneMedium

    def SetMedium(self, medium: Optional[HomogeneusMedium]):
        self.sceneMedium = medium
        self.flat = None

    def Add(self, prim: Primitive):
        self.primitives.append(prim)
        self.flat = None

    def BuildTlas(self):
        """Builds TLAS4 + per-Model BLAS4 with the native builder (reference
        algorithm) and lays out the flat scene (pathtracing_amd.flatten)."""
        from .flatten import flatten_scene
        self.flat = flatten_scene(self)
        return self.flat

    def GetLights(self) -> List[Light]:
        if self.flat is None:
            raise RuntimeError("call BuildTlas() first")
        return list(self.flat.tlas_lights) + list(self.infiniteLights)

    def BoundingBox(self) -> np.ndarray:
        if self.flat is None:
            raise RuntimeError("call BuildTlas() first")
        return self.flat.bbox.copy()


# --------------------------------------------------------------------------
# Film / filters / camera
# --------------------------------------------------------------------------
class Filter:
    kind = 0

    def __init__(self, radius=(1.5, 1.5)):
        r = np.asarray(radius, dtype=np.float32).reshape(-1)
        if r.size == 1:
            r = np.repeat(r, 2)
        self.radius = r


class MitchellFilter(Filter):
    kind = 0

    def __init__(self, radius=(1.5, 1.5), b: float = 1.0 / 3.0, c: float = 1.0 / 3.0):
        super().__init__(radius)
        self.b = float(b)
        self.c = float(c)

    def params(self):
        return (self.b, self.c)


class BoxFilter(Filter):
    kind = 1

    def __init__(self, radius=(0.5, 0.5)):
        super().__init__(radius)

    def params(self):
        return (0.0, 0.0)


class GaussianFilter(Filter):
    kind = 2

    def __init__(self, radius=(1.5, 1.5), sigma: float = 0.5):
        super().__init__(radius)
        self.sigma = float(np.float32(sigma))  # ctor takes double from a float literal 0.5f

    def params(self):
        return (self.sigma, 0.0)


class LanczosFilter(Filter):
    """LanczosFilter (Filter.hpp:114-144): WindowedSinc(x, r.x, tau) *
    WindowedSinc(y, r.y, tau), separable.  Integral() follows the reference's
    estimator (256 x 256 jittered strata over [-r, r], times its area term
    2 * r.x * r.y, Filter.hpp:130-143) with the unseeded random_double()
    jitter replaced by a fixed counter-based hash, so it is reproducible; the
    device takes the value from here (pt_render_desc.filter_params[1]), as
    the drop-in takes the reference object's own Integral()."""
    kind = 3

    def __init__(self, radius=(1.5, 1.5), tau: float = 3.0):
        super().__init__(radius)
        self.tau = float(tau)
        self._integral = None

    @staticmethod
    def _wsinc(x, radius, tau):
        x = np.asarray(x, np.float64)

        def sinc(v):
            with np.errstate(invalid="ignore", divide="ignore"):
                s = np.sin(np.pi * v) / (np.pi * v)
            return np.where(1.0 - v * v == 1.0, 1.0, s)
        return np.where(np.abs(x) > radius, 0.0, sinc(x) * sinc(x / tau))

    def Evaluate(self, p) -> np.ndarray:
        p = np.asarray(p, np.float32)
        return (self._wsinc(p[..., 0].astype(np.float64), float(self.radius[0]), self.tau) *
                self._wsinc(p[..., 1].astype(np.float64), float(self.radius[1]), self.tau))

    def Integral(self) -> float:
        if self._integral is None:
            n = 256
            ys, xs = np.meshgrid(np.arange(n, dtype=np.uint64), np.arange(n, dtype=np.uint64), indexing="ij")
            k = (ys * n + xs).astype(np.uint64)
            jx = (_hash_u32(k * np.uint64(2)) >> np.uint64(8)).astype(np.float64) / 16777216.0
            jy = (_hash_u32(k * np.uint64(2) + np.uint64(1)) >> np.uint64(8)).astype(np.float64) / 16777216.0
            u = np.stack([(xs + jx) / n, (ys + jy) / n], -1).astype(np.float32)
            r = self.radius.astype(np.float32)
            p = (-r + (r - -r) * u).astype(np.float32)  # glm::mix(-radius, radius, u)
            area = 2.0 * float(r[0]) * float(r[1])
            self._integral = area * float(self.Evaluate(p).sum()) / (n * n)
        return self._integral

    def params(self):
        return (self.tau, self.Integral())


def _hash_u32(v: np.ndarray) -> np.ndarray:
    """PCG-RXS-M-XS (the sample stream's hash) over uint64-held u32."""
    m = np.uint64(0xFFFFFFFF)
    v = np.asarray(v, np.uint64) & m
    s = (v * np.uint64(747796405) + np.uint64(2891336453)) & m
    w = (((s >> ((s >> np.uint64(28)) + np.uint64(4))) ^ s) * np.uint64(277803737)) & m
    return ((w >> np.uint64(22)) ^ w) & m


class Film:
    """Film.hpp:112-271: accumulation buffer of {sum RGB*w, sum w} in float64."""

    def __init__(self, resolution, filter: Optional[Filter] = None):
        self.xResolution = int(resolution[0])
        self.yResolution = int(resolution[1])
        self.filter = filter if filter is not None else MitchellFilter()
        self.accum = np.zeros((self.yResolution, self.xResolution, 4), dtype=np.float64)

    def Resolution(self):
        return (self.xResolution, self.yResolution)

    def Clear(self):
        self.accum[:] = 0

    def image(self) -> np.ndarray:
        w = self.accum[..., 3:4]
        with np.errstate(invalid="ignore", divide="ignore"):
            return np.where(w != 0, self.accum[..., :3] / w, 0.0)

    def Resolve(self, toneMapper: str = "reinhard_jodie", device: int = 0, accum=None) -> np.ndarray:
        """The writers' 8-bit image (Film.hpp:154-217): tone map + linear_to_sRGB
        + 255.999*clamp, on the GPU (pt_film_resolve).  Rows in film order
        (y = 0 first); `accum` (a host array or a cuda float64 tensor) defaults
        to this film's accumulator."""
        import ctypes as C
        from . import native as N
        from .integrator import get_context
        tm = {"reinhard_jodie": N.PT_TONEMAP_REINHARD_JODIE, "aces": N.PT_TONEMAP_ACES}[toneMapper]
        src = self.accum if accum is None else accum
        H, W = self.yResolution, self.xResolution
        out = np.zeros((H, W, 3), np.uint8)
        if hasattr(src, "data_ptr"):  # torch tensor (device film)
            ptr = src.data_ptr()
        else:
            src = np.ascontiguousarray(src, np.float64)
            ptr = src.ctypes.data
        ctx = get_context(device)
        N.check(N.lib().pt_film_resolve(ctx.ptr, C.c_void_p(ptr), W, H, tm, out.ctypes.data), ctx.ptr)
        return out

    def WritePPM(self, path: str, toneMapper: str = "reinhard_jodie"):
        """Film::WritePPM (Film.hpp:154-170): binary P6, bottom row first."""
        out = self.Resolve(toneMapper)[::-1]
        with open(path, "wb") as f:
            f.write(b"P6\n%d %d\n255\n" % (self.xResolution, self.yResolution))
            f.write(np.ascontiguousarray(out).tobytes())

    def WritePNG(self, path: str, toneMapper: str = "reinhard_jodie"):
        """Film::WritePNG (Film.hpp:172-196): 8-bit RGB, flipped vertically on
        write like stbi_flip_vertically_on_write(true).  Encoded with zlib
        (the pixels, not the encoder's byte stream, are the contract)."""
        import struct
        import zlib
        img = np.ascontiguousarray(self.Resolve(toneMapper)[::-1])
        raw = b"".join(b"\x00" + img[y].tobytes() for y in range(img.shape[0]))

        def chunk(t, d):
            return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)
        with open(path, "wb") as f:
            f.write(b"\x89PNG\r\n\x1a\n")
            f.write(chunk(b"IHDR", struct.pack(">IIBBBBB", self.xResolution, self.yResolution, 8, 2, 0, 0, 0)))
            f.write(chunk(b"IDAT", zlib.compress(raw, 6)))
            f.write(chunk(b"IEND", b""))


class Camera:
    """Camera.hpp:7-35.  The basis is built in float32 like the reference ctor."""

    def __init__(self, lookFrom, lookAt, fov: float, film: Film, FocusAngle=0.0, FocusDistance: float = 0.0,
                 medium: Optional[HomogeneusMedium] = None, shutterBounds=None):
        # Camera(lookFrom, lookAt, fov, film, glm::vec2 shutterBounds)
        # (Camera.hpp:16-19): a 2-sequence in FocusAngle's place, or the
        # keyword, is the shutter; that ctor has no lens (FocusAngle 0).
        # Rays carry time = mix(shutterStart, shutterEnd, u) (Camera.hpp:25);
        # without a shutter the reference's bounds are uninitialised (SURVEY
        # A.14) and rays carry time 0.
        if not np.isscalar(FocusAngle):
            if shutterBounds is not None or FocusDistance or medium is not None:
                raise TypeError("Camera(lookFrom, lookAt, fov, film, shutterBounds) takes no lens or medium")
            shutterBounds, FocusAngle = FocusAngle, 0.0
        self.shutter = None if shutterBounds is None else np.asarray(shutterBounds, np.float32).reshape(2)
        if self.shutter is not None and (FocusAngle or FocusDistance):
            raise TypeError("the reference's shutter camera has no thin lens (Camera.hpp:16-19)")
        self.cameraMedium = medium
        self.lookFrom = _v3(lookFrom)
        self.lookAt = _v3(lookAt)
        self.fov = f32(fov)
        self.film = film
        self.FocusAngle = f32(FocusAngle)
        self.FocusDistance = f32(FocusDistance)
        # the ctor's arithmetic as the reference build contracts it (fixture
        # search against Camera::GenerateRay): dot-pattern normalize, and
        # v.y = fma(w.z, u.x, -(u.z*w.x)); the other products are by 0 or 1
        w = _normalize_c((self.lookFrom - self.lookAt).astype(np.float32))
        u = _normalize_c(np.array([w[2], 0.0, -w[0]], dtype=np.float32))  # cross((0,1,0), w)
        v = np.array([f32(w[1] * u[2]), _fma32(w[2], u[0], -f32(u[2] * w[0])), -f32(u[0] * w[1])], np.float32)
        self.w, self.u, self.v = w, u, v
        self.defocusRadius = f32(float(self.FocusDistance) * math.tan(float(self.FocusAngle) / 2.0))
        self.halfWidth = f32(math.tan(float(self.fov) * 0.5))
        W, H = film.Resolution()
        self.halfHeight = f32(f32(self.halfWidth * f32(H)) / f32(W))

    def GetFilm(self) -> Film:
        return self.film

    def GetMedium(self) -> Optional[HomogeneusMedium]:
        return self.cameraMedium

    def SetMedium(self, medium: Optional[HomogeneusMedium]):
        self.cameraMedium = medium
