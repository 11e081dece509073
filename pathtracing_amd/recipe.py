"""Scene recipe writer: serialises a Scene (+ camera, sampler, integrator
settings) into the text format read by oracle/ref_harness.cpp, which rebuilds
the identical scene with the reference's own classes to produce golden
vectors.  Used only by tests/golden/gen_golden.py (test infrastructure).
"""
from __future__ import annotations

from pathlib import Path
from typing import Dict, List, Optional

import numpy as np

from .scene import (AnimatedPrimitive, AreaLight, CheckerTexture, DistantLight, FunctionInfiniteLight,
                    GeometricPrimitive, ImageTexture, TransformedPrimitive,
                    MicrofacetDielectric, MicrofacetDiffuse, Model, PointLight, PowerLightSampler, QuadShape,
                    SolidColor, SpecularConductor, SphereShape, ThinDielectric, UniformInfiniteLight,
                    FloatImageTexture, TextureInfiniteLight)


def _f(x) -> str:
    return repr(float(np.float32(x)))


def write_png(path: Path, data: np.ndarray):
    from PIL import Image  # available in this container; only the generator uses it
    data = np.asarray(data, dtype=np.uint8)
    if data.ndim == 3 and data.shape[2] == 1:
        data = data[:, :, 0]
    mode = {2: "L", 3: "RGB", 4: "RGBA"}[data.ndim if data.ndim == 2 else data.shape[2]] if data.ndim == 3 else "L"
    if data.ndim == 3 and data.shape[2] == 2:
        mode = "LA"
    Image.fromarray(data, mode=mode).save(path)


def write_hdr(path: Path, rgbe: np.ndarray):
    """Radiance RGBE, flat (not run-length) scanlines, rows top first: what
    stbi_loadf decodes back to FloatImageTexture.data exactly."""
    h, w = rgbe.shape[:2]
    with open(path, "wb") as f:
        f.write(b"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n" + f"-Y {h} +X {w}\n".encode())
        f.write(np.ascontiguousarray(rgbe, np.uint8).tobytes())


def pin_random_lights(setup) -> None:
    """Fix the two estimates the reference draws with unseeded jitter when it
    pre-processes lights (a sky's Power(), Light.cpp:79-104; an env map's
    accWeights, Light.cpp:154-200) at this package's deterministic values, so
    that a recipe written with pin=True renders the same in every run."""
    bbox = setup.scene.BoundingBox()
    for l in setup.scene.infiniteLights:
        if isinstance(l, FunctionInfiniteLight) and l.power_override is None:
            l.PreProcess(bbox)
            l.power_override = float(l.cachedPower)
        elif isinstance(l, TextureInfiniteLight) and l.accWeights is None:
            l.PreProcess(bbox)


def write_recipe(out_dir: Path, scene, camera, spp: int, seed: int, integrator: str, max_depth: int,
                 light_sampler=None, extra_lights: Optional[list] = None, pin: bool = False, strata=None) -> Path:
    """pin: carry the sky's power and the env map's running cell sums
    (pin_random_lights) so the harness replaces its random estimates."""
    out_dir = Path(out_dir)
    out_dir.mkdir(parents=True, exist_ok=True)
    lines: List[str] = ["ptscene 1"]
    if getattr(scene, "ref_models", False):
        # the harness holds the reference's own Model objects
        # (ResourceManager::CacheModel<BLAS4>, oracle/ref_model.cpp), not a
        # BLAS4 it builds over the same GeometricPrimitives
        lines.append("refmodels")
    tex_ids: Dict[int, int] = {}
    mat_ids: Dict[int, int] = {}
    med_ids: Dict[int, int] = {}
    mesh_ids: Dict[int, int] = {}

    def tex(t) -> int:
        if t is None:
            return -1
        if id(t) in tex_ids:
            return tex_ids[id(t)]
        if isinstance(t, CheckerTexture):
            a, b = tex(t.tex1), tex(t.tex2)
        i = len(tex_ids)
        tex_ids[id(t)] = i
        s = " ".join(_f(x) for x in t.colorScale)
        if isinstance(t, SolidColor):
            lines.append(f"texture {i} solid {' '.join(_f(x) for x in t.albedo)} {s}")
        elif isinstance(t, CheckerTexture):
            lines.append(f"texture {i} checker {a} {b} {_f(t.uvscale[0])} {_f(t.uvscale[1])} {s}")
        elif isinstance(t, FloatImageTexture):
            name = f"tex{i}.hdr"
            write_hdr(out_dir / name, t.rgbe)
            lines.append(f"texture {i} floatimage {name} {s}")
        elif isinstance(t, ImageTexture):
            name = f"tex{i}.png"
            write_png(out_dir / name, t.raw)
            lines.append(f"texture {i} image {name} {1 if t.gammaCorrection else 0} {s}")
        else:
            raise TypeError(type(t))
        return i

    def mat(m) -> int:
        if m is None:
            return -1
        if id(m) in mat_ids:
            return mat_ids[id(m)]
        if isinstance(m, MicrofacetDiffuse):
            args = [tex(m.tex), tex(m.norm), tex(m.roughnessTexture), tex(m.metallicTexture), tex(m.alpha)]
            mode = m.alphaTester.mode if m.tester_set else -1
            i = len(mat_ids)
            lines.append(f"material {i} diffuse {' '.join(map(str, args))} {mode} {_f(m.alphaTester.cutoff)}")
        elif isinstance(m, MicrofacetDielectric):
            args = [tex(m.tex), tex(m.norm), tex(m.roughnessTexture), tex(m.alpha)]
            mode = m.alphaTester.mode if m.tester_set else -1
            i = len(mat_ids)
            lines.append(f"material {i} dielectric {_f(m.ri)} {' '.join(map(str, args))} {mode} "
                         f"{_f(m.alphaTester.cutoff)}")
        elif isinstance(m, ThinDielectric):
            t = tex(m.tex)
            i = len(mat_ids)
            lines.append(f"material {i} thin {_f(m.ri)} {t}")
        elif isinstance(m, SpecularConductor):
            i = len(mat_ids)
            lines.append(f"material {i} conductor {' '.join(_f(x) for x in m.albedo)}")
        else:
            raise TypeError(type(m))
        mat_ids[id(m)] = i
        return i

    def med(md) -> int:
        if md is None:
            return -1
        if id(md) not in med_ids:
            i = len(med_ids)
            med_ids[id(md)] = i
            lines.append(f"medium {i} {' '.join(_f(x) for x in md.sigma_a_in)} "
                         f"{' '.join(_f(x) for x in md.sigma_s_in)} {_f(md.phaseFunction.G)} {_f(md.density)} "
                         f"{' '.join(_f(x) for x in md.Le_in)} {_f(md.LeDensity)}")
        return med_ids[id(md)]

    def mesh(me) -> int:
        if id(me) in mesh_ids:
            return mesh_ids[id(me)]
        m, em, md = mat(me.material), tex(me.emissiveTexture), med(me.medium)
        i = len(mesh_ids)
        mesh_ids[id(me)] = i
        name = f"mesh{i}.bin"
        with open(out_dir / name, "wb") as f:
            f.write(me.indices.astype("<u4").tobytes())
            f.write(me.vertices.astype("<f4").tobytes())
            f.write(me.normals.astype("<f4").tobytes())
            f.write(me.texCoords.astype("<f4").tobytes())
            if me.tangents is not None:
                f.write(me.tangents.astype("<f4").tobytes())
        lines.append(f"mesh {i} {name} {me.vertices.shape[0]} {me.GetTriangleCount()} "
                     f"{1 if me.tangents is not None else 0} {m} {em} {md}")
        return i

    blas_ids: Dict[int, int] = {}  # id(Model) -> BLAS index (model / blasdef line order)

    def model_ids(p):
        return [mesh(me) for me in p.meshes]

    def model_override(p):  # Model::BuildBlas(material, medium) (Model.hpp:62-80)
        if p.override_material is None and p.override_medium is None:
            return ""
        return f" override {mat(p.override_material)} {med(p.override_medium)}"


    def level(lv):  # (matrix, animation) operands of one wrapper level
        m16 = " ".join(_f(x) for x in lv.transform.reshape(16))
        anim = (f"{' '.join(_f(x) for x in lv.direction)} {_f(lv.timeBounds[0])} {_f(lv.timeBounds[1])}"
                if isinstance(lv, AnimatedPrimitive) else None)
        return m16, anim

    def wrap_line(lv):  # the harness wraps its last top primitive
        m16, anim = level(lv)
        return f"wrapanim {anim}" if anim else f"wrapprim {m16}"

    for k, p in enumerate(scene.primitives):
        wraps = []
        if isinstance(p, TransformedPrimitive):
            levels = []  # nested wrappers, outermost first
            while isinstance(p, TransformedPrimitive):
                levels.append(p)
                p = p.primitive
            if isinstance(p, Model):
                if id(p) not in blas_ids:
                    ids = model_ids(p)
                    blas_ids[id(p)] = len(blas_ids)
                    lines.append(f"blasdef {blas_ids[id(p)]} {len(ids)} {' '.join(map(str, ids))}{model_override(p)}")
                b = blas_ids[id(p)]
                m16, anim = level(levels[-1])
                lines.append(f"animinstance {k} {b} {anim}" if anim else f"instance {k} {b} {m16}")
                lines.extend(wrap_line(lv) for lv in reversed(levels[:-1]))
                continue
            wraps = [wrap_line(lv) for lv in reversed(levels)]
        if isinstance(p, Model):
            if id(p) in blas_ids:
                lines.append(f"topblas {k} {blas_ids[id(p)]}")
                continue
            ids = model_ids(p)
            blas_ids[id(p)] = len(blas_ids)
            lines.append(f"model {k} {len(ids)} {' '.join(map(str, ids))}{model_override(p)}")
        else:
            sh = p.shape
            m, md = mat(p.material), med(p.medium)
            em, one = -1, 0
            if p.areaLight is not None:
                em = tex(p.areaLight.emissiveTexture)
                one = 1 if p.areaLight.oneSided else 0
            if isinstance(sh, QuadShape):
                g = " ".join(_f(x) for x in [*sh.Q, *sh.u, *sh.v])
                lines.append(f"quad {k} {g} {m} {em} {one} {md}")
            elif isinstance(sh, SphereShape):
                g = " ".join(_f(x) for x in [*sh.center, sh.radius])
                lines.append(f"sphere {k} {g} {m} {em} {one} {md}")
            else:
                raise TypeError(type(sh))
            lines.extend(wraps)
    for l in scene.infiniteLights:
        if isinstance(l, UniformInfiniteLight):
            lines.append(f"infinite uniform {' '.join(_f(x) for x in l.color)}")
        elif isinstance(l, FunctionInfiniteLight):
            pw = f" power {_f(l.power_override)}" if pin and l.power_override is not None else ""
            lines.append(f"infinite sky {' '.join(_f(x) for x in [*l.c0, *l.c1, l.scale])}{pw}")
        elif isinstance(l, TextureInfiniteLight):
            acc = ""
            if pin and l.accWeights is not None:
                path = out_dir / f"accw{len(lines)}.f32"
                np.ascontiguousarray(l.accWeights, np.float32).tofile(path)
                acc = f" accw {path.resolve()}"
            lines.append(f"infinite texture {tex(l.tex)} {_f(l.LeScale)}{acc}")
        else:
            raise TypeError(type(l))
    for l in extra_lights or []:
        if isinstance(l, DistantLight):
            lines.append(f"extralight distant {' '.join(_f(x) for x in [*l.dir, *l.color])}")
        elif isinstance(l, PointLight):
            lines.append(f"extralight point {' '.join(_f(x) for x in [*l.p, *l.color])}")
        else:
            raise TypeError(type(l))
    lines.append(f"lightsampler {'power' if isinstance(light_sampler, PowerLightSampler) else 'uniform'}")
    if scene.GetMedium() is not None:
        lines.append(f"scenemedium {med(scene.GetMedium())}")
    if camera.GetMedium() is not None:
        lines.append(f"cameramedium {med(camera.GetMedium())}")
    W, H = camera.film.Resolution()
    lines.append(f"camera {' '.join(_f(x) for x in [*camera.lookFrom, *camera.lookAt])} {_f(camera.fov)} {W} {H} "
                 f"{_f(camera.FocusAngle)} {_f(camera.FocusDistance)}")
    if camera.shutter is not None:  # Camera(..., glm::vec2 shutterBounds) (Camera.hpp:16-19)
        lines.append(f"shutter {_f(camera.shutter[0])} {_f(camera.shutter[1])}")
    flt = camera.film.filter
    if flt.kind == 0:
        lines.append(f"filter mitchell {_f(flt.radius[0])} {_f(flt.radius[1])} {flt.b!r} {flt.c!r}")
    elif flt.kind == 1:
        lines.append(f"filter box {_f(flt.radius[0])} {_f(flt.radius[1])}")
    elif flt.kind == 3:
        lines.append(f"filter lanczos {_f(flt.radius[0])} {_f(flt.radius[1])} {flt.tau!r}")
    else:
        lines.append(f"filter gaussian {_f(flt.radius[0])} {_f(flt.radius[1])} {flt.sigma!r}")
    lines.append(f"integrator {integrator} {max_depth}")
    lines.append(f"sampler {seed} {spp}")
    if strata:  # a StratifiedSampler(xSamples, ySamples) host (Sampler.hpp:73-151)
        lines.append(f"strata {int(strata[0])} {int(strata[1])}")
    path = out_dir / "recipe.txt"
    path.write_text("\n".join(lines) + "\n")
    # recipe material index -> object, for mapping fixtures onto flat scenes
    write_recipe.material_objects = {i: k for k, i in mat_ids.items()}
    return path
