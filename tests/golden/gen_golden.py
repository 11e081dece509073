"""Generate the golden fixtures in tests/golden/*.npz from the reference itself.

TEST INFRASTRUCTURE.  Runs only where /root/reference exists: it builds
oracle/_ref/ref_harness from the reference sources (oracle/Makefile), writes a
recipe for each parity scene (pathtracing_amd.recipe), and records what the
reference computes on it:

  bvh_*      BVH4 clusters / root / primitive order        (F0)
  lights_*   light order, Power(), PMF; LightSampler::Sample picks (F4)
  trace_*    closest-hit interactions + any-hit booleans    (F1/F2)
  li_*       per-sample Integrator::Li under the PCG stream (F7)
  film       FilmTile splat of those samples + filter table (F6/F8)
  bsdf_*     Material scatter / calc_attenuation / PDF       (F3)
  lsample_*  Light::sample / PDF / L                         (F4)
  adaptive.npz  TileIntegrator::Render's own adaptive loop (Integrators.cpp:
             55-86) on the PCG stream: per-pixel sample counts + film
  stats.npz  the same Render with its own StratifiedSampler and unseeded RNGs:
             per-pixel sample count, mean and variance (F8)

    python tests/golden/gen_golden.py
"""
from __future__ import annotations

import subprocess
import sys
import tempfile
import zlib
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(Path(__file__).resolve().parent))

from pathtracing_amd import scenes  # noqa: E402
from pathtracing_amd.recipe import write_recipe  # noqa: E402
from pathtracing_amd.scene import FunctionInfiniteLight  # noqa: E402

HARNESS = ROOT / "oracle" / "_ref" / "ref_harness"
OUT = ROOT / "tests" / "golden"


HARNESS_LANCZOS = ROOT / "oracle" / "_ref" / "ref_harness_lanczos"


def harness(*args):
    exe = HARNESS
    # a Lanczos recipe's film needs the harness that parses that filter (a
    # separate build, oracle/Makefile ref_lanczos); every other command
    # ignores the filter and runs the default build
    if len(args) > 1 and args[1] == "film" and "filter lanczos" in Path(args[0]).read_text():
        if not HARNESS_LANCZOS.exists():
            subprocess.run(["make", "-s", "-j8", "-C", str(ROOT / "oracle"), "ref_lanczos"], check=True)
        exe = HARNESS_LANCZOS
    subprocess.run([str(exe), *map(str, args)], check=True)


def parity_scenes():
    from fixtures import parity_scenes as ps
    return {k: f() for k, f in ps().items()}


def random_rays(setup, n, rng):
    bb = setup.scene.BoundingBox().astype(np.float64)
    lo, hi = bb[:3], bb[3:]
    span = np.minimum(hi - lo, 20.0)
    mid = 0.5 * (lo + hi)
    o = mid + (rng.random((n, 3)) - 0.5) * span
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    # half the rays from the camera toward the scene centre region
    cam = setup.camera.lookFrom.astype(np.float64)
    k = n // 2
    o[:k] = cam
    tgt = mid + (rng.random((k, 3)) - 0.5) * span * 0.5
    dd = tgt - cam
    d[:k] = dd / np.linalg.norm(dd, axis=1, keepdims=True)
    tmax = np.full(n, np.inf)
    tmax[::4] = rng.random(len(tmax[::4])) * 3.0  # bounded queries too
    return np.concatenate([o, d, tmax[:, None]], 1).astype(np.float32)


def bsdf_cases(n, rng):
    def unit(m):
        v = rng.normal(size=(m, 3))
        return v / np.linalg.norm(v, axis=1, keepdims=True)
    ns = unit(n)
    ng = unit(n) * 0.3 + ns
    ng /= np.linalg.norm(ng, axis=1, keepdims=True)
    a = unit(n)
    tg = a - ns * np.sum(a * ns, 1, keepdims=True)
    tg /= np.linalg.norm(tg, axis=1, keepdims=True)
    d = unit(n)
    o = rng.normal(size=(n, 3))
    p = o + d * 1.0
    uv = rng.random((n, 2))
    u = rng.random((n, 1))
    uv2 = rng.random((n, 2))
    other = unit(n)
    cases = np.concatenate([o, d, p, ng, ns, tg, uv, np.ones((n, 1)), u, uv2, other], 1)
    return cases.astype(np.float32)


def gen(name, setup, rng, tmp: Path):
    d = tmp / name
    recipe = write_recipe(d, setup.scene, setup.camera, setup.spp, setup.seed, setup.integrator,
                          setup.max_depth, setup.light_sampler, setup.extra_lights, strata=setup.strata)
    out = d / "o"
    res = {}
    harness(recipe, "bvh", out)
    res["tlas_clusters"] = np.fromfile(f"{out}.tlas.clusters.bin", np.uint8)
    res["tlas_root"] = np.fromfile(f"{out}.tlas.root.bin", np.uint8)
    res["tlas_order"] = np.fromfile(f"{out}.tlas.order.bin", np.uint32)
    k = 0
    while Path(f"{out}.blas{k}.clusters.bin").exists():
        res[f"blas{k}_clusters"] = np.fromfile(f"{out}.blas{k}.clusters.bin", np.uint8)
        res[f"blas{k}_root"] = np.fromfile(f"{out}.blas{k}.root.bin", np.uint8)
        res[f"blas{k}_order"] = np.fromfile(f"{out}.blas{k}.order.bin", np.uint32)
        k += 1
    harness(recipe, "info", out)
    lines = Path(f"{out}.lights.txt").read_text().splitlines()
    owners, delta, power, pmf, picks_u, picks = [], [], [], [], [], []
    for ln in lines:
        f = ln.split()
        if f[0] == "sample":
            picks_u.append(float(f[1]))
            picks.append(f[2])
        else:
            owners.append(f[0])
            delta.append(int(f[1]))
            power.append(float(f[2]))
            pmf.append(float(f[3]))
    res["light_owner"] = np.array(owners)
    res["light_delta"] = np.array(delta, np.int32)
    res["light_power"] = np.array(power, np.float64)
    res["light_pmf"] = np.array(pmf, np.float64)
    res["pick_u"] = np.array(picks_u, np.float32)
    res["pick_owner"] = np.array(picks)
    rays = random_rays(setup, 2048, rng)
    rays.tofile(d / "rays.bin")
    sh = getattr(setup.camera, "shutter", None)
    if sh is not None:  # a shutter scene: each ray at its own time in the shutter (and past it)
        times = (float(sh[0]) + (rng.random(rays.shape[0]) * 1.2 - 0.1) * float(sh[1] - sh[0])).astype(np.float32)
        times.tofile(d / "times.bin")
        harness(recipe, "trace", out, d / "rays.bin", d / "times.bin")
        res["ray_times"] = times
    else:
        harness(recipe, "trace", out, d / "rays.bin")
    res["rays"] = rays
    res["hits"] = np.fromfile(f"{out}.hits.bin", np.float32).reshape(-1, 16)
    res["hit_ids"] = np.fromfile(f"{out}.ids.bin", np.int32).reshape(-1, 3)
    res["any"] = np.fromfile(f"{out}.any.bin", np.uint8)
    harness(recipe, "film", out)
    W, H = setup.camera.film.Resolution()
    res["film"] = np.fromfile(f"{out}.film.bin", np.float64).reshape(H, W, 4)
    res["filter_table"] = np.fromfile(f"{out}.filter.bin", np.float64)
    harness(recipe, "li", out)
    rec = np.fromfile(f"{out}.li.bin", dtype=np.dtype([("px", "<f8"), ("py", "<f8"), ("L", "<f4", 3),
                                                      ("dims", "<u4")]))
    res["li_p"] = np.stack([rec["px"], rec["py"]], 1).reshape(W * H, setup.spp, 2)
    res["li_L"] = rec["L"].reshape(W * H, setup.spp, 3)
    res["li_dims"] = rec["dims"].reshape(W * H, setup.spp)
    # material cases for every material in recipe order
    nmat = sum(1 for ln in recipe.read_text().splitlines() if ln.startswith("material "))
    cases = bsdf_cases(256, rng)
    cases.tofile(d / "bsdf.bin")
    res["bsdf_cases"] = cases
    mobj = write_recipe.material_objects
    res["bsdf_flat_ids"] = np.array([setup.scene.flat.material_ids[mobj[m]] for m in range(nmat)], np.int32)
    for m in range(nmat):
        harness(recipe, "bsdf", out, d / "bsdf.bin", m)
        res[f"bsdf{m}"] = np.fromfile(f"{out}.bsdf{m}.bin", np.float32).reshape(-1, 20)
    lc = np.concatenate([rng.random((64, 2)), rng.normal(size=(64, 3)) * 0.5], 1).astype(np.float32)
    lc.tofile(d / "lights.bin")
    harness(recipe, "lights", out, d / "lights.bin")
    res["lsample_cases"] = lc
    res["lsample"] = np.fromfile(f"{out}.lightsamples.bin", np.float32).reshape(-1, 18)
    nl = res["lsample"].shape[0] // lc.shape[0]
    if nl > 256:  # keep the fixture small: a spread of lights (first, evenly spaced, last)
        sel = np.unique(np.r_[np.arange(64), np.linspace(0, nl - 1, 128).astype(np.int64), np.arange(nl - 8, nl)])
        res["lsample_lights"] = sel
        res["lsample"] = res["lsample"].reshape(nl, lc.shape[0], 18)[sel].reshape(-1, 18)
    np.savez_compressed(OUT / f"{name}.npz", **res)
    sz = (OUT / f"{name}.npz").stat().st_size
    print(f"{name}: {sz / 1024:.0f} KiB, {len(owners)} lights, {k} BLAS, "
          f"nonzero Li {(res['li_L'].sum(-1) > 0).mean():.2f}")


def resolve_films(rng):
    """Film accumulations the resolve fixture covers: the parity scenes'
    reference films plus a synthetic HDR film with the edge cases (zero
    weight, tiny / huge / negative radiance, the sRGB knee)."""
    films = {}
    for name in ("example1", "cornell_c3", "fog", "sanmiguel"):
        films[name] = np.load(OUT / f"{name}.npz", allow_pickle=False)["film"]
    H, W = 40, 48
    rgb = np.exp(rng.uniform(np.log(1e-5), np.log(1e4), (H, W, 3)))
    w = rng.uniform(0.5, 30.0, (H, W, 1))
    syn = np.concatenate([rgb * w, w], -1)
    syn[0, :4] = 0.0                                   # zero weight: 0/0
    syn[1, :3, :3] = -syn[1, :3, :3]                   # negative radiance
    syn[2, :3, :3] = syn[2, :3, 3:4] * 0.0031308       # at the sRGB knee
    syn[3, :3, :3] = syn[3, :3, 3:4] * 1e30            # overflow in float
    films["synthetic"] = syn
    return films


def gen_resolve(rng, tmp: Path):
    """Film::WritePNG's tone map + sRGB + u8 (Film.hpp:183-196) by the
    reference's own functions, for pt_film_resolve."""
    res = {}
    for name, film in resolve_films(rng).items():
        H, W = film.shape[:2]
        p = tmp / f"{name}.film.bin"
        np.ascontiguousarray(film, np.float64).tofile(p)
        harness("tonemap", tmp / name, p, W, H)
        res[f"{name}_film"] = film
        res[f"{name}_jodie"] = np.fromfile(f"{tmp / name}.ldr_jodie.bin", np.uint8).reshape(H, W, 3)
        res[f"{name}_aces"] = np.fromfile(f"{tmp / name}.ldr_aces.bin", np.uint8).reshape(H, W, 3)
    np.savez_compressed(OUT / "film_resolve.npz", **res)
    print(f"film_resolve: {(OUT / 'film_resolve.npz').stat().st_size / 1024:.0f} KiB")


ADAPTIVE_SCENES = ("cornell_c3", "example1", "example1_simple", "zoo", "fog", "lens_box", "instances", "mitchell2",
                   "stratified", "motion_path")


def gen_adaptive(tmp: Path):
    """The reference's TileIntegrator::Render, adaptive rounds included, run
    by ref_harness `adaptive` (one thread, DetSampler numbering round r's
    samples r*spp + index) on the parity scenes without a randomly
    pre-processed sky (their Power() would differ between harness runs)."""
    from fixtures import load
    res = {}
    for name in ADAPTIVE_SCENES:
        setup, _, _ = load(name)
        d = tmp / f"adaptive_{name}"
        recipe = write_recipe(d, setup.scene, setup.camera, setup.spp, setup.seed, setup.integrator,
                              setup.max_depth, setup.light_sampler, setup.extra_lights, strata=setup.strata)
        out = d / "o"
        subprocess.run([str(HARNESS), str(recipe), "adaptive", str(out)], check=True, stdout=subprocess.DEVNULL)
        W, H = setup.camera.film.Resolution()
        res[f"{name}_counts"] = np.fromfile(f"{out}.adaptive_counts.bin", np.uint32).reshape(H, W)
        res[f"{name}_film"] = np.fromfile(f"{out}.adaptive_film.bin", np.float64).reshape(H, W, 4)
    np.savez_compressed(OUT / "adaptive.npz", **res)
    print(f"adaptive: {(OUT / 'adaptive.npz').stat().st_size / 1024:.0f} KiB, {len(ADAPTIVE_SCENES)} scenes")


def gen_c4_band(tmp: Path):
    """The full-size C4 scene (~10 M triangles, sanmiguel at detail 1) at
    192 x 108: the reference's own per-sample Li (ref_harness li, PCG stream)
    for the pixel rows 40..47 at 2 spp, with that run's light powers (the
    sky's is a random estimate per run).  Only the samples are kept."""
    setup = scenes.sanmiguel(W=192, H=108, spp=2)
    d = tmp / "c4band"
    recipe = write_recipe(d, setup.scene, setup.camera, setup.spp, setup.seed, setup.integrator,
                          setup.max_depth, setup.light_sampler, setup.extra_lights)
    out = d / "o"
    harness(recipe, "li", out, 0, 40, 192, 48, 2)
    rec = np.fromfile(f"{out}.li.bin", dtype=np.dtype([("px", "<f8"), ("py", "<f8"), ("L", "<f4", 3),
                                                      ("dims", "<u4")]))
    np.savez_compressed(OUT / "c4_band.npz", li_L=rec["L"].reshape(192 * 8, 2, 3),
                        li_p=np.stack([rec["px"], rec["py"]], 1).reshape(192 * 8, 2, 2),
                        light_power=np.fromfile(f"{out}.lipower.bin", np.float64))
    print(f"c4_band: {(OUT / 'c4_band.npz').stat().st_size / 1024:.0f} KiB")


def gen_emission_power(tmp: Path):
    """AreaLight::PreProcess's Power() with textured emission (Light.cpp:
    277-287), by the reference (ref_harness info, 5 runs: its jittered
    estimate is random), for scenes.textured_emitters."""
    setup = scenes.textured_emitters()
    d = tmp / "emission"
    recipe = write_recipe(d, setup.scene, setup.camera, setup.spp, setup.seed, setup.integrator,
                          setup.max_depth, setup.light_sampler, setup.extra_lights)
    runs = []
    for r in range(5):
        harness(recipe, "info", d / f"o{r}")
        runs.append([float(ln.split()[2]) for ln in Path(f"{d}/o{r}.lights.txt").read_text().splitlines()
                     if not ln.startswith("sample")])
    np.savez_compressed(OUT / "emission_power.npz", power=np.array(runs, np.float64))
    print(f"emission_power: {len(runs[0])} lights x 5 runs")


def gen_envmap(tmp: Path):
    """TextureInfiniteLight (Light.cpp:110-200) through the reference: Le(dir)
    and PDF(dir) for a spread of directions and Power(), ref_harness `envle`
    (its PreProcess is randomly jittered: PDF and Power vary by the estimate's
    noise; Le is exact)."""
    setup = scenes.envmap(W=32, H=32, spp=4)
    d = tmp / "envmap"
    recipe = write_recipe(d, setup.scene, setup.camera, setup.spp, setup.seed, setup.integrator,
                          setup.max_depth, setup.light_sampler, setup.extra_lights)
    rng = np.random.default_rng(20261016)
    dirs = rng.normal(size=(1024, 3))
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    dirs = dirs.astype(np.float32)
    dirs.tofile(d / "dirs.bin")
    out = d / "o"
    harness(recipe, "envle", out, d / "dirs.bin")
    raw = np.fromfile(f"{out}.envle.bin", np.float32)
    np.savez_compressed(OUT / "envmap.npz", dirs=dirs, le_pdf=raw[:-1].reshape(-1, 4), power=raw[-1:])
    print(f"envmap: {(OUT / 'envmap.npz').stat().st_size / 1024:.0f} KiB")


STATS_SCENES = {
    "example1": lambda: scenes.example_1(W=48, H=48, spp=1024, seed=0x5EED0051),
    "cornell_c3": lambda: scenes.cornell(W=48, H=48, spp=1024, config="c3", seed=0x5EED0052),
    "blend_box": lambda: scenes.blend_box(W=48, H=48, spp=1024, seed=0x5EED0053),
    "envmap": lambda: scenes.envmap(W=48, H=48, spp=1024, seed=0x5EED0054),
    # the C4 recipe class (textures, alpha-masked foliage, sun + sky, lamps,
    # glass, depth 128, PowerLightSampler, Mitchell) at 2 % detail
    "sanmiguel_c4": lambda: scenes.sanmiguel(W=64, H=64, spp=1024, detail=0.02, tex_size=256),
}


def gen_stats(tmp: Path, only=None):
    """F8: the reference's own TileIntegrator::Render with main.cpp's
    StratifiedSampler(32, 32) and its unseeded random numbers (8 threads,
    adaptive rounds): per pixel the samples traced, their mean and variance.
    only: regenerate these scenes and keep the others' committed entries."""
    res = {}
    if only and (OUT / "stats.npz").exists():
        old = np.load(OUT / "stats.npz", allow_pickle=False)
        res = {k: old[k] for k in old.files}
    for name, make in STATS_SCENES.items():
        if only and name not in only:
            continue
        setup = make()
        d = tmp / f"stats_{name}"
        recipe = write_recipe(d, setup.scene, setup.camera, setup.spp, setup.seed, setup.integrator,
                              setup.max_depth, setup.light_sampler, setup.extra_lights)
        out = d / "o"
        subprocess.run([str(HARNESS), str(recipe), "stats", str(out), "8"], check=True, stdout=subprocess.DEVNULL)
        W, H = setup.camera.film.Resolution()
        res[name] = np.fromfile(f"{out}.stats.bin", np.float64).reshape(H, W, 7)
    np.savez_compressed(OUT / "stats.npz", **res)
    print(f"stats: {(OUT / 'stats.npz').stat().st_size / 1024:.0f} KiB, {len(res)} scenes")


def gen_mat4_inverse(rng, tmp: Path):
    """glm::inverse(mat4) by the reference's own build of glm
    (oracle/glm_inverse_probe.cpp): what TransformedPrimitive's ctor stores
    as invTransform (Primitive.hpp:37), for pt_mat4_inverse.  Instance-like
    matrices (rotate / non-uniform scale / translate in every order, axis
    rotations with exact zeros) and general ones."""
    from pathtracing_amd.scene import mat4_identity, mat4_rotate, mat4_scale, mat4_translate
    I = mat4_identity()
    ms = []
    for k in range(3000):
        ops = [lambda m: mat4_translate(m, rng.normal(size=3)),
               lambda m: mat4_rotate(m, rng.uniform(-3.2, 3.2), rng.normal(size=3)),
               lambda m: mat4_scale(m, rng.uniform(0.2, 3.0, 3))]
        m = I
        for j in rng.permutation(3)[:1 + k % 3]:
            m = ops[j](m)
        ms.append(m)
    for k in range(1500):
        m = mat4_rotate(I, rng.uniform(-3.2, 3.2), [(1, 0, 0), (0, 1, 0), (0, 0, 1)][k % 3])
        if k % 2:
            m = mat4_translate(m, rng.normal(size=3))
        if k % 5 == 0:
            m = mat4_scale(m, rng.uniform(0.2, 3.0, 3))
        ms.append(m)
    ms += [rng.normal(size=(4, 4)) for _ in range(1500)]
    A = np.stack([np.ascontiguousarray(m, np.float32).reshape(16) for m in ms])
    A.tofile(tmp / "m.bin")
    subprocess.run([str(HARNESS.parent / "glm_inverse_probe"), str(tmp / "m.bin"), str(tmp / "inv.bin")], check=True)
    inv = np.fromfile(tmp / "inv.bin", np.float32).reshape(-1, 16)
    np.savez_compressed(OUT / "mat4_inverse.npz", m=A, inv=inv)
    print(f"mat4_inverse: {(OUT / 'mat4_inverse.npz').stat().st_size / 1024:.0f} KiB, {len(A)} matrices")


def gen_anim_inverse(rng, tmp: Path):
    """glm::inverse of identity + translation t by the reference's own build
    of glm (oracle/glm_inverse_probe.cpp): the matrix AnimatedPrimitive
    inverts at each ray's time (Primitive.cpp:82-89), for the device's closed
    form (pt_shading.h anim_inverse, test hook pt_anim_inverse_cases).  Every
    sign pattern of +0 and +-{denormal, tiny, unit, large, near-max} per axis,
    and random translations over 20 decades.  No -0 component: the device
    builds the column as v + 0 (anim_transform), as glm's matrix product
    rounds it."""
    mags = [1e-40, 1e-30, 0.3, 1.0, 7.5, 1e20, 3e38]
    vals = [0.0] + [s * m for m in mags for s in (1.0, -1.0)]
    t = [(a, b, c) for a in vals for b in vals for c in vals]
    r = rng.normal(size=(2000, 3)) * 10.0 ** rng.uniform(-10, 10, (2000, 1))
    r[rng.random((2000, 3)) < 0.2] = 0.0
    t = np.concatenate([np.asarray(t, np.float64), r]).astype(np.float32) + np.float32(0.0)  # (-0 -> +0)
    A = np.tile(np.eye(4, dtype=np.float32).reshape(16), (t.shape[0], 1))
    A[:, 12:15] = t
    A.tofile(tmp / "anim.bin")
    subprocess.run([str(HARNESS.parent / "glm_inverse_probe"), str(tmp / "anim.bin"), str(tmp / "anim_inv.bin")],
                   check=True)
    inv = np.fromfile(tmp / "anim_inv.bin", np.float32).reshape(-1, 16)
    np.savez_compressed(OUT / "anim_inverse.npz", t=t, inv=inv)
    print(f"anim_inverse: {(OUT / 'anim_inverse.npz').stat().st_size / 1024:.0f} KiB, {len(t)} translations")


def main(names=None):
    """All scenes share one rng stream (the committed round-1 fixtures); a
    scene regenerated alone (`gen_golden.py NAME...`) uses its own stream
    seeded from its name."""
    if not HARNESS.exists():
        subprocess.run(["make", "-s", "-j8", "-C", str(ROOT / "oracle"), "ref"], check=True)
    from fixtures import parity_scenes as ps
    rng = np.random.default_rng(20261015)
    with tempfile.TemporaryDirectory() as t:
        for name, make in ps().items():
            if names and name not in names:
                continue
            r = np.random.default_rng([20261015, zlib.crc32(name.encode())]) if names else rng
            gen(name, make(), r, Path(t))
        if not names or "film_resolve" in names:
            gen_resolve(np.random.default_rng([20261016, 7]), Path(t))
        if not names or "adaptive" in names:
            gen_adaptive(Path(t))
        if not names or "stats" in names:
            gen_stats(Path(t))
        elif any(n.startswith("stats:") for n in names):  # stats:NAME regenerates one stats scene
            gen_stats(Path(t), [n[6:] for n in names if n.startswith("stats:")])
        if not names or "envmap" in names:
            gen_envmap(Path(t))
        if not names or "c4_band" in names:
            gen_c4_band(Path(t))
        if not names or "emission_power" in names:
            gen_emission_power(Path(t))
        if not names or "mat4_inverse" in names:
            gen_mat4_inverse(np.random.default_rng([20261018, 4]), Path(t))
        if not names or "anim_inverse" in names:
            gen_anim_inverse(np.random.default_rng([20261019, 6]), Path(t))


if __name__ == "__main__":
    main(sys.argv[1:] or None)
