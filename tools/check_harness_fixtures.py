"""TEST INFRASTRUCTURE.  Re-run the reference harness (oracle/_ref/ref_harness,
rebuilt from the current oracle/ sources) on the committed parity fixtures'
own inputs and compare what it computes with the committed outputs, bit for
bit: BVH arrays, light order / PMF, closest / any hits, per-sample Li, film,
BSDF and light-sample cases.  A change to the harness's own sources (its
translation unit inlines reference material code, whose FMA contractions GCC
could then form differently: oracle/Makefile) must leave every fixture as it
was.  Runs only where /root/reference exists.

    python tools/check_harness_fixtures.py [NAME ...]
"""
from __future__ import annotations

import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests" / "golden"))

from fixtures import load, parity_scenes  # noqa: E402
from pathtracing_amd.recipe import write_recipe  # noqa: E402

HARNESS = ROOT / "oracle" / "_ref" / "ref_harness"
HARNESS_LANCZOS = ROOT / "oracle" / "_ref" / "ref_harness_lanczos"


def run(*args, exe=HARNESS):
    subprocess.run([str(exe), *map(str, args)], check=True, stdout=subprocess.DEVNULL)


def check(name: str, tmp: Path) -> list[str]:
    setup, _, fx = load(name)  # the fixture's sky power pinned (fixtures.load)
    d = tmp / name
    recipe = write_recipe(d, setup.scene, setup.camera, setup.spp, setup.seed, setup.integrator, setup.max_depth,
                          setup.light_sampler, setup.extra_lights, pin=True, strata=setup.strata)
    out = d / "o"
    bad = []

    def same(key, got):
        want = fx[key]
        g = np.asarray(got).reshape(want.shape) if np.asarray(got).size == want.size else None
        if g is None or g.dtype != want.dtype or g.tobytes() != want.tobytes():
            bad.append(key)

    run(recipe, "bvh", out)
    same("tlas_clusters", np.fromfile(f"{out}.tlas.clusters.bin", np.uint8))
    same("tlas_order", np.fromfile(f"{out}.tlas.order.bin", np.uint32))
    k = 0
    while Path(f"{out}.blas{k}.clusters.bin").exists():
        same(f"blas{k}_clusters", np.fromfile(f"{out}.blas{k}.clusters.bin", np.uint8))
        same(f"blas{k}_order", np.fromfile(f"{out}.blas{k}.order.bin", np.uint32))
        k += 1
    run(recipe, "info", out)
    owners = [ln.split()[0] for ln in Path(f"{out}.lights.txt").read_text().splitlines() if not ln.startswith("sample")]
    if owners != list(fx["light_owner"]):
        bad.append("light_owner")
    fx["rays"].tofile(d / "rays.bin")
    if "ray_times" in fx:
        fx["ray_times"].tofile(d / "times.bin")
        run(recipe, "trace", out, d / "rays.bin", d / "times.bin")
    else:
        run(recipe, "trace", out, d / "rays.bin")
    same("hits", np.fromfile(f"{out}.hits.bin", np.float32))
    same("hit_ids", np.fromfile(f"{out}.ids.bin", np.int32))
    same("any", np.fromfile(f"{out}.any.bin", np.uint8))
    lanczos = "filter lanczos" in recipe.read_text()
    run(recipe, "film", out, exe=HARNESS_LANCZOS if lanczos else HARNESS)
    if not lanczos:  # (its film normalisation is a random estimate, fixtures.RANDOM_INTEGRAL)
        same("film", np.fromfile(f"{out}.film.bin", np.float64))
    run(recipe, "li", out)
    rec = np.fromfile(f"{out}.li.bin", dtype=np.dtype([("px", "<f8"), ("py", "<f8"), ("L", "<f4", 3), ("dims", "<u4")]))
    same("li_L", rec["L"])
    fx["bsdf_cases"].tofile(d / "bsdf.bin")
    m = 0
    while f"bsdf{m}" in fx:
        run(recipe, "bsdf", out, d / "bsdf.bin", m)
        same(f"bsdf{m}", np.fromfile(f"{out}.bsdf{m}.bin", np.float32))
        m += 1
    fx["lsample_cases"].tofile(d / "lights.bin")
    run(recipe, "lights", out, d / "lights.bin")
    ls = np.fromfile(f"{out}.lightsamples.bin", np.float32).reshape(-1, 18)
    if "lsample_lights" in fx:
        nl = ls.shape[0] // fx["lsample_cases"].shape[0]
        ls = ls.reshape(nl, -1, 18)[fx["lsample_lights"]].reshape(-1, 18)
    same("lsample", ls)
    return bad


def main(names=None):
    names = names or list(parity_scenes().keys())
    if not HARNESS_LANCZOS.exists():
        subprocess.run(["make", "-s", "-j8", "-C", str(ROOT / "oracle"), "ref_lanczos"], check=True)
    failed = 0
    with tempfile.TemporaryDirectory() as t:
        for name in names:
            if not (ROOT / "tests" / "golden" / f"{name}.npz").exists():
                print(f"{name}: no fixture")
                continue
            bad = check(name, Path(t))
            failed += bool(bad)
            print(f"{name}: {'identical' if not bad else 'DIFFERS in ' + ', '.join(bad)}", flush=True)
    sys.exit(1 if failed else 0)


if __name__ == "__main__":
    main(sys.argv[1:] or None)
