"""Reference films for the C++ drop-in tests (tests/test_gpu_integration.py).

TEST INFRASTRUCTURE.  Runs only where /root/reference exists (this
container): for each drop-in recipe, with the two randomly pre-processed light
estimates pinned (pathtracing_amd.recipe.pin_random_lights), it records the
reference's own frame computed by oracle/_ref/ref_harness on the CPU:

  film_<scene>             FilmTile splat of Integrator::Li over every pixel's
                           spp samples of the PCG stream (fixed SPP)
  adaptive_film_<scene>    TileIntegrator::Render's own adaptive rounds
  adaptive_counts_<scene>  its per-pixel sample counts

so the GPU box runs only the drop-in (hip_harness ... noref) and compares its
film with these (the reference never runs there).

    python tests/golden/gen_dropin.py
"""
from __future__ import annotations

import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(Path(__file__).resolve().parent))

from pathtracing_amd.recipe import pin_random_lights, write_recipe  # noqa: E402

HARNESS = ROOT / "oracle" / "_ref" / "ref_harness"
FILM_SCENES = ["example1", "cornell_c2", "cornell_c3", "zoo", "heightfield", "sanmiguel", "example1_volpath", "fog",
               "instances", "lit_instances", "motion_blur", "motion_path", "stratified", "nested_instances",
               "ref_models", "ref_transformed_models"]
ADAPTIVE_SCENES = ["example1", "cornell_c3", "zoo", "fog", "instances", "sanmiguel", "lens_box", "lit_instances",
                   "motion_blur", "motion_path", "stratified", "stratified_motion", "nested_instances",
                   "ref_models", "ref_transformed_models"]


def pinned_recipe(tmp: Path, setup) -> Path:
    pin_random_lights(setup)
    return write_recipe(tmp, setup.scene, setup.camera, setup.spp, setup.seed, setup.integrator, setup.max_depth,
                        setup.light_sampler, setup.extra_lights, pin=True, strata=setup.strata)


def main(names=None) -> None:
    """names: regenerate only these scenes' entries, keeping the others"""
    from fixtures import parity_scenes
    ps = parity_scenes()
    path = ROOT / "tests" / "golden" / "dropin.npz"
    out = {}
    if names and path.exists():
        with np.load(path, allow_pickle=False) as old:
            out = {k: old[k] for k in old.files}
    for name in sorted(set(FILM_SCENES) | set(ADAPTIVE_SCENES)):
        if names and name not in names:
            continue
        setup = ps[name]()
        W, H = setup.camera.film.Resolution()
        with tempfile.TemporaryDirectory() as td:
            td = Path(td)
            recipe = pinned_recipe(td, setup)
            o = td / "o"
            if name in FILM_SCENES:
                subprocess.run([str(HARNESS), str(recipe), "film", str(o)], check=True)
                out[f"film_{name}"] = np.fromfile(f"{o}.film.bin", np.float64).reshape(H, W, 4)
            if name in ADAPTIVE_SCENES:
                subprocess.run([str(HARNESS), str(recipe), "adaptive", str(o)], check=True)
                out[f"adaptive_film_{name}"] = np.fromfile(f"{o}.adaptive_film.bin", np.float64).reshape(H, W, 4)
                out[f"adaptive_counts_{name}"] = np.fromfile(f"{o}.adaptive_counts.bin", np.uint32).reshape(H, W)
        print(name, flush=True)
    np.savez_compressed(path, **out)


if __name__ == "__main__":
    main(sys.argv[1:] or None)
