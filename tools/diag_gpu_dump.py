"""GPU diagnostics dump (run on the GPU box): per-sample Li of the mini C4
scene at several depths, and the interaction / BSDF hooks on its fixture
cases, saved to gpurun_out/diag/ for offline comparison with the oracle."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "tests" / "golden"):
    sys.path.insert(0, str(p))

from fixtures import NAMES, load  # noqa: E402
from pathtracing_amd import scenes  # noqa: E402


def main():
    out = ROOT / "gpurun_out" / "diag"
    out.mkdir(parents=True, exist_ok=True)
    res = {}
    for depth in (1, 2, 3, 5, 128):
        setup = scenes.sanmiguel(W=48, H=27, spp=2, detail=0.02, tex_size=64, max_depth=depth)
        res[f"L_d{depth}"] = setup.make_integrator().RenderSamples()
    setup, integ, fx = load("sanmiguel")
    rays = np.zeros(fx["rays"].shape[0], dtype=[("o", "<f4", 3), ("d", "<f4", 3), ("tmax", "<f4")])
    rays["o"], rays["d"], rays["tmax"] = fx["rays"][:, :3], fx["rays"][:, 3:6], fx["rays"][:, 6]
    ctx = integ.context()
    res["interact"] = ctx.interact(rays)
    for m, fid in enumerate(fx["bsdf_flat_ids"]):
        res[f"bsdf{m}"] = ctx.bsdf_cases(int(fid), fx["bsdf_cases"])
    res["lights"] = ctx.light_cases(fx["lsample_cases"], integ.flat.lights.shape[0])
    for name in NAMES:
        _, ig, fxn = load(name)
        rr = np.zeros(fxn["rays"].shape[0], dtype=rays.dtype)
        rr["o"], rr["d"], rr["tmax"] = fxn["rays"][:, :3], fxn["rays"][:, 3:6], fxn["rays"][:, 6]
        res[f"interact_{name}"] = ig.context().interact(rr)
    np.savez_compressed(out / "c4mini.npz", **res)
    print("wrote", out / "c4mini.npz")


if __name__ == "__main__":
    main()
