"""GPU diagnostics dump (run on the GPU box): the BSDF hook and per-sample Li
of every parity scene, saved to gpurun_out/diag/bsdf_li.npz for offline
comparison with the oracle."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "tests" / "golden"):
    sys.path.insert(0, str(p))

from fixtures import NAMES, load  # noqa: E402


def main():
    out = ROOT / "gpurun_out" / "diag"
    out.mkdir(parents=True, exist_ok=True)
    res = {}
    for name in NAMES:
        _, integ, fx = load(name)
        ctx = integ.context()
        for m, fid in enumerate(fx["bsdf_flat_ids"]):
            res[f"{name}_bsdf{m}"] = ctx.bsdf_cases(int(fid), fx["bsdf_cases"])
        res[f"{name}_L"] = integ.RenderSamples()
    np.savez_compressed(out / "bsdf_li.npz", **res)
    print("wrote", out / "bsdf_li.npz")


if __name__ == "__main__":
    main()
