"""Diagnostic (GPU box): find the C3 frame's non-finite film pixels, their
non-finite samples (pt_frame_samples), and the oracle's Li for the same
(pixel, sample) pairs -- whether the reference's own integrator produces the
value (oracle, the reference's restatement) or the device does alone.
    python tools/c3_nonfinite.py [config]
"""
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
import bench  # noqa: E402
import oracle  # noqa: E402
from pathtracing_amd.distributed import render_frame  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
setup = bench.build_setup(cfg)
integ = setup.make_integrator()
W, H = setup.camera.GetFilm().Resolution()
film = torch.zeros((H, W, 4), dtype=torch.float64, device="cuda:0")
render_frame(integ, film)
torch.cuda.synchronize()
f = film.cpu().numpy()
bad = np.argwhere(~np.isfinite(f).all(-1))
out = {"config": cfg, "nonfinite_pixels": int(bad.shape[0]), "pixels": []}
ctx = integ.context(0)
lo, hi = ctx.frame_sample_range()
for y, x in bad[:8]:
    p = int(y) * W + int(x)
    smp = np.arange(lo, hi + 1, dtype=np.uint32)
    L = ctx.frame_samples(np.full(smp.shape, p, np.uint32), smp)
    nf = np.nonzero(~np.isfinite(L).all(1))[0]
    rec = {"pixel": [int(x), int(y)], "film": f[y, x].tolist(), "nonfinite_samples": smp[nf].tolist()[:8],
           "gpu": L[nf[:8]].tolist()}
    if nf.size:
        want, _ = oracle.li_pairs(integ, np.full(min(8, nf.size), p, np.uint32), smp[nf[:8]])
        rec["oracle"] = np.asarray(want).tolist()
    out["pixels"].append(rec)
print(json.dumps(out, indent=1))
