"""Bit-level agreement of the oracle with the reference's fixtures on the
unit cases (CPU, this container; diagnostics for the FMA-contraction map):
per scene, per material, the fraction of BSDF / light-sample / interaction
outputs whose float words equal the reference's, column by column.

  python tools/orc_bits.py [scene ...]"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "oracle"), str(ROOT / "tests" / "golden")]


def _bits(a, b):
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    return (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))


def main(names):
    import oracle
    from fixtures import NAMES, load
    for name in names or NAMES:
        setup, integ, fx = load(name)
        cases = fx["bsdf_cases"]
        for m, fid in enumerate(fx["bsdf_flat_ids"]):
            got = oracle.bsdf(integ.flat, int(fid), cases)
            ref = fx[f"bsdf{m}"]
            b = _bits(got, ref)
            bad = np.nonzero(b.mean(0) < 1)[0]
            print(f"{name:14s} bsdf{m} kind={int(integ.flat.materials[int(fid)]['kind']) if 'kind' in integ.flat.materials.dtype.names else '?'}"
                  f" cases {b.all(1).mean():.4f} cols<1: " + " ".join(f"{c}:{b[:, c].mean():.3f}" for c in bad))
        nc = fx["lsample_cases"].shape[0]
        got = oracle.lights(integ.flat, fx["lsample_cases"]).reshape(-1, nc, 18)
        ref = fx["lsample"].reshape(-1, nc, 18)
        n = min(got.shape[0], ref.shape[0])
        if "lsample_lights" not in fx.files:
            b = _bits(got[:n].reshape(-1, 18), ref[:n].reshape(-1, 18))
            bad = np.nonzero(b.mean(0) < 1)[0]
            print(f"{name:14s} light cases {b.all(1).mean():.4f} cols<1: " + " ".join(f"{c}:{b[:, c].mean():.3f}" for c in bad))
        rays = np.zeros(fx["rays"].shape[0], dtype=[("o", "<f4", 3), ("d", "<f4", 3), ("tmax", "<f4")])
        rays["o"], rays["d"], rays["tmax"] = fx["rays"][:, :3], fx["rays"][:, 3:6], fx["rays"][:, 6]
        got = oracle.trace(integ.flat, rays, any_hit=False)
        ref = fx["hits"]
        both = (got["hit"] > 0) & (ref[:, 0] > 0)
        cols = [("t", got["t"][both], ref[both, 1])]
        for k, sl in (("p", slice(2, 5)), ("n", slice(5, 8)), ("ns", slice(8, 11)), ("uv", slice(11, 13)),
                      ("tangent", slice(13, 16))):
            cols.append((k, got[k][both], ref[both, sl]))
        print(f"{name:14s} hits " + " ".join(f"{k}:{_bits(g, r).all(-1).mean() if g.ndim > 1 else _bits(g, r).mean():.4f}"
                                            for k, g, r in cols))


if __name__ == "__main__":
    main(sys.argv[1:])
