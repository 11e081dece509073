"""Diagnostics: per-sample GPU vs oracle vs reference differences per parity scene."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "oracle", ROOT / "tests" / "golden"):
    sys.path.insert(0, str(p))

import oracle  # noqa: E402
from fixtures import NAMES, load  # noqa: E402


def main():
    for name in NAMES:
        setup, integ, fx = load(name)
        L = integ.RenderSamples()
        Lo, _, _ = oracle.li(integ)
        ref = fx["li_L"]
        for tag, a, b in (("gpu-oracle", L, Lo), ("gpu-ref", L, ref), ("oracle-ref", Lo, ref)):
            err = np.abs(a - b).max(-1)
            tol = 1e-4 * np.maximum(1.0, np.abs(b).max(-1))
            bad = np.argwhere(err > tol)
            print(f"{name:16s} {tag:11s} within={1 - len(bad) / err.size:.5f} bad={len(bad)}")
            for pix, s in bad[:4]:
                print(f"     pix={pix} s={s} a={a[pix, s]} b={b[pix, s]}")


if __name__ == "__main__":
    main()
