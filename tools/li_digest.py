"""Per-sample radiance of the parity scenes through one library build, for
bit-level A/B of two builds (GPU box):

  PT_HIP_LIB=<lib.so> python tools/li_digest.py <out.npz>
  python tools/li_digest.py --compare a.npz b.npz

A change meant to keep results bit-identical (layout, inlining, scheduling)
must report 100 % identical samples on every scene."""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests" / "golden")]


def render(out: str) -> None:
    from fixtures import NAMES, load
    res = {}
    for name in NAMES:
        _, integ, _ = load(name)  # with the reference's sky powers, as the parity tests
        res[name] = np.asarray(integ.RenderSamples(), np.float32)
        print(name, res[name].shape, flush=True)
    np.savez(out, **res)


def compare(a: str, b: str) -> int:
    """Bit-identical fraction of b against a, and of each against the
    reference's own per-sample Li (tests/golden/<scene>.npz li_L)."""
    from fixtures import fixture
    A, B = np.load(a), np.load(b)
    bad = 0
    for k in A.files:
        ref = np.asarray(fixture(k)["li_L"], np.float32)
        x, y = A[k].reshape(ref.shape), B[k].reshape(ref.shape)
        same = (x.view(np.uint32) == y.view(np.uint32)).all(-1).mean()
        ra = (x.view(np.uint32) == ref.view(np.uint32)).all(-1).mean()
        rb = (y.view(np.uint32) == ref.view(np.uint32)).all(-1).mean()
        print(f"{k:20s} {same:.6f} of samples bit-identical; vs the reference: a {ra:.4f}, b {rb:.4f}")
        bad += same < 1.0
    return int(bad)


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(compare(sys.argv[2], sys.argv[3]))
    render(sys.argv[1])
