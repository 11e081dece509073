"""Device vs oracle light cases, mismatching rows in full (GPU box; diagnostics):

  python tools/diag_lightcases.py <scene>"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "oracle"), str(ROOT / "tests" / "golden")]


def main(name):
    import oracle
    from fixtures import load
    setup, integ, fx = load(name)
    ctx = integ.context()
    cases = fx["lsample_cases"]
    got = np.asarray(ctx.light_cases(cases, integ.flat.lights.shape[0]), np.float32)
    orc = np.asarray(oracle.lights(integ.flat, cases), np.float32)
    nc = len(cases)
    bad = np.nonzero((got.view(np.uint32) != orc.view(np.uint32)).any(1))[0]
    lights = sorted({int(i) // nc for i in bad})
    print("cases", len(cases), "bad rows", len(bad), "lights", lights)
    for li in lights:
        rows = [int(i) for i in bad if int(i) // nc == li]
        print("light", li, integ.flat.lights[li], "rows", len(rows))
        for i in rows[:3]:
            print(" case", cases[i % nc])
            print("  got", [float(x).hex() for x in got[i]])
            print("  orc", [float(x).hex() for x in orc[i]])
    inst = getattr(integ.flat, "instances", None)
    if inst is not None:
        for k, r in enumerate(inst):
            print("instance", k, r)

if __name__ == "__main__":
    main(sys.argv[1])
