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
    bad = np.nonzero((got.view(np.uint32) != orc.view(np.uint32)).any(1))[0]
    print("cases", cases.dtype, len(cases), "bad", bad.tolist())
    print("lights", integ.flat.lights.dtype.names)
    for i in bad:
        print("case", i, cases[i])
        li = int(cases[i][0]) if cases.dtype.names is None else int(cases[i][cases.dtype.names[0]])
        print(" light", integ.flat.lights[li] if 0 <= li < len(integ.flat.lights) else li)
        print(" got", [float(x).hex() for x in got[i]])
        print(" orc", [float(x).hex() for x in orc[i]])
    for k, inst in enumerate(integ.flat.instances if hasattr(integ.flat, "instances") else []):
        print("instance", k, inst)


if __name__ == "__main__":
    main(sys.argv[1])
