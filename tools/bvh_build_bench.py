"""Device vs host BVH build on the C4 San-Miguel-class scene's BLAS
(§6 quotes the reference's host build at 4.1 s for
10 M triangles on 8 threads).

    python tools/bvh_build_bench.py [--detail 1.0] [--reps 3] > out.json

The scene is generated once through the reference-API mirror; the triangle
boxes its Model BLAS is built from are captured, then built by pt_bvh4_build
(host, the reference's threaded recursion) and pt_bvh4_build_device (GPU),
checked byte-identical, and timed.  One JSON line.
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from pathtracing_amd import flatten, scenes  # noqa: E402
from pathtracing_amd import native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--detail", type=float, default=1.0)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    captured = []
    orig = flatten.bvh_build

    def capture(boxes):
        captured.append(np.array(boxes, np.float32, copy=True))
        return orig(boxes)

    flatten.bvh_build = capture
    t0 = time.perf_counter()
    scenes.sanmiguel(W=64, H=36, spp=1, detail=a.detail, tex_size=64).make_integrator()
    t_scene = time.perf_counter() - t0
    flatten.bvh_build = orig
    boxes = max(captured, key=len)
    n = boxes.shape[0]
    print(f"{n} boxes captured (scene build {t_scene:.1f} s)", file=sys.stderr, flush=True)

    host_s = []
    for _ in range(a.reps):
        t = time.perf_counter()
        h = N.bvh4_build(boxes)
        host_s.append(time.perf_counter() - t)
    N.bvh4_build_device(boxes[: min(n, 100000)])  # warm the device and the code object
    dev = []
    for _ in range(a.reps):
        st = {}
        t = time.perf_counter()
        d = N.bvh4_build_device(boxes, stats=st)
        st["wall_s"] = time.perf_counter() - t
        dev.append(st)
    ident = (d[0].tobytes() == h[0].tobytes() and np.array_equal(d[2], h[2]) and np.array_equal(d[3], h[3]))
    best = min(dev, key=lambda s: s["ms_total"])
    out = {
        "workload": f"C4 San-Miguel-class model BLAS, {n} triangle boxes (detail {a.detail})",
        "n_prims": n,
        "clusters": int(h[0].shape[0]),
        "host_ms": round(1e3 * min(host_s), 1),
        "device_ms_total": round(best["ms_total"], 1),
        "device_ms_gpu": round(best["ms_device"], 1),
        "device_ms_collapse": round(best["ms_collapse"], 1),
        "levels": best["levels"],
        "small_tasks": best["small_tasks"],
        "nodes": best["nodes"],
        "speedup": round(min(host_s) * 1e3 / best["ms_total"], 2),
        "mprims_per_s": round(n / best["ms_total"] / 1e3, 1),
        "byte_identical": bool(ident),
    }
    print(json.dumps(out))
    if not ident:
        sys.exit(1)


if __name__ == "__main__":
    main()
