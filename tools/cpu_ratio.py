"""Speed of the CPU restatement (oracle/pt_oracle.c, the `port` bench.py
times on the GPU box) against the reference itself (oracle/_ref/ref_harness,
built from /root/reference; it cannot travel to the GPU box), on the same
scenes, sample stream and thread count, in this container (BASELINE.md §3,
SURVEY.md §8(d) "CPU baseline timing").  TEST INFRASTRUCTURE.

    python tools/cpu_ratio.py profiles/r02_cpu_ratio.json
    python tools/cpu_ratio.py OUT --scenes NAME[,NAME] --threads 1,8 --merge OLD.json

(--scenes / --threads: a subset; --merge: keep OLD.json's other scenes)

Both sides run a fixed-SPP tile loop over Li with the counter-based sample
stream (ref_harness `time ... li`; oracle.render); Mrays/s counts every
Scene::Intersect + Scene::IntersectPred.  Median of 3 runs each.  The
reference's own TileIntegrator::Render (adaptive rounds, UniformSampler) is
timed beside them for scale.
"""
import json
import os
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))

HARNESS = ROOT / "oracle" / "_ref" / "ref_harness"


def scenes_():
    from pathtracing_amd import scenes
    return {
        "c1_example1_path_256x256_16spp": lambda: scenes.example_1(W=256, H=256, spp=16),
        "heightfield_1M_tris_256x256_16spp": lambda: scenes.heightfield(n=700, W=256, H=256, spp=16),
        "c4_recipe_2pct_160x90_16spp_depth128": lambda: scenes.sanmiguel(W=160, H=90, spp=16, detail=0.02,
                                                                       tex_size=64),
        # the full-detail C4 scene (~10 M triangles, the benched one) on a
        # small film: what bench.py's cpu_baseline times the port on
        "c4_full_192x108_32spp_depth128": lambda: scenes.sanmiguel(W=192, H=108, spp=32),
    }


def _rec(stdout):
    # Render's progress line ends in '\r' without a newline: take the record from its brace
    return next(json.loads(l[l.index("{"):]) for l in stdout.replace("\r", "\n").splitlines()
                if "{" in l)["mrays_per_s"]


def median(xs):
    return sorted(xs)[len(xs) // 2]


def _time_ref(recipe, tmp, threads, spp, mode):
    r = subprocess.run([str(HARNESS), str(recipe), "time", str(Path(tmp) / "o"), str(threads), str(spp), mode],
                       capture_output=True, text=True, check=True)
    return _rec(r.stdout)


def _time_port(integ, threads):
    import oracle
    t0 = time.perf_counter()
    _, cnt = oracle.render(integ, threads=threads)
    dt = time.perf_counter() - t0
    return (cnt["closest"] + cnt["any"]) / dt / 1e6


def main(out, names=None, threads=None, merge=None):
    """port / reference at every thread count 1, 2, 4, ... up to this
    container's CPUs (bench.py applies the ratio measured at the thread count
    closest to the one it times the port at)."""
    from pathtracing_amd.recipe import write_recipe
    ncpu = os.cpu_count() or 8
    counts = threads or sorted({1 << k for k in range(ncpu.bit_length()) if (1 << k) <= ncpu} | {ncpu})
    res = {"_meta": {"threads": counts, "host": "build container", "runs": 3,
                     "cpu": next((l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo")
                                  if l.startswith("model name")), "?")}}
    if merge:
        old = json.loads(Path(merge).read_text())
        res.update({k: v for k, v in old.items() if k not in ("_meta", "summary")})
        res["_meta"]["merged_from"] = Path(merge).name
    for name, mk in scenes_().items():
        if names and name not in names:
            continue
        setup = mk()
        integ = setup.make_integrator()
        entry = {"by_threads": {}}
        with tempfile.TemporaryDirectory() as tmp:
            recipe = write_recipe(Path(tmp), setup.scene, setup.camera, setup.spp, setup.seed, setup.integrator,
                                  setup.max_depth, setup.light_sampler, setup.extra_lights)
            for t in counts:
                ref = median([_time_ref(recipe, tmp, t, setup.spp, "li") for _ in range(3)])
                port = median([_time_port(integ, t) for _ in range(3)])
                entry["by_threads"][str(t)] = {"reference_li_loop_mrays": round(ref, 3), "port_mrays": round(port, 3),
                                               "port_over_reference": round(port / ref, 3)}
                print(name, t, entry["by_threads"][str(t)], flush=True)
            entry["reference_render_mrays"] = round(
                median([_time_ref(recipe, tmp, max(counts), setup.spp, "render") for _ in range(3)]), 3)
        top = entry["by_threads"][str(max(counts))]
        entry.update(top)  # the full-container figures at the top level
        res[name] = entry
    ratios = [v["port_over_reference"] for k, v in res.items() if not k.startswith("_")]
    res["summary"] = {"port_over_reference_min": min(ratios), "port_over_reference_max": max(ratios),
                      "threads": max(counts), "source": f"{Path(out).name} (tools/cpu_ratio.py)"}
    Path(out).write_text(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--scenes", default=None)
    ap.add_argument("--threads", default=None)
    ap.add_argument("--merge", default=None)
    a = ap.parse_args()
    main(a.out, a.scenes.split(",") if a.scenes else None,
         [int(t) for t in a.threads.split(",")] if a.threads else None, a.merge)
