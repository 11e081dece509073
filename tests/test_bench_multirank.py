"""bench.py's own N > 1 path on the CPU (SURVEY.md §8e, C5 readiness).

`python bench.py --gpus 2` starts its ranks itself (launch_ranks ->
torch.distributed.run), each rank checks WORLD_SIZE, renders its interleaved
sample shard, the films are SUM-reduced onto rank 0 and rank 0 prints the JSON
line.  On this GPU-less machine the ranks use gloo and the CPU stand-in
renderer of tests/bench_cpu_hook.py (the oracle); everything else is the code
the driver runs on an 8-GPU node.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
HOOK = ROOT / "tests" / "bench_cpu_hook.py"


def _bench(n, film, extra=()):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", str(n), "--backend", "gloo", "--render-hook", str(HOOK),
           "--config", "c3", "--res", "24x16", "--spp", "5", "--steps", "1", "--warmup", "1", "--save-film", str(film),
           "--verify-pairs", "16", *extra]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    return json.loads(lines[0]), np.load(film)


def test_bench_two_ranks_end_to_end_over_gloo(tmp_path):
    one, f1 = _bench(1, tmp_path / "f1.npy")
    two, f2 = _bench(2, tmp_path / "f2.npy")
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["config"]["world_size"] == 2
    assert two["config"]["parallelism"] == "sample-shard x2"
    assert "gloo" in two["config"]["film_reduce"]
    # the ranks' rays sum to the 1-rank frame's (the same samples, split)
    assert two["config"]["rays_per_step"] == one["config"]["rays_per_step"] > 0
    # rank 0's reduced film is the 1-rank film up to summation order
    np.testing.assert_allclose(f2, f1, rtol=1e-12, atol=1e-12)
    assert (f2[..., 3] > 0).all()
    # the untimed frame check ran on both ranks
    assert two["verified"]["ok"] and two["verified"]["ranks_ok"] == 2
    assert two["verified"]["pairs_all_ranks"] == 32
    assert "not a GPU measurement" in two["renderer"]


def test_bench_refuses_a_world_size_mismatch(tmp_path):
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--backend", "gloo", "--render-hook",
                        str(HOOK)], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE=1" in (r.stderr + r.stdout)
