"""bench.py --render-hook for the CPU suite (TEST INFRASTRUCTURE ONLY).

Stands in for the HIP library so that tests/test_bench_multirank.py can run
bench.py's own multi-rank path end to end on a machine without a GPU:
launch_ranks -> torch.distributed.run -> WORLD_SIZE check -> per-rank shard
render -> film reduce -> JSON line.  The shard render is the oracle (the CPU
restatement of the reference's per-sample loop); its numbers are not GPU
numbers and bench.py labels the line as a CPU rehearsal.
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "oracle"))
import oracle  # noqa: E402


def _integ(setup):
    if not hasattr(setup, "_hook_integ"):
        setup._hook_integ = setup.make_integrator()
    return setup._hook_integ


def render_shard(setup, shard_index, shard_count, film):
    arr, cnt = oracle.render(_integ(setup), threads=1, shard_index=shard_index, shard_count=shard_count)
    film.copy_(torch.from_numpy(arr))
    return {"paths": cnt["paths"], "rays_closest": cnt["closest"], "rays_any": cnt["any"]}


def frame_samples(setup, pixels, samples):
    L, _ = oracle.li_pairs(_integ(setup), pixels, samples)
    return L
