"""Multi-rank frame on the CPU: gloo, world_size 2 and 3.

Each rank renders its interleaved sample shard (s % world == rank) with the
oracle standing in for the GPU renderer (injected through `render_shard`), the
films are SUM-reduced onto rank 0 by `pathtracing_amd.distributed.render_frame`
— the same code bench.py runs over RCCL — and the result must equal the
single-process frame up to summation order.
"""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _setup(config):
    from pathtracing_amd import scenes
    return scenes.cornell(W=24, H=16, spp=5, config=config)


def _worker(rank, world, port, config, q):
    import torch.distributed as dist
    import oracle
    from pathtracing_amd.distributed import local_samples, reduce_stats, render_frame

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        setup = _setup(config)
        integ = setup.make_integrator()
        W, H = setup.camera.GetFilm().Resolution()
        film = torch.zeros((H, W, 4), dtype=torch.float64)

        def shard(i, n, f):
            arr, cnt = oracle.render(integ, threads=1, shard_index=i, shard_count=n)
            f.copy_(torch.from_numpy(arr))
            return {"paths": cnt["paths"], "rays_closest": cnt["closest"], "rays_any": cnt["any"], "ms_total": 1.0}

        st = render_frame(integ, film, render_shard=shard)
        assert st["paths"] == W * H * local_samples(setup.spp, rank, world)
        tot = reduce_stats(st, torch.device("cpu"))
        if rank == 0:
            q.put((film.numpy().copy(), tot))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,config", [(2, "c3"), (3, "c2")])
def test_sharded_frame_reduces_to_the_single_process_frame(world, config):
    import oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, config, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        film, tot = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)

    setup = _setup(config)
    integ = setup.make_integrator()
    ref, cnt = oracle.render(integ, threads=1)
    np.testing.assert_allclose(film, ref, rtol=1e-12, atol=1e-12)
    assert tot["paths"] == cnt["paths"]
    assert tot["rays_closest"] == cnt["closest"]
    assert tot["rays_any"] == cnt["any"]


def test_local_samples_partition_the_frame():
    from pathtracing_amd.distributed import local_samples
    for spp in (0, 1, 5, 8, 1024):
        for n in (1, 2, 3, 4, 8):
            counts = [local_samples(spp, r, n) for r in range(n)]
            assert sum(counts) == spp
            assert counts == [len(range(r, spp, n)) for r in range(n)]


def test_render_frame_validates_the_film():
    from pathtracing_amd.distributed import render_frame
    setup = _setup("c2")
    integ = setup.make_integrator()
    with pytest.raises(ValueError):
        render_frame(integ, torch.zeros((16, 24, 4), dtype=torch.float32), render_shard=lambda i, n, f: {})
    with pytest.raises(ValueError):  # the HIP path needs device memory
        render_frame(integ, torch.zeros((16, 24, 4), dtype=torch.float64))
