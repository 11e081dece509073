"""The multi-rank frame with the real HIP renderer: two processes share the
one GPU of the test box, each renders its interleaved sample shard through
`pathtracing_amd.distributed.render_frame` (the code bench.py runs per rank)
into a device film, and the films are SUM-reduced onto rank 0 (gloo, over
host copies: RCCL needs one GPU per rank).  The sum must equal the
one-process frame up to summation order.
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

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _setup():
    from pathtracing_amd import scenes
    return scenes.cornell(W=64, H=48, spp=6, config="c3")


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from pathtracing_amd.distributed import local_samples, reduce_stats, render_frame

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        setup = _setup()
        integ = setup.make_integrator()
        W, H = setup.camera.GetFilm().Resolution()
        film = torch.full((H, W, 4), 7.0, dtype=torch.float64, device="cuda:0")  # overwritten
        st = render_frame(integ, film)
        assert st["paths"] == W * H * local_samples(setup.spp, rank, world)
        tot = reduce_stats(st, torch.device("cpu"))
        if rank == 0:
            q.put((film.cpu().numpy(), tot))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_two_gpu_ranks_sum_to_the_one_process_frame():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    film, tot = q.get(timeout=200)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    setup = _setup()
    integ = setup.make_integrator()
    W, H = setup.camera.GetFilm().Resolution()
    one = torch.zeros((H, W, 4), dtype=torch.float64, device="cuda:0")
    torch.cuda.synchronize()
    st = integ.Render(film_ptr=one.data_ptr())
    torch.cuda.synchronize()
    np.testing.assert_allclose(film, one.cpu().numpy(), rtol=1e-9, atol=1e-12)
    assert tot["paths"] == st["paths"] == W * H * setup.spp
