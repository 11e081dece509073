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


# ---------------------------------------------------------------- init_film_comm's agreement steps
class _StubCtx:
    """Stands in for the library context: records the calls init_film_comm
    makes, fails comm_init_rank on the ranks told to."""

    def __init__(self, fail: bool, joined: int = 0):
        self.fail = fail
        self.comm_ranks = joined
        self.calls = []

    def comm_init_rank(self, n, rank, uid):
        self.calls.append(("init", n, rank, uid))
        if self.fail:
            raise RuntimeError("stub: RCCL refused")
        self.comm_ranks = n

    def comm_destroy(self):
        self.calls.append(("destroy",))
        self.comm_ranks = 0


class _StubIntegrator:
    def __init__(self, ctx):
        self.ctx = ctx

    def context(self, device):
        return self.ctx


def _comm_worker(rank, world, port, fail_ranks, joined, q):
    import torch.distributed as dist
    from pathtracing_amd import distributed
    from pathtracing_amd.integrator import Context

    # rank 0's id comes from the stub, not from RCCL (no GPU here)
    Context.comm_unique_id = staticmethod(lambda: bytes(range(128)))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ctx = _StubCtx(rank in fail_ranks, joined)
        ok = distributed.init_film_comm(_StubIntegrator(ctx), 0)
        q.put((rank, ok, ctx.calls, ctx.comm_ranks))
    finally:
        dist.destroy_process_group()


def _run_comm(world, fail_ranks, joined=0):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_comm_worker, args=(r, world, port, fail_ranks, joined, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        got = sorted(q.get(timeout=120) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    return got


@pytest.mark.timeout(180)
def test_init_film_comm_falls_back_on_every_rank_when_one_rank_fails():
    """Rank 1's comm_init_rank fails: neither rank hangs, both return False,
    and the rank whose init succeeded drops its communicator so the frame
    reduces through torch.distributed on both."""
    got = _run_comm(2, fail_ranks=(1,))
    for rank, ok, calls, comm_ranks in got:
        assert ok is False
        assert comm_ranks == 0
        assert calls[0][:3] == ("init", 2, rank) and calls[0][3] == bytes(range(128))
    assert got[0][2][-1] == ("destroy",)      # rank 0 had joined: dropped
    assert ("destroy",) not in got[1][2]      # rank 1 never joined


@pytest.mark.timeout(180)
def test_init_film_comm_joins_every_rank_with_rank0s_id():
    got = _run_comm(2, fail_ranks=())
    for rank, ok, calls, comm_ranks in got:
        assert ok is True and comm_ranks == 2
        assert calls == [("init", 2, rank, bytes(range(128)))]


@pytest.mark.timeout(180)
def test_init_film_comm_all_already_joined_is_a_no_op():
    got = _run_comm(2, fail_ranks=(0, 1), joined=2)
    for rank, ok, calls, comm_ranks in got:
        assert ok is True and comm_ranks == 2 and calls == []


@pytest.mark.timeout(180)
def test_init_film_comm_drops_a_stale_communicator_before_rejoining():
    """Every rank holds a communicator of another size (a stale one): it is
    destroyed first, then the ranks join afresh."""
    got = _run_comm(2, fail_ranks=(), joined=3)
    for rank, ok, calls, comm_ranks in got:
        assert ok is True and comm_ranks == 2
        assert calls == [("destroy",), ("init", 2, rank, bytes(range(128)))]
