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


# ---------------------------------------------------------------- the library's own RCCL film reduce
def test_library_rccl_film_reduce_one_rank():
    """pt_comm_unique_id + pt_comm_init_rank + pt_film_reduce on a one-rank
    communicator: the in-place ncclReduce(SUM) runs on the library's stream
    and leaves the film unchanged (the sum over one rank)."""
    from pathtracing_amd.integrator import Context
    ctx = Context(0)
    try:
        ctx.comm_init_rank(1, 0, Context.comm_unique_id())
        rng = np.random.default_rng(1)
        host = rng.uniform(-1, 1, (48, 64, 4))
        film = torch.from_numpy(host).to("cuda:0")
        torch.cuda.synchronize()
        ctx.film_reduce(film.data_ptr(), film.numel(), 0)
        np.testing.assert_array_equal(film.cpu().numpy(), host)
    finally:
        ctx.close()


@pytest.mark.parametrize("adaptive", [False, True])
def test_multi_device_context_path_on_one_gpu(monkeypatch, adaptive):
    """pt_render through render_multi (the n-GPU path of pt_create(ctx, n,
    ids): per-device host threads, device films, the grouped ncclReduce of the
    films and adaptive counts onto the first device, the copy into a host
    film) forced on a one-device context: bit-identical to the one-device
    render, host and device films, fixed SPP and adaptive."""
    from pathtracing_amd.integrator import Context
    setup = _setup()
    integ = setup.make_integrator()
    W, H = setup.camera.GetFilm().Resolution()
    cam, rd = integ.desc()
    ref = np.zeros((H, W, 4))
    base = integ.context(0)
    if adaptive:
        st0, c0 = base.render_adaptive(cam, rd, ref.ctypes.data)
    else:
        st0 = base.render(cam, rd, ref.ctypes.data)
    monkeypatch.setenv("PT_MULTI_DEVICE_PATH", "1")
    ctx = Context(devices=[0])
    try:
        ctx.upload(integ.flat)
        got = np.zeros((H, W, 4))
        dev = torch.zeros((H, W, 4), dtype=torch.float64, device="cuda:0")
        torch.cuda.synchronize()
        if adaptive:
            st1, c1 = ctx.render_adaptive(cam, rd, got.ctypes.data)
            st2, c2 = ctx.render_adaptive(cam, rd, dev.data_ptr())
            np.testing.assert_array_equal(c1, c0)
            np.testing.assert_array_equal(c2, c0)
        else:
            st1 = ctx.render(cam, rd, got.ctypes.data)
            st2 = ctx.render(cam, rd, dev.data_ptr())
        np.testing.assert_array_equal(got, ref)
        np.testing.assert_array_equal(dev.cpu().numpy(), ref)
        assert st1["n_devices"] == 1 and st1["paths"] == st0["paths"] and st1["stack_overflows"] == 0
    finally:
        ctx.close()


# ---------------------------------------------------------------- bench's nccl path at N = 1
def _nccl_worker(port, fake_polls, q):
    import torch.distributed as dist
    from pathtracing_amd.distributed import init_film_comm, render_frame

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        setup = _setup()
        integ = setup.make_integrator()
        W, H = setup.camera.GetFilm().Resolution()
        # rank 0's id, broadcast_object_list, _agree on CUDA tensors, pt_comm_init_rank
        ok = init_film_comm(integ, 0)
        ctx = integ.context(0)
        joined = ctx.comm_ranks
        film = torch.zeros((H, W, 4), dtype=torch.float64, device="cuda:0")
        st = render_frame(integ, film)
        before = film.clone()
        # the reduce on the library's own communicator; PT_COMM_FAKE_INPROGRESS
        # makes its enqueue and the first polls report ncclInProgress (what a
        # non-blocking communicator may return): waited for, not an error
        os.environ["PT_COMM_FAKE_INPROGRESS"] = str(fake_polls)
        ctx.film_reduce(film.data_ptr(), film.numel(), 0)
        torch.cuda.synchronize()
        q.put((ok, joined, st["paths"], torch.equal(film, before), film.cpu().numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(240)
@pytest.mark.parametrize("fake_polls", [0, 25])
def test_init_film_comm_over_nccl_one_rank(fake_polls):
    """bench.py's nccl path at N = 1: init_process_group("nccl", device_id=...),
    init_film_comm (id broadcast, agreement on CUDA tensors, the library's
    non-blocking communicator), render_frame into a device film, then the
    library's film reduce; the film equals the one-process render."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(_free_port(), fake_polls, q))
    p.start()
    try:
        ok, joined, paths, unchanged, film = q.get(timeout=200)
    finally:
        p.join(timeout=60)
    assert p.exitcode == 0
    assert ok is True and joined == 1 and unchanged
    setup = _setup()
    integ = setup.make_integrator()
    W, H = setup.camera.GetFilm().Resolution()
    one = torch.zeros((H, W, 4), dtype=torch.float64, device="cuda:0")
    torch.cuda.synchronize()
    st = integ.Render(film_ptr=one.data_ptr())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(film, one.cpu().numpy())
    assert paths == st["paths"] == W * H * setup.spp
