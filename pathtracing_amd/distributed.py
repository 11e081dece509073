"""Multi-GPU frames: one process per GPU, samples interleaved across ranks.

SURVEY.md §8(e): every rank holds a full scene replica and renders the samples
s ≡ rank (mod world) of every pixel with the same per-sample stream keys, so
the ranks' films sum to the single-GPU film up to summation order.  The one
exchange is a SUM reduce of the W×H×4 f64 accumulator {ΣRGB·w, Σw}
(Film.hpp:227-268) onto the destination rank over xGMI: the library's own
RCCL communicator (`init_film_comm` -> pt_comm_init_rank, pt_film_reduce)
when it has one, else torch.distributed's reduce (RCCL with the "nccl"
backend, gloo for the CPU tests).  It replaces the reference's
`atomic<double>` film merge (Film.hpp:125-132, 244-249).  (One process
driving several GPUs uses a multi-device context instead: pt_create(ctx, n,
ids) reduces inside pt_render.)
"""
from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist

# stats that are sums over ranks (the rest are per-rank timings)
_SUMMED = ("paths", "rays_closest", "rays_any", "nodes_closest", "tris_closest", "nodes_any", "tris_any",
           "shade_hits", "launches_closest", "launches_any")


def world() -> tuple[int, int]:
    """(rank, world_size) of the default process group, (0, 1) without one."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def local_samples(spp: int, rank: int, world_size: int) -> int:
    """Number of the frame's samples s in [0, spp) with s % world_size == rank."""
    return (spp - rank + world_size - 1) // world_size if spp > rank else 0


def _agree(flag: bool, device: int, group) -> bool:
    """True iff `flag` holds on every rank of the group (MIN all-reduce)."""
    t = torch.tensor([1 if flag else 0], dtype=torch.int32,
                     device=f"cuda:{device}" if dist.get_backend(group) == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(int(t.item()))


def init_film_comm(integrator, device: int, group=None) -> bool:
    """Give this rank's library context an RCCL communicator over the group's
    ranks (rank 0 draws the id, the group broadcasts it).  Returns False, with
    the reason logged, if RCCL refuses; render_frame then reduces through
    torch.distributed instead.

    Every decision is agreed before the next collective step, so no rank
    enters ncclCommInitRank while another has already given up: (1) all
    ranks already joined -> done; (2) stale or partial communicators are
    dropped (pt_comm_destroy); (3) rank 0's id is broadcast and every rank
    must hold one; (4) the collective init, itself bounded by
    PT_COMM_TIMEOUT_S inside the library (a rank whose peers never join aborts
    instead of blocking); (5) all ranks must have succeeded, else every rank
    drops its communicator and the torch.distributed reduce is used."""
    import sys
    from .integrator import Context
    rank, n = world() if group is None else (dist.get_rank(group), dist.get_world_size(group))
    ctx = integrator.context(device)
    if _agree(ctx.comm_ranks == n, device, group):
        return True
    if ctx.comm_ranks:
        ctx.comm_destroy()
    uid = None
    if rank == 0:
        try:
            uid = Context.comm_unique_id()
        except RuntimeError as e:  # N.NativeError
            print(f"[distributed] rank 0: no RCCL id ({e}); reducing through torch.distributed",
                  file=sys.stderr, flush=True)
    obj = [uid]
    dist.broadcast_object_list(obj, src=0, group=group)
    if not _agree(obj[0] is not None, device, group):
        return False
    ok = True
    try:
        ctx.comm_init_rank(n, rank, obj[0])
    except RuntimeError as e:  # N.NativeError
        print(f"[distributed] rank {rank}: library RCCL communicator unavailable ({e}); "
              "reducing through torch.distributed", file=sys.stderr, flush=True)
        ok = False
    if not _agree(ok, device, group):
        if ctx.comm_ranks:
            ctx.comm_destroy()  # a communicator some ranks built stays unusable: drop it
        return False
    return True


def render_frame(integrator, film: torch.Tensor, *, flags: int = 0, paths_in_flight: int = 0, dst: int = 0,
                 group=None, render_shard: Optional[Callable[[int, int, torch.Tensor], dict]] = None) -> dict:
    """Render this rank's sample shard of one frame into `film` and reduce it
    onto rank `dst`.

    film: float64 tensor (H, W, 4) — on this rank's GPU for RCCL; on the CPU
    for gloo.  It is overwritten (zeroed, then accumulated).
    render_shard(shard_index, shard_count, film) -> stats overrides the
    default, which is `integrator.Render` on the tensor's device memory.
    Returns this rank's stats (use `reduce_stats` for job totals).
    """
    rank, n = world() if group is None else (dist.get_rank(group), dist.get_world_size(group))
    H, W = film.shape[0], film.shape[1]
    fw, fh = integrator.camera.GetFilm().Resolution()
    if film.dtype != torch.float64 or tuple(film.shape) != (fh, fw, 4) or not film.is_contiguous():
        raise ValueError(f"film must be a contiguous float64 ({fh}, {fw}, 4) tensor, got "
                         f"{tuple(film.shape)} {film.dtype}")
    if render_shard is None:
        if film.device.type != "cuda":
            raise ValueError("the HIP renderer accumulates into device memory: pass a cuda film tensor")
        dev = film.device.index or 0
        # the library's launches go on torch's current stream of the film's
        # device, so they are ordered after zero_() and after any earlier
        # collective that wrote into the same tensor.  On torch's null stream
        # (handle 0) the library keeps its own non-blocking stream, which does
        # not wait for the null stream: synchronise it first.
        torch_stream = torch.cuda.current_stream(dev)
        ctx = integrator.context(dev)
        ctx.set_stream(torch_stream.cuda_stream)
        film.zero_()
        if torch_stream.cuda_stream == 0:
            torch_stream.synchronize()
        try:
            st = integrator.Render(device=dev, shard_index=rank, shard_count=n,
                                   film_ptr=film.data_ptr(), flags=flags, paths_in_flight=paths_in_flight)
        finally:
            ctx.set_stream(None)  # the cached context goes back to its own stream
    else:
        film.zero_()
        st = render_shard(rank, n, film)
    if n > 1:
        ctx = integrator.context(film.device.index or 0) if render_shard is None else None
        if ctx is not None and ctx.comm_ranks == n:
            # the library's RCCL communicator: in-place ncclReduce on its stream
            ctx.film_reduce(film.data_ptr(), film.numel(), dst)
        elif film.is_cuda and dist.get_backend(group) == "gloo":
            # gloo has no device reduce: sum host copies (CPU rehearsals of the
            # multi-rank path with the real device renderer)
            host = film.cpu()
            dist.reduce(host, dst=dst, op=dist.ReduceOp.SUM, group=group)
            if rank == dst:
                film.copy_(host)
        else:
            dist.reduce(film, dst=dst, op=dist.ReduceOp.SUM, group=group)
    return st


def reduce_stats(st: dict, device: torch.device, group=None) -> dict:
    """Job-wide stats: counts summed over ranks, timings max over ranks."""
    rank, n = world() if group is None else (dist.get_rank(group), dist.get_world_size(group))
    out = dict(st)
    if n == 1:
        return out
    keys = [k for k in _SUMMED if k in st]
    t = torch.tensor([float(st[k]) for k in keys], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    for k, v in zip(keys, t.tolist()):
        out[k] = int(v)
    tk = [k for k in st if k.startswith("ms_")]
    if tk:
        t = torch.tensor([float(st[k]) for k in tk], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        for k, v in zip(tk, t.tolist()):
            out[k] = v
    return out
