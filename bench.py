#!/usr/bin/env python3
"""Benchmark: Mrays/s of the HIP wavefront path tracer on a BASELINE.json config.

A step is one frame at fixed SPP (adaptive sampling off): every camera sample
of the frame traced to termination, NEE shadow rays included, and the film
gathered (+ the RCCL reduce onto rank 0 for N > 1).  One ray = one BVH query
(Scene::Intersect or Scene::IntersectPred), counted as the reference does
(SURVEY.md §8d).  Default workload = configs[1] (C2: Cornell box, 1024x1024,
256 SPP, SimplePath, maxDepth 8).  Inputs (scene, BVH) are resident in HBM
before the timed region.

  python bench.py [--gpus N --steps K --warmup W --config c2|c3|c1|c4]

For N > 1 the driver launches one rank per GPU (torch.distributed, RCCL);
samples are interleaved across ranks (s % N == rank), the per-rank films are
summed onto rank 0 with dist.reduce; value = all ranks' rays / max-rank time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)


def build_setup(config: str, spp: int | None = None):
    from pathtracing_amd import scenes
    if config == "c1":
        return scenes.example_1(W=256, H=256, spp=spp or 16)
    if config == "c2":
        return scenes.cornell(W=1024, H=1024, spp=spp or 256, config="c2")
    if config == "c3":
        return scenes.cornell(W=1024, H=1024, spp=spp or 256, config="c3")
    if config == "c4":
        return scenes.sanmiguel(W=1920, H=1080, spp=spp or 1024)
    if config == "c1v":  # examples/example_1.cpp's VolPathIntegrator frame, at C2's size
        return scenes.example_1(W=1024, H=1024, spp=spp or 256, integrator="volpath", max_depth=8,
                                seed=0x5EED0021)
    if config == "fog":  # C3 box in fog, VolPathIntegrator
        return scenes.cornell(W=1024, H=1024, spp=spp or 256, fog=True)
    if config == "inst":  # instancing: C2 room + instanced meshes / shapes (TransformedPrimitive)
        return scenes.instances(W=1024, H=1024, spp=spp or 256)
    if config.startswith("hf"):  # heightfield probe, e.g. hf1000 = 2M triangles
        return scenes.heightfield(n=int(config[2:]), W=1024, H=1024, spp=spp or 16)
    raise ValueError(config)


WORKLOADS = {
    "c1": "C1 examples/example_1 scene 256x256 16spp depth 8 PathIntegrator",
    "c2": "C2 Cornell box (34 tris + quad light) 1024x1024 256spp depth 8 SimplePathIntegrator, Lambertian",
    "c3": "C3 Cornell box + GGX dielectric/conductor 1024x1024 256spp depth 8 PathIntegrator NEE+MIS+RR",
    "c4": "C4 San-Miguel-class procedural ~10M tris 1920x1080 1024spp depth 128 PathIntegrator",
    "c1v": "C1 examples/example_1 scene (HG medium sphere) 1024x1024 256spp depth 8 VolPathIntegrator",
    "fog": "C3 Cornell box in a homogeneous fog (scene+camera medium, emissive medium, point light) "
           "1024x1024 256spp depth 8 VolPathIntegrator",
    "inst": "C2 room + 3 instanced glossy meshes, instanced glass sphere / metal quad, animated sphere "
            "(TransformedPrimitive / AnimatedPrimitive) 1024x1024 256spp depth 8 PathIntegrator",
}


def cpu_baseline(setup, target_s: float = 15.0):
    """The oracle (CPU restatement, 'port') on the host cores, on a bounded
    sample of the same workload: full frame at a reduced SPP sized from a
    pilot run to take about target_s seconds."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle
    threads = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()))
    integ = setup.make_integrator()
    W, H = setup.camera.GetFilm().Resolution()
    t0 = time.perf_counter()
    _, cnt = oracle.render(integ, threads=threads, spp=1)
    pilot = time.perf_counter() - t0
    spp = max(1, min(setup.spp, int(target_s / max(pilot, 1e-3))))
    if spp > 1:
        t0 = time.perf_counter()
        _, cnt = oracle.render(integ, threads=threads, spp=spp)
        dt = time.perf_counter() - t0
    else:
        dt = pilot
    rays = cnt["closest"] + cnt["any"]
    return {"value": round(rays / dt / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"oracle/pt_oracle.c, same scene {W}x{H} at {spp} spp ({rays} rays in {dt:.1f} s, "
                      f"{threads} threads)"}


def pmc_traffic(config: str, spp: int, world: int):
    """HBM bytes per k_closest launch from the committed rocprofv3 counter
    summary of this workload (tools/profile_pmc.sh + tools/pmc_summary.py,
    profiles/*_<config>_pmc.json): FETCH_SIZE doubled (gfx950 reports half
    of 16-byte-per-lane reads, MI355X_MICROARCH.md "HBM") + WRITE_SIZE, both
    in KB per dispatch.  None when no profile of this configuration exists."""
    import glob
    cands = sorted(glob.glob(str(ROOT / "profiles" / f"*_{config}_pmc.json")))
    for path in reversed(cands):
        try:
            prof = json.load(open(path))
        except (OSError, ValueError):
            continue
        meta = prof.get("_meta", {})
        if meta.get("spp") != spp or meta.get("n_gpus", 1) != world:
            continue
        k = prof.get(meta.get("kernel", "k_closest<false>"), {})
        if "FETCH_SIZE_per_dispatch" not in k:
            continue
        b = (2.0 * k["FETCH_SIZE_per_dispatch"] + k.get("WRITE_SIZE_per_dispatch", 0.0)) * 1024.0
        return round(b), Path(path).name
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--paths-in-flight", type=int, default=0)
    ap.add_argument("--traversal", choices=("auto", "pool", "simple"), default="auto",
                    help="BVH traversal kernel (auto: by BVH size)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from pathtracing_amd import native as N
    from pathtracing_amd.distributed import render_frame

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = local if world > 1 else 0
    torch.cuda.set_device(device)

    setup = build_setup(args.config, args.spp)
    integ = setup.make_integrator()
    W, H = setup.camera.GetFilm().Resolution()
    film = torch.zeros((H, W, 4), dtype=torch.float64, device=f"cuda:{device}")
    ctx = integ.context(device)
    ctx.set_stream(torch.cuda.current_stream(device).cuda_stream)

    tflag = {"auto": 0, "pool": N.PT_RENDER_TRAVERSAL_POOL, "simple": N.PT_RENDER_TRAVERSAL_SIMPLE}[args.traversal]

    def step(flags=0):
        # this rank's sample shard into the device film, then the RCCL SUM
        # reduce of the film onto rank 0 (pathtracing_amd/distributed.py)
        return render_frame(integ, film, flags=flags | tflag, paths_in_flight=args.paths_in_flight)

    for _ in range(args.warmup):
        step()
    # traversal work per closest-hit ray (untimed, instrumented pass over the
    # first spp/16 samples of every pixel: same scene, same sample stream)
    count_spp = max(1, setup.spp // 16)
    integ.sampler.samples = count_spp
    cst = step(N.PT_RENDER_COUNT_NODES)
    integ.sampler.samples = setup.spp
    nodes_per_ray = cst["nodes_closest"] / max(1, cst["rays_closest"])
    tris_per_ray = cst["tris_closest"] / max(1, cst["rays_closest"])
    bytes_per_ray = 128.0 * nodes_per_ray + 48.0 * tris_per_ray

    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    totals = {"rays_closest": 0, "rays_any": 0, "ms_closest": 0.0, "launches_closest": 0, "paths": 0}
    for _ in range(args.steps):
        st = step(N.PT_RENDER_TIMING)
        for k in totals:
            totals[k] += st[k]
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{device}")
    rays = torch.tensor([float(totals["rays_closest"] + totals["rays_any"])], dtype=torch.float64,
                        device=f"cuda:{device}")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(rays, op=dist.ReduceOp.SUM)
    elapsed_max = float(t.item())
    total_rays = float(rays.item())

    if rank == 0:
        avg_ms = totals["ms_closest"] / max(1, totals["launches_closest"])
        launch_bytes = bytes_per_ray * totals["rays_closest"] / max(1, totals["launches_closest"])
        achieved = launch_bytes / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
        traffic, traffic_src = pmc_traffic(args.config, setup.spp, world)
        out = {
            "metric": "Mrays/s",
            "value": round(total_rays / elapsed_max / 1e6, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed_max / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": WORKLOADS.get(args.config, args.config), "width": W, "height": H,
                       "spp": setup.spp, "max_depth": setup.max_depth, "integrator": setup.integrator,
                       "rays_per_step": int(total_rays / args.steps), "parallelism": f"sample-shard x{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": "k_closest (BVH4 closest-hit traversal)",
                         "bytes_per_ray": round(bytes_per_ray, 1), "nodes_per_ray": round(nodes_per_ray, 2),
                         "tris_per_ray": round(tris_per_ray, 2), "avg_launch_ms": round(avg_ms, 4),
                         "launches": totals["launches_closest"]},
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(build_setup(args.config, args.spp), args.cpu_seconds)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
