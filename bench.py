#!/usr/bin/env python3
"""Benchmark: Mrays/s of the HIP wavefront path tracer on a BASELINE.json config.

A step is one frame at fixed SPP (adaptive sampling off): every camera sample
of the frame traced to termination, NEE shadow rays included, and the film
gathered (+ the RCCL reduce onto rank 0 for N > 1).  One ray = one BVH query
(Scene::Intersect or Scene::IntersectPred), counted as the reference does
(SURVEY.md §8d).  Default workload = C4 (configs[3]: San-Miguel-class
procedural scene, ~10 M triangles, 1920x1080, 1024 SPP, PathIntegrator,
maxDepth 128) — BASELINE.json publishes no number, so the headline is the
largest single-GPU configuration.  Inputs (scene, BVH) are resident in HBM
before the timed region.

  python bench.py [--gpus N --steps K --warmup W --config c4|c2|c3|c1|...]

--gpus N without a torch.distributed environment starts N ranks itself
(torch.distributed.run, one process per GPU) before anything touches the GPU;
under the driver's own launcher (WORLD_SIZE set) it checks WORLD_SIZE == N.
Samples are interleaved across ranks (s % N == rank), the per-rank films are
summed onto rank 0 by the library's own RCCL communicator (pt_film_reduce;
torch.distributed's reduce if RCCL refuses it); value = all ranks' rays /
max-rank time.  Total work per frame is fixed as N grows ("scaling": "strong").
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
# configurations whose BVH + primitive slots exceed the 256 MiB Infinity Cache:
# their traversal bytes stream from HBM.  The small scenes live in L2/MALL.
HBM_CONFIGS = ("c4",)


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


def src_sha() -> str:
    """Hash of the sources libpt_hip.so is built from (csrc/ + the C ABI
    header): ties a committed counter profile to the binary being benched
    (.git does not travel to the GPU box)."""
    h = hashlib.sha256()
    files = sorted((ROOT / "pathtracing_amd" / "csrc").glob("*")) + [ROOT / "include" / "pt_api.h"]
    for p in files:
        if p.is_file():
            h.update(p.name.encode())
            h.update(p.read_bytes())
    return h.hexdigest()[:16]


def _json(path: Path):
    try:
        return json.loads(path.read_text())
    except (OSError, ValueError):
        return None


def cpu_baseline(setup, config: str, target_s: float = 15.0):
    """The oracle (CPU restatement, 'port') on the host cores, on a bounded
    sample of the same workload: full frame at a reduced SPP sized from a
    pilot run to take about target_s seconds.  The port/reference speed ratio
    measured in the build container (tools/cpu_ratio.py, where the reference
    itself compiles; it cannot travel to the GPU box) rides along."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle
    nproc = os.cpu_count() or 1
    affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    threads = max(1, min(16, affinity))
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
    value = rays / dt / 1e6
    per_core = value / threads
    out = {"value": round(value, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
           "nproc": nproc, "affinity": affinity,
           "sample": f"oracle/pt_oracle.c, same scene {W}x{H} at {spp} spp ({rays} rays in {dt:.1f} s, "
                     f"{threads} threads; the box's cpu budget is 16 threads)",
           "per_core": round(per_core, 4),
           # linear in cores: an upper bound for the whole host (memory
           # bandwidth and SMT make real scaling sub-linear)
           "full_host_estimate": {"value": round(per_core * affinity, 3), "cores": affinity,
                                  "method": "per-core rate x affinity (linear)"}}
    ratio = _json(ROOT / "profiles" / "r03_cpu_ratio.json") or _json(ROOT / "profiles" / "r02_cpu_ratio.json")
    if ratio:
        out["port_vs_reference"] = ratio.get("summary")
        # the reference's own speed on this host, estimated from the port
        # through the ratio measured on the closest scene class, at the
        # measured thread count closest to the one timed here
        key = {"c4": "c4_recipe_2pct_160x90_16spp_depth128", "c1": "c1_example1_path_256x256_16spp"}.get(
            config, "c1_example1_path_256x256_16spp")
        ent = ratio.get(key, {})
        by = ent.get("by_threads", {})
        t_used = min(by, key=lambda t: abs(int(t) - threads)) if by else str(ratio.get("_meta", {}).get("threads"))
        r = by[t_used]["port_over_reference"] if by else ent.get("port_over_reference")
        if r:
            out["reference_estimate"] = {"value": round(value / r, 3), "port_over_reference": r,
                                         "ratio_threads": int(t_used) if t_used and t_used != "None" else None,
                                         "scene_class": key}
    out["_counts"] = cnt  # traversal counts in the reference's visit order (consumed by main)
    return out


def pmc_traffic(config: str, spp: int, world: int, kernel: str, sha: str):
    """HBM bytes per launch of `kernel` from a committed rocprofv3 counter
    summary of this workload AND this build (profiles/r0*_<config>_pmc.json,
    written by tools/profile_bench.sh; `_meta.src_sha` must equal the sources
    being benched).  FETCH_SIZE is scaled by the factor calibrated on this
    kernel's own access pattern (profiles/r03_fetch_calib.json, known byte
    counts): FETCH_SIZE counts 64 B per touched 128-B line; a full-line read
    (128-B clusters, `factor_node_gather` 2.0) moves both 64-B halves, a
    64-B quantized node or a 48-B slot only its half (`factor_qnode_gather`
    1.0: 1.5x the full-line gather's line rate; HBM3E bursts are 64 B).
    WRITE_SIZE is exact for 16-B stores (MI355X_MICROARCH.md "HBM").
    Returns (bytes|None, info)."""
    import glob
    cname = "r03_fetch_calib.json" if (ROOT / "profiles" / "r03_fetch_calib.json").exists() else "r02_fetch_calib.json"
    calib = _json(ROOT / "profiles" / cname) or {}
    key = "factor_qnode_gather" if kernel.endswith(", true>") else "factor_node_gather"
    factor = calib.get(key)
    info = {"fetch_factor": factor, "fetch_factor_source": f"{cname} {key}" if factor else None}
    for path in sorted(glob.glob(str(ROOT / "profiles" / f"r*_{config}_pmc.json")), reverse=True):
        prof = _json(Path(path))
        if not prof:
            continue
        meta = prof.get("_meta", {})
        if meta.get("spp") != spp or meta.get("n_gpus", 1) != world:
            continue
        k = prof.get(kernel, {})
        if "FETCH_SIZE_per_dispatch" not in k:
            continue
        info["traffic_source"] = Path(path).name
        info["traffic_src_sha"] = meta.get("src_sha")
        if meta.get("src_sha") != sha:
            info["traffic_note"] = "newest counter profile is of another build; traffic not reported"
            return None, info
        if factor is None:
            info["traffic_note"] = "no FETCH_SIZE calibration for this access pattern"
            return None, info
        b = (factor * k["FETCH_SIZE_per_dispatch"] + k.get("WRITE_SIZE_per_dispatch", 0.0)) * 1024.0
        info["traffic_raw_fetch_kb"] = round(k["FETCH_SIZE_per_dispatch"], 1)
        return round(b), info
    info["traffic_note"] = "no counter profile of this workload"
    return None, info


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int) -> int:
    """Start n ranks of this script (one per GPU) as children; nothing in this
    process has touched the GPU."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(Path(__file__).resolve()),
           *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def log(msg: str):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c4")
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--paths-in-flight", type=int, default=0)
    ap.add_argument("--traversal", choices=("auto", "pool", "simple"), default="auto",
                    help="BVH traversal kernel (auto: by BVH size)")
    ap.add_argument("--nodes", choices=("auto", "full", "quant"), default="auto",
                    help="node layout of the pool traversal (auto: 64-B quantized nodes)")
    ap.add_argument("--sort-material", action="store_true",
                    help="shade each bounce binned by hit material (PT_RENDER_SORT_MATERIAL)")
    ap.add_argument("--sort-spatial", action="store_true",
                    help="shade each bounce binned by the hit point's cell (PT_RENDER_SORT_SPATIAL; "
                         "the library's default for large scenes)")
    ap.add_argument("--no-sort", action="store_true", help="no hit sort before shading (PT_RENDER_NO_SORT)")
    ap.add_argument("--sort-rays", action="store_true",
                    help="trace closest-hit rays in origin-cell + octant order (PT_RENDER_SORT_RAYS)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-count", action="store_true", help="skip the instrumented node-count pass")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))

    import torch
    import torch.distributed as dist
    from pathtracing_amd import native as N
    from pathtracing_amd.distributed import render_frame

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}")
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        assert dist.get_world_size() == args.gpus
    device = local if world > 1 else 0
    torch.cuda.set_device(device)

    t_setup = time.perf_counter()
    setup = build_setup(args.config, args.spp)
    integ = setup.make_integrator()
    W, H = setup.camera.GetFilm().Resolution()
    film = torch.zeros((H, W, 4), dtype=torch.float64, device=f"cuda:{device}")
    integ.context(device)  # scene upload
    torch.cuda.synchronize(device)
    setup_s = time.perf_counter() - t_setup
    film_reduce = None
    if world > 1:  # the film reduce through the library's own RCCL communicator
        from pathtracing_amd.distributed import init_film_comm
        film_reduce = ("pt_film_reduce (library RCCL communicator)" if init_film_comm(integ, device)
                       else "torch.distributed.reduce (RCCL)")
    if rank == 0:
        log(f"{args.config}: scene + BVH + upload {setup_s:.1f} s, {world} rank(s)")

    tflag = {"auto": 0, "pool": N.PT_RENDER_TRAVERSAL_POOL, "simple": N.PT_RENDER_TRAVERSAL_SIMPLE}[args.traversal]
    tflag |= {"auto": 0, "full": N.PT_RENDER_NODES_FULL, "quant": N.PT_RENDER_NODES_QUANTIZED}[args.nodes]
    if args.sort_material:
        tflag |= N.PT_RENDER_SORT_MATERIAL
    if args.sort_spatial:
        tflag |= N.PT_RENDER_SORT_SPATIAL
    if args.no_sort:
        tflag |= N.PT_RENDER_NO_SORT
    if args.sort_rays:
        tflag |= N.PT_RENDER_SORT_RAYS

    def step(flags=0):
        # this rank's sample shard into the device film, then the RCCL SUM
        # reduce of the film onto rank 0 (pathtracing_amd/distributed.py)
        return render_frame(integ, film, flags=flags | tflag, paths_in_flight=args.paths_in_flight)

    for i in range(args.warmup):
        t0 = time.perf_counter()
        step()
        if rank == 0:
            log(f"warmup {i + 1}/{args.warmup}: {time.perf_counter() - t0:.2f} s")
    # traversal work per ray (untimed, instrumented pass over the first spp/16
    # samples of every pixel: same scene, same sample stream)
    bytes_closest = bytes_any = None
    cst = {}
    if not args.no_count:
        count_spp = max(1, setup.spp // 16)
        integ.sampler.samples = count_spp
        cst = step(N.PT_RENDER_COUNT_NODES)
        integ.sampler.samples = setup.spp
        bytes_closest = (128.0 * cst["nodes_closest"] + 48.0 * cst["tris_closest"]) / max(1, cst["rays_closest"])
        if cst["rays_any"]:
            bytes_any = (128.0 * cst["nodes_any"] + 48.0 * cst["tris_any"]) / cst["rays_any"]

    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    totals = {"rays_closest": 0, "rays_any": 0, "ms_closest": 0.0, "ms_any": 0.0, "ms_shade": 0.0,
              "launches_closest": 0, "launches_any": 0, "paths": 0}
    for i in range(args.steps):
        ts = time.perf_counter()
        st = step(N.PT_RENDER_TIMING)
        for k in totals:
            totals[k] += st[k]
        if rank == 0:
            log(f"step {i + 1}/{args.steps}: {time.perf_counter() - ts:.2f} s")
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

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(setup, args.config, args.cpu_seconds)
    if rank == 0:
        pool = args.traversal == "pool" or (args.traversal == "auto" and args.config in HBM_CONFIGS)
        quant = pool and args.nodes != "full"
        q = ", true" if quant else ", false"
        kname = f"k_closest_pool<false, false{q}>" if pool else "k_closest<false, false>"
        sname = f"k_shadow_pool<false, false{q}>" if pool else "k_shadow<false, false>"
        node_bytes = 64.0 if quant else 128.0  # what this kernel's node step reads
        sha = src_sha()

        def kernel_roof(name, bpr, lbpr, ms, launches, nrays):
            # bpr: SURVEY §8(d) algorithmic bytes per ray (128 B per node visit,
            # 48 B per primitive test: the reference's layout); lbpr: the
            # bytes this kernel's layout reads for the same visits
            avg_ms = ms / max(1, launches)
            if bpr is None or avg_ms <= 0:
                return None
            launch_bytes = bpr * nrays / max(1, launches)
            achieved = launch_bytes / (avg_ms * 1e-3) / 1e9
            layout = lbpr * nrays / max(1, launches) / (avg_ms * 1e-3) / 1e9 if lbpr else None
            return {"kernel": name, "achieved": round(achieved, 1), "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "bytes_per_ray": round(bpr, 1), "bytes_per_launch": round(launch_bytes),
                    "layout_bytes_per_ray": round(lbpr, 1) if lbpr else None,
                    "layout_achieved": round(layout, 1) if layout else None,
                    "layout_frac": round(layout / HBM_PEAK_GBS, 4) if layout else None,
                    "avg_launch_ms": round(avg_ms, 4), "launches": launches}

        # the algorithmic bytes come from the reference's own
        # visit order (the oracle's BVH4::Intersect / IntersectPred restatement,
        # entry-distance cull included) over the cpu_baseline sample of the
        # same frame; the GPU's instrumented count rides beside it (and stands
        # in when no CPU sample ran, e.g. N > 1)
        ref_counts = cpu.pop("_counts") if cpu else None
        count_source = "gpu"
        if ref_counts and ref_counts["closest"]:
            bytes_closest = (128.0 * ref_counts["nodes_closest"] + 48.0 * ref_counts["tris_closest"]) / \
                ref_counts["closest"]
            if ref_counts["any"]:
                bytes_any = (128.0 * ref_counts["nodes_any"] + 48.0 * ref_counts["tris_any"]) / ref_counts["any"]
            count_source = f"oracle reference order ({ref_counts['closest']} closest / {ref_counts['any']} any rays)"
        lb_closest = lb_any = None
        if cst:
            lb_closest = (node_bytes * cst["nodes_closest"] + 48.0 * cst["tris_closest"]) / max(1, cst["rays_closest"])
            if cst["rays_any"]:
                lb_any = (node_bytes * cst["nodes_any"] + 48.0 * cst["tris_any"]) / cst["rays_any"]

        rc = kernel_roof(kname, bytes_closest, lb_closest, totals["ms_closest"], totals["launches_closest"],
                         totals["rays_closest"])
        ra = kernel_roof(sname, bytes_any, lb_any, totals["ms_any"], totals["launches_any"], totals["rays_any"])
        traffic, tinfo = pmc_traffic(args.config, setup.spp, world, kname, sha)
        roof = {"bound": "hbm" if args.config in HBM_CONFIGS else "l2/latency",
                "achieved": rc["achieved"] if rc else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": rc["frac"] if rc else None, "traffic": traffic,
                "traffic_frac": (round(traffic / (rc["avg_launch_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                                 if traffic and rc else None),
                "src_sha": sha, **tinfo}
        if rc:
            def per(c, k, n):
                return round(c[k] / max(1, c[n]), 2) if c else None
            roof.update({"kernel": kname, "bytes_per_ray": rc["bytes_per_ray"], "count_source": count_source,
                         "nodes_per_ray": per(ref_counts, "nodes_closest", "closest") if ref_counts
                         else per(cst, "nodes_closest", "rays_closest"),
                         "tris_per_ray": per(ref_counts, "tris_closest", "closest") if ref_counts
                         else per(cst, "tris_closest", "rays_closest"),
                         "gpu_nodes_per_ray": per(cst, "nodes_closest", "rays_closest"),
                         "gpu_tris_per_ray": per(cst, "tris_closest", "rays_closest"),
                         "gpu_order_frac": (round(rc["frac"] * (128.0 * cst["nodes_closest"] + 48.0 *
                                                               cst["tris_closest"]) / max(1, cst["rays_closest"])
                                                  / rc["bytes_per_ray"], 4) if cst else None),
                         "avg_launch_ms": rc["avg_launch_ms"], "launches": rc["launches"],
                         "bytes_per_launch": rc["bytes_per_launch"], "node_layout_bytes": node_bytes,
                         "layout_bytes_per_ray": rc["layout_bytes_per_ray"],
                         "layout_achieved": rc["layout_achieved"], "layout_frac": rc["layout_frac"]})
        if ra:
            ra["nodes_per_ray"] = (round(ref_counts["nodes_any"] / max(1, ref_counts["any"]), 2) if ref_counts
                                   else round(cst["nodes_any"] / max(1, cst["rays_any"]), 2))
            ra["tris_per_ray"] = (round(ref_counts["tris_any"] / max(1, ref_counts["any"]), 2) if ref_counts
                                  else round(cst["tris_any"] / max(1, cst["rays_any"]), 2))
            if cst:
                ra["gpu_nodes_per_ray"] = round(cst["nodes_any"] / max(1, cst["rays_any"]), 2)
                ra["gpu_tris_per_ray"] = round(cst["tris_any"] / max(1, cst["rays_any"]), 2)
                # the same 128 B / 48 B pricing over the visits this kernel makes
                gb = (128.0 * cst["nodes_any"] + 48.0 * cst["tris_any"]) / max(1, cst["rays_any"])
                ra["gpu_order_frac"] = round(ra["frac"] * gb / ra["bytes_per_ray"], 4)
                if ra["frac"] > 1.0:
                    ra["note"] = ("frac above 1: the reference's slot order (BVH.hpp:1099-1102) visits more "
                                  "nodes than this kernel's octant order; gpu_order_frac prices the visits it makes")
            roof["shadow"] = ra
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
                       "rays_per_step": int(total_rays / args.steps), "parallelism": f"sample-shard x{world}",
                       "world_size": dist.get_world_size() if world > 1 else 1,
                       "film_reduce": film_reduce,
                       "setup_s": round(setup_s, 1)},
            # rank 0's per-frame kernel time by class (HIP events on the library's stream)
            "kernel_ms_per_step": {k[3:]: round(totals[k] / args.steps, 1)
                                   for k in ("ms_closest", "ms_any", "ms_shade")},
            "roofline": roof,
        }
        if cpu:
            v = out["value"]
            cpu["gpu_over_cpu"] = round(v / cpu["value"], 1)
            cpu["gpu_over_full_host_estimate"] = round(v / cpu["full_host_estimate"]["value"], 1)
            out["cpu_baseline"] = cpu
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
