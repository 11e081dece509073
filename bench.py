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
MI355X_CUS = 256
CLOCK_GHZ = 2.4  # the engine clock GRBM_GUI_ACTIVE shows under load


def gather_ceiling(pattern: str = "P3", level: str = "L2") -> dict:
    """The measured ceiling of the traversal's access pattern: a dependent
    random gather per lane, three 16-B loads of one 48-B record per step (P3,
    the PT_Q48 node / slot read), on an L2-resident table -- tools/gather_rate.hip
    on one MI355X, committed as profiles/r05_gather_rate.json.  The vector
    memory pipe takes about one lane address per clock per CU whatever the
    occupancy; in GB/s at 16 B per lane-load."""
    path = ROOT / "profiles" / "r05_gather_rate.json"
    prof = json.loads(path.read_text()) if path.exists() else {}
    rates = [r["lane_loads_per_clk_cu"] for r in prof.get("rows", [])
             if r.get("pattern") == pattern and r.get("level") == level]
    if not rates:
        return {}
    lpc = max(rates)
    return {"pattern": f"{pattern} {level}", "lane_loads_per_clk_cu": lpc,
            "gbs_at_16B": round(lpc * 16 * MI355X_CUS * CLOCK_GHZ, 1), "source": "profiles/r05_gather_rate.json"}


# the chip-wide ceiling of a kernel whose reads are L2 hits (its "l2-latency"
# bound): the measured gather rate of the traversal's own access pattern
L2_GATHER_PEAK_GBS = (lambda g: g.get("gbs_at_16B") or 14150.0)(gather_ceiling())
# configurations whose BVH + primitive slots exceed the 256 MiB Infinity Cache:
# their traversal bytes stream from HBM.  The small scenes live in L2/MALL.
HBM_CONFIGS = ("c4",)
# bytes a node step reads: the PT_Q48 record (the default pool traversal,
# pt_device.h), the 64-B quantized node (PT_Q48=0 builds), the reference's
# 128-B cluster (full nodes)
NODE_BYTES = {"q48": 48.0, "q64": 64.0, "full": 128.0}


def build_setup(config: str, spp: int | None = None, res: str | None = None):
    from pathtracing_amd import scenes
    if res:  # tests only: the same scene at another film size
        import inspect
        w, h = (int(v) for v in res.lower().split("x"))
        orig = {"c1": scenes.example_1, "c2": scenes.cornell, "c3": scenes.cornell, "c4": scenes.sanmiguel}
        fn = orig.get(config)
        if fn is None or "W" not in inspect.signature(fn).parameters:
            raise SystemExit(f"bench: --res is not supported for {config}")
        kw = {"W": w, "H": h, "spp": spp or 4}
        if config in ("c2", "c3"):
            kw["config"] = config
        return fn(**kw)
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
    ratio = (_json(ROOT / "profiles" / "r06_cpu_ratio.json") or _json(ROOT / "profiles" / "r03_cpu_ratio.json") or
             _json(ROOT / "profiles" / "r02_cpu_ratio.json"))
    if ratio:
        out["port_vs_reference"] = ratio.get("summary")
        # the reference's own speed on this host, estimated from the port
        # through the ratio measured on the closest scene class, at the
        # measured thread count closest to the one timed here
        # C4: the full-detail scene itself (r06; the 2 %-detail recipe before)
        key = {"c4": "c4_full_192x108_32spp_depth128", "c1": "c1_example1_path_256x256_16spp"}.get(
            config, "c1_example1_path_256x256_16spp")
        if key not in ratio:
            key = {"c4": "c4_recipe_2pct_160x90_16spp_depth128"}.get(config, "c1_example1_path_256x256_16spp")
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
    # k_shade's gathers (slots, texel rows, path state) move 64-B halves like
    # the quantized nodes: FETCH_SIZE counts each touched half once (x 1.0)
    key = ("factor_qnode_gather" if kernel.startswith("k_shade") or kernel.endswith(", true>")
           else "factor_node_gather")
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
        # what bounds the kernel besides bytes: the share of wave cycles spent
        # waiting on memory and the L2 hit rate of the same profile
        if k.get("SQ_WAVE_CYCLES_per_dispatch"):
            wc = k["SQ_WAVE_CYCLES_per_dispatch"]
            info["wait_ratio"] = round(k["SQ_WAIT_ANY_per_dispatch"] / wc, 3)
            # issue-stalled (an instruction ready but not issued) and active shares
            if k.get("SQ_WAIT_INST_ANY_per_dispatch") is not None:
                info["issue_stall_ratio"] = round(k["SQ_WAIT_INST_ANY_per_dispatch"] / wc, 3)
            if k.get("SQ_ACTIVE_INST_ANY_per_dispatch") is not None:
                info["active_ratio"] = round(k["SQ_ACTIVE_INST_ANY_per_dispatch"] / wc, 3)
            # resident waves per SIMD, time-averaged over the launch: the wave
            # quad-cycles (SQ_WAVE_CYCLES counts quad-cycles, MI355X_MICROARCH.md
            # "SQ PMC units") x 4 over the launch's cycles x 1024 SIMDs, the
            # launch's cycles being SQ_BUSY_CYCLES over its 32 SQ instances
            # (8 XCDs x 4 shader engines; = avg_us x 2.4 GHz within 2 %)
            if k.get("SQ_BUSY_CYCLES_per_dispatch"):
                info["waves_per_simd"] = round(4.0 * wc * 32.0 / (k["SQ_BUSY_CYCLES_per_dispatch"] * 4.0 * MI355X_CUS), 2)
        hits, miss = k.get("TCC_HIT_sum_per_dispatch"), k.get("TCC_MISS_sum_per_dispatch")
        if hits is not None and miss is not None and hits + miss > 0:
            info["l2_hit_rate"] = round(hits / (hits + miss), 3)
        if k.get("avg_us"):
            info["profile_avg_launch_ms"] = round(k["avg_us"] / 1e3, 3)
            if k.get("SQ_INSTS_VMEM_RD_per_dispatch"):
                # issued vector-memory lane addresses per clock per CU (every
                # lane of each wave instruction counted)
                clk = k["avg_us"] * 1e-6 * CLOCK_GHZ * 1e9 * MI355X_CUS
                info["issued_lane_loads_per_clk_cu"] = round(64.0 * k["SQ_INSTS_VMEM_RD_per_dispatch"] / clk, 3)
                info["vmem_rd_insts_per_dispatch"] = round(k["SQ_INSTS_VMEM_RD_per_dispatch"])
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


def _shard_arg(v: str | None):
    if not v:
        return None
    i, _, n = v.partition("/")
    i, n = int(i), int(n)
    if not (n >= 1 and 0 <= i < n):
        raise SystemExit(f"bench: bad --shard {v} (want I/N with 0 <= I < N)")
    return i, n


def _load_hook(path: str):
    """--render-hook: a Python file (test infrastructure, e.g. tests/bench_cpu_hook.py)
    defining render_shard(setup, shard_index, shard_count, film) -> stats and
    optionally frame_samples(setup, pixels, samples) -> (n, 3) float32.  It
    stands in for the HIP library so the CPU suite can drive this script's
    multi-rank path end to end over gloo; its numbers are not GPU numbers."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_render_hook", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _nonfinite_vs_oracle(setup, integ, film, frame_samples, sample_range, oracle, max_pixels: int = 64) -> dict:
    """The film's non-finite pixels traced to their samples.  Every sample of
    every pixel within the filter radius of each non-finite pixel is read back
    from the frame's sample buffer; each non-finite one must be non-finite in
    the same channels (and equal in the others) in the oracle's Li -- the
    reference itself produces it.  explained: the sample buffer holds the
    whole frame (a multi-chunk frame keeps only its last chunk, so a NaN could
    come from a sample no longer there: not explained), at most max_pixels
    pixels are non-finite, every one of them has a non-finite sample in its
    footprint, and every non-finite sample in every footprint is the oracle's."""
    import numpy as np
    W, H = setup.camera.GetFilm().Resolution()
    f = film.detach().cpu().numpy()
    bad = np.argwhere(~np.isfinite(f).all(-1))
    lo, hi = sample_range if sample_range is not None else (0, setup.spp - 1)
    whole = lo == 0 and hi >= setup.spp - 1
    smp = np.arange(lo, hi + 1, dtype=np.uint32)
    rad = int(np.ceil(float(np.max(setup.camera.GetFilm().filter.radius)) - 0.5))
    checked, matched, seen, explained = 0, 0, {}, 0
    for y, x in bad[:max_pixels]:
        found, all_ok = False, True
        for yy in range(max(0, y - rad), min(H, y + rad + 1)):
            for xx in range(max(0, x - rad), min(W, x + rad + 1)):
                p = yy * W + xx
                if p not in seen:
                    L = np.asarray(frame_samples(np.full(smp.shape, p, np.uint32), smp), np.float32).reshape(-1, 3)
                    nf = np.nonzero(~np.isfinite(L).all(1))[0]  # every non-finite sample of the pixel
                    ok_p = True
                    if nf.size:
                        want, _ = oracle.li_pairs(integ, np.full(nf.size, p, np.uint32), smp[nf])
                        want = np.asarray(want, np.float32).reshape(-1, 3)
                        same = (np.isfinite(L[nf]) == np.isfinite(want)).all(1) & \
                               np.where(np.isfinite(want), L[nf] == want, True).all(1)
                        checked += int(nf.size)
                        matched += int(same.sum())
                        ok_p = bool(same.all())
                    seen[p] = (int(nf.size), ok_p)
                found = found or seen[p][0] > 0
                all_ok = all_ok and seen[p][1]
        explained += int(found and all_ok)
    n = int(min(bad.shape[0], max_pixels))
    return {"pixels": int(bad.shape[0]), "pixels_checked": n, "pixels_explained": explained,
            "samples_checked": checked, "samples_as_oracle": matched, "whole_frame_in_buffer": bool(whole),
            "explained": bool(whole and 0 < bad.shape[0] <= max_pixels and explained == n and checked == matched)}


def verify_frame(setup, integ, rank: int, world: int, pairs: int, frame_samples, film=None, seed: int = 0x5EED0B0C,
                 sample_range=None, overflows=None):
    """Untimed check of the frame just timed: per-sample Li of
    `pairs` (pixel, sample) pairs read back from the frame's own sample buffer
    (pt_frame_samples) must equal the oracle's Li bit for bit; half the pairs
    take the shard's highest sample indices (the top of the 31-bit sample-id
    range of the frame); and the film (rank 0, after the reduce) must be
    finite with a positive filter weight on every pixel.  The oracle is the
    checker here, never the thing timed.  sample_range = (first, last): the
    frame samples the sample buffer still holds (its last chunk,
    pt_frame_sample_range); the pairs are drawn from those.  overflows: the
    timed steps' summed pt_stats stack_overflows / tie_overflows, both 0 for
    a frame whose traversal dropped nothing."""
    import numpy as np
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle
    W, H = setup.camera.GetFilm().Resolution()
    spp = setup.spp
    local = list(range(rank, spp, world))
    if sample_range is not None:
        local = [s for s in local if sample_range[0] <= s <= sample_range[1]]
    out = {"pairs": 0, "bit_exact": 0}
    if pairs > 0 and local:
        rng = np.random.default_rng(seed + rank)
        half = max(1, pairs // 2)
        pix = rng.integers(0, W * H, size=2 * half, dtype=np.int64).astype(np.uint32)
        lo = rng.choice(local, size=half)
        hi = np.asarray(local[-min(len(local), 8):])[rng.integers(0, min(len(local), 8), size=half)]
        smp = np.concatenate([lo, hi]).astype(np.uint32)
        t0 = time.perf_counter()
        got = np.asarray(frame_samples(pix, smp), np.float32).reshape(-1, 3)
        want, _ = oracle.li_pairs(integ, pix, smp)
        same = np.all(got.view(np.uint32) == want.view(np.uint32), axis=1)
        bad = np.nonzero(~same)[0]
        out.update({"pairs": int(pix.size), "bit_exact": int(same.sum()), "max_sample": int(smp.max()),
                    "check_s": round(time.perf_counter() - t0, 2),
                    "mismatches": [{"pixel": int(pix[k]), "sample": int(smp[k]), "got": got[k].tolist(),
                                    "want": want[k].tolist()} for k in bad[:4]]})
    ok = out["pairs"] == out["bit_exact"]
    if overflows is not None:
        out.update({k: int(v) for k, v in overflows.items()})
        ok = ok and not any(overflows.values())
    if film is not None:
        import torch
        out["film_finite"] = bool(torch.isfinite(film).all().item())
        out["film_weight_positive"] = bool((film[..., 3] > 0).all().item())
        film_ok = out["film_finite"]
        if not film_ok:
            # a non-finite pixel is accepted when it is the reference's own:
            # every such pixel lies within the filter footprint of a pixel
            # whose non-finite samples the oracle returns non-finite too
            out["nonfinite"] = _nonfinite_vs_oracle(setup, integ, film, frame_samples, sample_range, oracle)
            film_ok = out["nonfinite"]["explained"]
        ok = ok and film_ok and out["film_weight_positive"]
    out["ok"] = bool(ok)
    out["method"] = ("per-sample Li of the timed frame (pt_frame_samples) vs the oracle, bit-exact; "
                     "no traversal stack push or exact-tie entry dropped in the timed steps; "
                     "film finite with sum w > 0 on every pixel, a non-finite pixel only where every "
                     "non-finite sample in its footprint is the oracle's too")
    return out


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
    ap.add_argument("--any-stackless", action="store_true",
                    help="NEE any-hit rays through the stackless traversal (PT_RENDER_ANY_STACKLESS)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-count", action="store_true", help="skip the instrumented node-count pass")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--shard", default=None,
                    help="I/N: time only rank I's sample shard of an N-GPU frame on this one GPU (no reduce): "
                         "the per-rank work of the N-GPU run")
    ap.add_argument("--bvh", choices=("auto", "host", "device"), default="auto",
                    help="BVH build of the scene (auto: device build, byte-identical, for >= 1 M primitives)")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="torch.distributed backend for N > 1 (gloo: CPU rehearsal with --render-hook)")
    ap.add_argument("--render-hook", default=None, help="test only: CPU stand-in renderer (see _load_hook)")
    ap.add_argument("--save-film", default=None, help="rank 0 writes the reduced film (.npy)")
    ap.add_argument("--no-verify", action="store_true", help="skip the untimed check of the timed frame")
    ap.add_argument("--verify-pairs", type=int, default=1024)
    ap.add_argument("--res", default=None, help="tests only: WxH film of the same scene")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))

    import torch
    import torch.distributed as dist
    from pathtracing_amd import flatten
    from pathtracing_amd import native as N
    from pathtracing_amd.distributed import render_frame

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}")
    shard = _shard_arg(args.shard)
    if shard and world > 1:
        raise SystemExit("bench: --shard emulates one rank on one GPU (--gpus 1)")
    hook = _load_hook(args.render_hook) if args.render_hook else None
    if hook is None and args.backend != "nccl":
        raise SystemExit("bench: --backend gloo needs --render-hook (the HIP films live in device memory)")
    cpu_run = hook is not None
    if world > 1:
        if cpu_run:
            dist.init_process_group(args.backend)
        else:
            torch.cuda.set_device(local)
            dist.init_process_group(args.backend, device_id=torch.device("cuda", local))
        assert dist.get_world_size() == args.gpus
    device = local if world > 1 else 0
    dev = torch.device("cpu") if cpu_run else torch.device("cuda", device)
    if not cpu_run:
        torch.cuda.set_device(device)

    def sync():
        if not cpu_run:
            torch.cuda.synchronize(device)

    # large BVHs build on this rank's GPU (byte-identical to the host build,
    # ~60x faster): every rank builds its own replica without sharing the
    # host's cores with the other ranks
    if not cpu_run and args.bvh != "host":
        flatten.set_bvh_device(device, min_prims=0 if args.bvh == "device" else 1 << 20)
    t_setup = time.perf_counter()
    setup = build_setup(args.config, args.spp, args.res)
    integ = setup.make_integrator()
    W, H = setup.camera.GetFilm().Resolution()
    film = torch.zeros((H, W, 4), dtype=torch.float64, device=dev)
    if not cpu_run:
        integ.context(device)  # scene upload
    sync()
    setup_s = time.perf_counter() - t_setup
    bvh_build = flatten.last_bvh_build()
    film_reduce = None
    if world > 1 and not cpu_run:  # the film reduce through the library's own RCCL communicator
        from pathtracing_amd.distributed import init_film_comm
        film_reduce = ("pt_film_reduce (library RCCL communicator)" if init_film_comm(integ, device)
                       else "torch.distributed.reduce (RCCL)")
    elif world > 1:
        film_reduce = f"torch.distributed.reduce ({args.backend}, CPU rehearsal)"
    if rank == 0:
        log(f"{args.config}: scene + BVH ({bvh_build}) + upload {setup_s:.1f} s, {world} rank(s)"
            + (f", emulating shard {shard[0]}/{shard[1]}" if shard else ""))

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
    if args.any_stackless:
        tflag |= N.PT_RENDER_ANY_STACKLESS

    def step(flags=0):
        # this rank's sample shard into the film, then the SUM reduce of the
        # film onto rank 0 (pathtracing_amd/distributed.py)
        if shard:  # one emulated rank of an N-GPU frame: its shard, no reduce
            film.zero_()
            ctx = integ.context(device)
            ctx.set_stream(torch.cuda.current_stream(device).cuda_stream)
            try:
                return integ.Render(device=device, shard_index=shard[0], shard_count=shard[1],
                                    film_ptr=film.data_ptr(), flags=flags | tflag,
                                    paths_in_flight=args.paths_in_flight)
            finally:
                ctx.set_stream(None)
        if cpu_run:
            return render_frame(integ, film, render_shard=lambda i, n, f: hook.render_shard(setup, i, n, f))
        return render_frame(integ, film, flags=flags | tflag, paths_in_flight=args.paths_in_flight)

    for i in range(args.warmup):
        t0 = time.perf_counter()
        step()
        if rank == 0:
            log(f"warmup {i + 1}/{args.warmup}: {time.perf_counter() - t0:.2f} s")
    # traversal work per ray (untimed, instrumented pass over the first spp/16
    # samples of every pixel: same scene, same sample stream)
    cst = {}
    if not args.no_count and not cpu_run:
        count_spp = max(1, setup.spp // 16)
        integ.sampler.samples = count_spp
        cst = step(N.PT_RENDER_COUNT_NODES)
        integ.sampler.samples = setup.spp

    sync()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    totals = {"rays_closest": 0, "rays_any": 0, "ms_closest": 0.0, "ms_any": 0.0, "ms_shade": 0.0,
              "launches_closest": 0, "launches_any": 0, "paths": 0, "stack_overflows": 0, "tie_overflows": 0}
    for i in range(args.steps):
        ts = time.perf_counter()
        st = step(N.PT_RENDER_TIMING)
        for k in totals:
            totals[k] += st.get(k, 0)
        if rank == 0:
            log(f"step {i + 1}/{args.steps}: {time.perf_counter() - ts:.2f} s")
    sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    rays = torch.tensor([float(totals["rays_closest"] + totals["rays_any"])], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(rays, op=dist.ReduceOp.SUM)
    elapsed_max = float(t.item())
    total_rays = float(rays.item())

    # ---- untimed: the check of the frame just timed (every rank: its shard)
    verified = None
    if not args.no_verify:
        srange = None
        if cpu_run:
            fs = (lambda p, s: hook.frame_samples(setup, p, s)) if hasattr(hook, "frame_samples") else None
        else:
            fs = integ.context(device).frame_samples
            ctx = integ.context(device)
            srange = ctx.frame_sample_range() if hasattr(ctx._lib, "pt_frame_sample_range") else None
        sh_i, sh_n = shard if shard else (rank, world)
        verified = verify_frame(setup, integ, sh_i, sh_n, args.verify_pairs if fs else 0, fs,
                                film if rank == 0 and not shard else None, sample_range=srange,
                                overflows=None if cpu_run else {k: totals[k] for k in ("stack_overflows",
                                                                                       "tie_overflows")})
        if world > 1:
            ok = torch.tensor([1 if verified["ok"] else 0, verified["pairs"], verified["bit_exact"]],
                              dtype=torch.int64, device=dev)
            dist.all_reduce(ok, op=dist.ReduceOp.SUM)
            verified["ranks_ok"] = int(ok[0].item())
            verified["pairs_all_ranks"] = int(ok[1].item())
            verified["bit_exact_all_ranks"] = int(ok[2].item())
            verified["ok"] = verified["ranks_ok"] == world
        if rank == 0:
            log(f"verify: {verified['bit_exact']}/{verified['pairs']} samples bit-exact, ok={verified['ok']}")
    if args.save_film and rank == 0:
        import numpy as np
        np.save(args.save_film, film.cpu().numpy())

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not shard and not cpu_run:
        cpu = cpu_baseline(setup, args.config, args.cpu_seconds)
    if rank == 0:
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
            "config": {"workload": WORKLOADS.get(args.config, args.config) + (f" (film {args.res}: test)" if args.res else ""), "width": W, "height": H,
                       "spp": setup.spp, "max_depth": setup.max_depth, "integrator": setup.integrator,
                       "rays_per_step": int(total_rays / args.steps),
                       "parallelism": (f"one rank's shard {shard[0]}/{shard[1]} (emulated, no reduce)" if shard
                                       else f"sample-shard x{world}"),
                       "world_size": dist.get_world_size() if world > 1 else 1,
                       "film_reduce": film_reduce,
                       "setup_s": round(setup_s, 1), "bvh_build": bvh_build},
            # rank 0's per-frame kernel time by class (HIP events on the library's stream)
            "kernel_ms_per_step": {k[3:]: round(totals[k] / args.steps, 1)
                                   for k in ("ms_closest", "ms_any", "ms_shade")},
        }
        if cpu_run:
            out["renderer"] = "render hook (CPU rehearsal of the multi-rank path; not a GPU measurement)"
            out["dtype"] = "f64 film / CPU"
        else:
            out["roofline"] = roofline(args, setup, world, totals, cst, cpu)
        if verified is not None:
            out["verified"] = verified
        if cpu:
            v = out["value"]
            cpu["gpu_over_cpu"] = round(v / cpu["value"], 1)
            cpu["gpu_over_full_host_estimate"] = round(v / cpu["full_host_estimate"]["value"], 1)
            ref = cpu.get("reference_estimate")
            if ref:
                # north_star: >= 100x the reference CPU path on this box's host
                # cores -- the reference's estimated rate scaled linearly to
                # every core of the host (an upper bound for the CPU)
                full = ref["value"] / cpu["cores"] * cpu["affinity"]
                cpu["north_star_100x"] = {"target": 100.0, "reference_full_host_estimate": round(full, 2),
                                          "gpu_over_reference_full_host": round(v / full, 1),
                                          "met": bool(v / full >= 100.0),
                                          "note": f"reference estimate at {cpu['cores']} threads scaled "
                                                  f"linearly to {cpu['affinity']} cores"}
            out["cpu_baseline"] = cpu
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def bound_peak(e: dict, large: bool, counted: bool, achieved: float = 0.0) -> None:
    """The bound a kernel's counters show and the ceiling its fraction is
    priced against (a hierarchical roofline: the memory level that serves its
    reads).  HBM bytes near the HBM peak: "hbm" (8 TB/s).  Far below it, with
    most reads L2 hits: "l2-latency", priced against the L2 gather rate
    (L2_GATHER_PEAK_GBS) — each ray's loads form a dependent chain, one round
    trip per step, and the waves wait on it.  Far below it with a low L2 hit
    rate: "memory-latency" (misses served by the Infinity Cache / HBM,
    priced against HBM).  No counter profile of this build: HBM, label
    unknown."""
    tf, hit = e.get("traffic_frac"), e.get("l2_hit_rate")
    if not large:
        e["bound"], peak = "l2/latency", L2_GATHER_PEAK_GBS
    elif (not counted or tf is None) and achieved > HBM_PEAK_GBS:
        # no counters, but more algorithmic bytes than HBM could deliver:
        # caches serve at least part of them
        e["bound"], peak = "l2-latency (no counter profile of this build; algorithmic bytes above the HBM peak)", \
            L2_GATHER_PEAK_GBS
    elif not counted or tf is None:
        e["bound"], peak = "unknown (no counter profile of this build)", HBM_PEAK_GBS
    elif tf >= 0.6:
        e["bound"], peak = "hbm", HBM_PEAK_GBS
    elif hit is not None and hit >= 0.7:
        e["bound"], peak = "l2-latency", L2_GATHER_PEAK_GBS
    else:
        e["bound"], peak = "memory-latency", HBM_PEAK_GBS
    e["peak"] = peak
    e["peak_source"] = ("MI355X_MICROARCH.md 'Indexed rows' L2-served gather, chip-wide"
                        if peak == L2_GATHER_PEAK_GBS else "MI355X_MICROARCH.md HBM3E peak")


def roofline(args, setup, world, totals, cst, cpu):
    """Per-kernel roofline entries."""
    pool = args.traversal == "pool" or (args.traversal == "auto" and args.config in HBM_CONFIGS)
    quant = pool and args.nodes != "full"
    q = ", true" if quant else ", false"
    kname = f"k_closest_pool<false, false{q}>" if pool else "k_closest<false, false>"
    sname = ("k_shadow_sl<false>" if getattr(args, "any_stackless", False) and quant else
             f"k_shadow_pool<false, false{q}>" if pool else "k_shadow<false, false>")
    # the default library reads PT_Q48 records (pt_device.h); PT_Q48=0 tuning
    # builds (64-B nodes) are A/B variants only
    node_bytes = NODE_BYTES["q48"] if quant else NODE_BYTES["full"]
    sha = src_sha()

    def per_ray(c, n, t, r):
        # 128 B per node visit, 48 B per primitive test
        return (128.0 * c[n] + 48.0 * c[t]) / max(1, c[r]) if c and c.get(r) else None

    # the reference's visit order: the oracle's BVH4::Intersect / IntersectPred
    # restatement (entry-distance cull included) over the cpu_baseline sample
    # of the same frame; the GPU's own instrumented count rides beside it
    ref_counts = cpu.pop("_counts") if cpu else None
    ref_c = per_ray(ref_counts, "nodes_closest", "tris_closest", "closest")
    ref_a = per_ray(ref_counts, "nodes_any", "tris_any", "any")
    own_c = per_ray(cst, "nodes_closest", "tris_closest", "rays_closest")
    own_a = per_ray(cst, "nodes_any", "tris_any", "rays_any")

    def entry(name, ref_b, own_b, layout_b, ms, launches, nrays, own_visits=None):
        """frac = algorithmic bytes / launch time / peak, the bytes priced on
        the FEWER of the two visit counts (the reference's order, or the visits
        this kernel makes), so it never credits work the kernel skips."""
        avg_ms = ms / max(1, launches)
        cands = [b for b in (ref_b, own_b) if b]
        if avg_ms <= 0:
            return None
        if not cands:  # no visit counts (--no-count, no CPU sample): timing only
            return {"kernel": name, "avg_launch_ms": round(avg_ms, 4), "launches": launches, "achieved": None,
                    "frac": None, "traffic": None, "bound": None}
        bpr = min(cands)
        per_launch = nrays / max(1, launches)
        gbs = lambda b: b * per_launch / (avg_ms * 1e-3) / 1e9  # noqa: E731
        e = {"kernel": name, "achieved": round(gbs(bpr), 1),
             "bytes_per_ray": round(bpr, 1), "priced_on": "reference order" if bpr == ref_b else "own visits",
             "bytes_per_launch": round(bpr * per_launch), "avg_launch_ms": round(avg_ms, 4), "launches": launches}
        traffic, info = pmc_traffic(args.config, setup.spp, world, name, sha)
        e["traffic"] = traffic
        e.update(info)
        if traffic:
            e["traffic_achieved"] = round(traffic / (avg_ms * 1e-3) / 1e9, 1)
            e["traffic_frac"] = round(e["traffic_achieved"] / HBM_PEAK_GBS, 4)
        bound_peak(e, args.config in HBM_CONFIGS, traffic is not None, gbs(bpr))
        peak = e["peak"]
        e["frac"] = round(gbs(bpr) / peak, 4)
        # SURVEY §8(d)'s own fraction: the algorithmic bytes over the HBM peak
        # (above 1 when caches serve what HBM could not: reuse, not skipped work)
        e["hbm_frac"] = round(gbs(bpr) / HBM_PEAK_GBS, 4)
        if ref_b:
            e["ref_order_bytes_per_ray"] = round(ref_b, 1)
            e["ref_order_frac"] = round(gbs(ref_b) / peak, 4)
        if own_b:
            e["own_visits_bytes_per_ray"] = round(own_b, 1)
            e["own_visits_frac"] = round(gbs(own_b) / peak, 4)
        if layout_b:
            e["layout_bytes_per_ray"] = round(layout_b, 1)
            e["layout_achieved"] = round(gbs(layout_b), 1)
            e["layout_frac"] = round(gbs(layout_b) / peak, 4)
        # the gather ceiling of this access pattern (measured): the loads the
        # visits need (three 16-B loads per 48-B record) and the loads the
        # kernel issues, in lane addresses per clock per CU
        gc = gather_ceiling()
        if gc and own_visits and quant:
            clk = avg_ms * 1e-3 * CLOCK_GHZ * 1e9 * MI355X_CUS
            useful = 3.0 * own_visits * per_launch / clk
            e["gather"] = dict(gc, useful_lane_loads_per_clk_cu=round(useful, 3),
                               useful_frac_of_ceiling=round(useful / gc["lane_loads_per_clk_cu"], 4))
            if e.get("issued_lane_loads_per_clk_cu"):
                e["gather"]["issued_lane_loads_per_clk_cu"] = e["issued_lane_loads_per_clk_cu"]
                e["gather"]["useful_over_issued"] = round(useful / e["issued_lane_loads_per_clk_cu"], 4)
        return e

    lb_c = (node_bytes * cst["nodes_closest"] + 48.0 * cst["tris_closest"]) / max(1, cst["rays_closest"]) if cst else None
    lb_a = ((node_bytes * cst["nodes_any"] + 48.0 * cst["tris_any"]) / cst["rays_any"]
            if cst and cst.get("rays_any") else None)
    vis_c = (cst["nodes_closest"] + cst["tris_closest"]) / max(1, cst["rays_closest"]) if cst else None
    vis_a = (cst["nodes_any"] + cst["tris_any"]) / cst["rays_any"] if cst and cst.get("rays_any") else None
    rc = entry(kname, ref_c, own_c, lb_c, totals["ms_closest"], totals["launches_closest"], totals["rays_closest"],
               vis_c)
    ra = entry(sname, ref_a, own_a, lb_a, totals["ms_any"], totals["launches_any"], totals["rays_any"], vis_a)
    # the headline is north_star's measure: HBM bytes the counters measured per
    # launch over the HBM peak.  SURVEY 8(d)'s algorithmic bytes stay beside
    # it (frac_algorithmic, above 1 where the L2 serves what HBM could not),
    # and the measured gather ceiling of the access pattern under "gather".
    measured = bool(rc and rc.get("traffic_achieved"))
    roof = {"bound": rc["bound"] if rc else None,
            "achieved": (rc["traffic_achieved"] if measured else rc.get("achieved")) if rc else None,
            "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": (rc["traffic_frac"] if measured else rc.get("hbm_frac")) if rc else None,
            "traffic": rc["traffic"] if rc else None,
            "frac_basis": ("rocprofv3 HBM bytes (FETCH_SIZE x calibration + WRITE_SIZE) per launch of this build "
                           "/ the kernel's average launch time / 8 TB/s" if measured else
                           "SURVEY 8(d) algorithmic bytes / 8 TB/s (no counter profile of this build)"),
            "achieved_algorithmic": rc.get("achieved") if rc else None,
            "frac_algorithmic": rc.get("hbm_frac") if rc else None,
            "frac_algorithmic_note": "SURVEY 8(d) bytes (128 B per node, 48 B per primitive) over the HBM peak; "
                                     "> 1 = served by L2, not skipped work",
            "src_sha": sha,
            "count_source": (f"oracle reference order ({ref_counts['closest']} closest / {ref_counts['any']} any rays)"
                             if ref_counts and ref_counts["closest"] else "gpu")}
    if rc:
        for k, v in rc.items():
            roof.setdefault(k, v)
        roof["nodes_per_ray"] = round(ref_counts["nodes_closest"] / max(1, ref_counts["closest"]), 2) \
            if ref_counts else (round(cst["nodes_closest"] / max(1, cst["rays_closest"]), 2) if cst else None)
        roof["tris_per_ray"] = round(ref_counts["tris_closest"] / max(1, ref_counts["closest"]), 2) \
            if ref_counts else (round(cst["tris_closest"] / max(1, cst["rays_closest"]), 2) if cst else None)
        if cst:
            roof["gpu_nodes_per_ray"] = round(cst["nodes_closest"] / max(1, cst["rays_closest"]), 2)
            roof["gpu_tris_per_ray"] = round(cst["tris_closest"] / max(1, cst["rays_closest"]), 2)
        roof["node_layout_bytes"] = node_bytes
    if ra:
        if ref_counts:
            ra["nodes_per_ray"] = round(ref_counts["nodes_any"] / max(1, ref_counts["any"]), 2)
            ra["tris_per_ray"] = round(ref_counts["tris_any"] / max(1, ref_counts["any"]), 2)
        if cst:
            ra["gpu_nodes_per_ray"] = round(cst["nodes_any"] / max(1, cst["rays_any"]), 2)
            ra["gpu_tris_per_ray"] = round(cst["tris_any"] / max(1, cst["rays_any"]), 2)
        roof["shadow"] = ra
    # k_shade: SURVEY §8(d)'s shading bytes per closest-hit ray that hits
    # (96 B attributes + 32 B material record) + 4*C B per bilinear texel
    # fetch, counted by the oracle over the cpu_baseline sample
    shade_name = "k_shade<0>" if setup.integrator == "path" else None
    if shade_name and ref_counts and ref_counts.get("closest"):
        bpr = (128.0 * ref_counts["hits"] + ref_counts["tex_bytes"]) / ref_counts["closest"]
        launches = totals["launches_closest"]
        avg_ms = totals["ms_shade"] / max(1, launches)
        if avg_ms > 0:
            per_launch = totals["rays_closest"] / max(1, launches)
            ach = bpr * per_launch / (avg_ms * 1e-3) / 1e9
            sh = {"kernel": shade_name, "achieved": round(ach, 1),
                  "bytes_per_ray": round(bpr, 1),
                  "hit_fraction": round(ref_counts["hits"] / ref_counts["closest"], 4),
                  "texel_bytes_per_ray": round(ref_counts["tex_bytes"] / ref_counts["closest"], 1),
                  "avg_launch_ms": round(avg_ms, 4), "launches": launches,
                  "pricing": "SURVEY 8(d): (96 B attributes + 32 B material) per hit + 4*C B per bilinear fetch; "
                             "avg_launch_ms includes the hit sort (HIP events bracket sort + shade)"}
            traffic, info = pmc_traffic(args.config, setup.spp, world, shade_name, sha)
            sh["traffic"] = traffic
            sh.update(info)
            if traffic:
                prof_ms = info.get("profile_avg_launch_ms") or avg_ms
                sh["traffic_achieved"] = round(traffic / (prof_ms * 1e-3) / 1e9, 1)
                sh["traffic_frac"] = round(sh["traffic_achieved"] / HBM_PEAK_GBS, 4)
            bound_peak(sh, True, traffic is not None, ach)
            sh["frac"] = round(ach / sh["peak"], 4)
            sh["hbm_frac"] = round(ach / HBM_PEAK_GBS, 4)
            roof["shade"] = sh
    return roof


if __name__ == "__main__":
    main()
