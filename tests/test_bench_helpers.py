"""bench.py's host-side accounting (no GPU): the HBM-traffic reading of a
committed counter profile and its calibration factor per access pattern, and
the CPU-baseline ratio table."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def test_traffic_uses_the_profile_of_this_build_only():
    sha = bench.src_sha()
    traffic, info = bench.pmc_traffic("c4", 1024, 1, "k_closest_pool<false, false, true>", sha)
    prof = json.loads((ROOT / "profiles" / info["traffic_source"]).read_text())
    if prof["_meta"]["src_sha"] != sha:  # sources edited since the last profile
        assert traffic is None and "another build" in info["traffic_note"]
        return
    k = prof["k_closest_pool<false, false, true>"]
    # 64-B quantized nodes: FETCH_SIZE x 1.0 (the half-line calibration entry)
    assert info["fetch_factor_source"].endswith("factor_qnode_gather")
    want = (info["fetch_factor"] * k["FETCH_SIZE_per_dispatch"] + k["WRITE_SIZE_per_dispatch"]) * 1024.0
    assert traffic == round(want)
    # a different build's sources never borrow it
    t2, i2 = bench.pmc_traffic("c4", 1024, 1, "k_closest_pool<false, false, true>", "0" * 16)
    assert t2 is None and "another build" in i2["traffic_note"]


def test_full_cluster_kernels_use_the_full_line_factor():
    _, info = bench.pmc_traffic("c4", 1024, 1, "k_closest_pool<false, false, false>", "0" * 16)
    assert info["fetch_factor_source"].endswith("factor_node_gather")
    calib = json.loads((ROOT / "profiles" / "r03_fetch_calib.json").read_text())
    assert abs(calib["factor_node_gather"] - 2.0) < 0.01 and abs(calib["factor_qnode_gather"] - 1.0) < 0.01
    # FETCH_SIZE counts 64 B per touched line for every pattern
    assert abs(calib["k_texel_gather"]["fetch_bytes_per_line"] - 64.0) < 1.0


def test_cpu_ratio_table_covers_the_thread_counts():
    r = json.loads((ROOT / "profiles" / "r03_cpu_ratio.json").read_text())
    for key in ("c1_example1_path_256x256_16spp", "c4_recipe_2pct_160x90_16spp_depth128"):
        by = r[key]["by_threads"]
        assert set(by) >= {"1", "2", "4", "8"}
        for t, e in by.items():
            assert abs(e["port_mrays"] / e["reference_li_loop_mrays"] - e["port_over_reference"]) < 0.01


def test_cpu_ratio_r06_full_detail_c4():
    """r06: the port / reference ratio on the full-detail C4 scene itself
    (tools/cpu_ratio.py), which bench.py's cpu_baseline now prefers."""
    r = json.loads((ROOT / "profiles" / "r06_cpu_ratio.json").read_text())
    e = r["c4_full_192x108_32spp_depth128"]
    assert set(e["by_threads"]) >= {"1", "8"}
    for t, v in e["by_threads"].items():
        assert abs(v["port_mrays"] / v["reference_li_loop_mrays"] - v["port_over_reference"]) < 0.01
    # the r03 entries merged in, so c1 keeps its ratio
    assert "c1_example1_path_256x256_16spp" in r
