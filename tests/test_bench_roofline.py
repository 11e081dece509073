"""bench.py's roofline pricing (CPU): the bound label and the ceiling a
kernel's fraction is priced against come from its counters."""
import bench


def _entry(tf=None, hit=None):
    e = {}
    if tf is not None:
        e["traffic_frac"] = tf
    if hit is not None:
        e["l2_hit_rate"] = hit
    return e


def test_hbm_bound_when_counted_hbm_traffic_is_near_the_peak():
    e = _entry(tf=0.75, hit=0.3)
    bench.bound_peak(e, True, True, 6500.0)
    assert e["bound"] == "hbm" and e["peak"] == bench.HBM_PEAK_GBS


def test_l2_latency_when_hbm_traffic_is_low_and_reads_hit_l2():
    e = _entry(tf=0.11, hit=0.81)
    bench.bound_peak(e, True, True, 9000.0)
    assert e["bound"] == "l2-latency" and e["peak"] == bench.L2_GATHER_PEAK_GBS
    assert 9000.0 / e["peak"] <= 1.0


def test_memory_latency_when_hbm_traffic_is_low_and_l2_misses():
    e = _entry(tf=0.30, hit=0.56)
    bench.bound_peak(e, True, True, 640.0)
    assert e["bound"] == "memory-latency" and e["peak"] == bench.HBM_PEAK_GBS


def test_without_counters_algorithmic_bytes_above_hbm_are_priced_on_l2():
    e = _entry()
    bench.bound_peak(e, True, False, 9100.0)
    assert e["bound"].startswith("l2-latency") and e["peak"] == bench.L2_GATHER_PEAK_GBS
    e = _entry()
    bench.bound_peak(e, True, False, 5000.0)
    assert e["bound"].startswith("unknown") and e["peak"] == bench.HBM_PEAK_GBS


def test_small_scenes_are_labelled_cache_resident():
    e = _entry(tf=0.01, hit=0.99)
    bench.bound_peak(e, False, True, 20000.0)
    assert e["bound"] == "l2/latency" and e["peak"] == bench.L2_GATHER_PEAK_GBS


def test_q48_records_are_priced_at_48_bytes_per_node_step():
    """The default pool traversal reads PT_Q48 records (pt_device.h): 48 B per
    node step, as per primitive slot."""
    assert bench.NODE_BYTES["q48"] == 48.0
    assert bench.NODE_BYTES["full"] == 128.0


def test_gather_ceiling_comes_from_the_committed_microbenchmark(tmp_path, monkeypatch):
    """bench.gather_ceiling reads profiles/r05_gather_rate.json (tools/gather_rate.hip,
    parsed by tools/gather_rate_json.py): the best P3 L2 rate in lane-loads per
    clock per CU, in GB/s at 16 B per lane-load over 256 CUs at 2.4 GHz."""
    import sys
    sys.path.insert(0, str(bench.ROOT / "tools"))
    import gather_rate_json
    text = ("L2     P3  waves/SIMD 2      1.87 ms     4.48 G wave-steps/s   1.399 lane-loads/clk/CU     1098 clk/step/wave\n"
            "L2     P3  waves/SIMD 4      3.64 ms     4.61 G wave-steps/s   1.441 lane-loads/clk/CU     2131 clk/step/wave\n"
            "HBM    P3  waves/SIMD 4      3.23 ms     1.30 G wave-steps/s   0.405 lane-loads/clk/CU     7578 clk/step/wave\n")
    prof = gather_rate_json.parse(text)
    assert len(prof["rows"]) == 3
    (tmp_path / "profiles").mkdir()
    (tmp_path / "profiles" / "r05_gather_rate.json").write_text(__import__("json").dumps(prof))
    monkeypatch.setattr(bench, "ROOT", tmp_path)
    g = bench.gather_ceiling()
    assert g["lane_loads_per_clk_cu"] == 1.441
    assert abs(g["gbs_at_16B"] - 1.441 * 16 * 256 * 2.4) < 0.1
    assert bench.gather_ceiling("P3", "HBM")["lane_loads_per_clk_cu"] == 0.405


def _roof(monkeypatch, traffic_bytes):
    import types
    args = types.SimpleNamespace(traversal="auto", config="c4", nodes="auto")
    setup = types.SimpleNamespace(spp=1024, integrator="path")
    totals = {"ms_closest": 29 * 121.0, "launches_closest": 29, "rays_closest": 6_857_000_000,
              "ms_any": 29 * 38.0, "launches_any": 29, "rays_any": 2_000_000_000, "ms_shade": 1205.0}
    cst = {"nodes_closest": 33.86e9, "tris_closest": 15.57e9, "rays_closest": 1e9,
           "nodes_any": 21.6e9, "tris_any": 9.0e9, "rays_any": 1e9}

    def fake_pmc(config, spp, world, kernel, sha):
        if traffic_bytes is None:
            return None, {"traffic_note": "none"}
        return traffic_bytes, {"l2_hit_rate": 0.82, "issued_lane_loads_per_clk_cu": 1.9}
    monkeypatch.setattr(bench, "pmc_traffic", fake_pmc)
    monkeypatch.setattr(bench, "gather_ceiling", lambda *a: {"pattern": "P3 L2", "lane_loads_per_clk_cu": 1.441,
                                                             "gbs_at_16B": 14165.0, "source": "test"})
    return bench.roofline(args, setup, 1, totals, cst, None)


def test_headline_frac_is_the_counted_hbm_fraction(monkeypatch):
    """With a counter profile of the build the headline is north_star's
    measure (HBM bytes per launch / launch time / 8 TB/s); SURVEY 8(d)'s
    algorithmic figure stays beside it as frac_algorithmic."""
    per_launch = 103.6e9
    roof = _roof(monkeypatch, per_launch)
    assert roof["peak"] == bench.HBM_PEAK_GBS and roof["unit"] == "GB/s"
    assert abs(roof["achieved"] - per_launch / 0.121 / 1e9) < 1.0
    assert abs(roof["frac"] - roof["achieved"] / bench.HBM_PEAK_GBS) < 1e-3
    assert roof["frac_algorithmic"] > 1.0 and roof["frac"] < 0.2
    assert roof["node_layout_bytes"] == 48.0
    g = roof["gather"]
    assert g["useful_lane_loads_per_clk_cu"] > 0 and g["issued_lane_loads_per_clk_cu"] == 1.9


def test_without_counters_the_headline_is_algorithmic_and_says_so(monkeypatch):
    roof = _roof(monkeypatch, None)
    assert roof["frac"] == roof["frac_algorithmic"]
    assert roof["frac_basis"].startswith("SURVEY 8(d) algorithmic")


def test_timing_only_runs_keep_a_headline_without_fractions(monkeypatch):
    """--no-count with no CPU sample (the A/B runs): no visit counts, so the
    entries carry launch times only and the headline's fractions are null."""
    import types
    monkeypatch.setattr(bench, "pmc_traffic", lambda *a: (None, {}))
    args = types.SimpleNamespace(traversal="auto", config="c4", nodes="auto")
    setup = types.SimpleNamespace(spp=1024, integrator="path")
    totals = {"ms_closest": 29 * 121.0, "launches_closest": 29, "rays_closest": 6_857_000_000,
              "ms_any": 29 * 38.0, "launches_any": 29, "rays_any": 2_000_000_000, "ms_shade": 1205.0}
    roof = bench.roofline(args, setup, 1, totals, None, None)
    assert roof["frac"] is None and roof["achieved"] is None and roof["frac_algorithmic"] is None
    assert abs(roof["avg_launch_ms"] - 121.0) < 1e-6
