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
