"""FETCH_SIZE calibration (GPU box): run tools/fetch_calib.hip under
rocprofv3 (one FETCH_SIZE pass, one kernel-trace pass) and write the factors
known_bytes / (FETCH_SIZE * 1024) per access pattern.

    python3 tools/fetch_calib.py <out.json>

bench.py multiplies the traversal kernel's FETCH_SIZE by
`factor_node_gather` (one 128-B cluster per lane, 8 x 16-B loads — the
pattern of k_closest_pool's node steps) to turn the counter into HBM bytes.
"""
import csv
import glob
import json
import os
import subprocess
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
BIN = ROOT / "tools" / "_bin" / "fetch_calib"


def run(out_dir: Path, args):
    os.makedirs(out_dir, exist_ok=True)
    cmd = ["timeout", "-s", "KILL", "120", "rocprofv3", *args, "--output-format", "csv", "-d", str(out_dir), "-o",
           "run", "--", str(BIN)]
    r = subprocess.run(cmd, capture_output=True, text=True, cwd="/tmp", env={**os.environ, "TMPDIR": "/tmp"})
    if r.returncode:
        sys.stderr.write(r.stdout[-4000:] + r.stderr[-4000:])
        raise SystemExit(r.returncode)
    return r.stdout


def main(out_json):
    work = ROOT / "gpurun_out" / "fetch_calib"
    stdout = run(work / "fetch", ["--pmc", "FETCH_SIZE"])
    known = {}
    for line in stdout.splitlines():
        if line.startswith("{"):
            rec = json.loads(line)
            known[rec["kernel"]] = rec["bytes"]
    per = defaultdict(list)
    for f in glob.glob(str(work / "fetch" / "**" / "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if r["Counter_Name"] == "FETCH_SIZE":
                per[k].append(float(r["Counter_Value"]))
    trace_out = run(work / "trace", ["--kernel-trace", "--stats"])
    res = {"_meta": {"tool": "tools/fetch_calib.hip", "table_bytes": 4 << 30,
                     "note": "factor = known bytes / (FETCH_SIZE KB * 1024), per dispatch"}}
    for k, vals in per.items():
        if k not in known:
            continue
        kb = sum(vals) / len(vals)
        res[k] = {"known_bytes": known[k], "fetch_size_kb_per_dispatch": round(kb, 1), "dispatches": len(vals),
                  "factor": round(known[k] / (kb * 1024.0), 4)}
    stats = glob.glob(str(work / "trace" / "**" / "*kernel_stats.csv"), recursive=True)
    for f in stats:
        for r in csv.DictReader(open(f)):
            k = r["Name"].split("(")[0].replace("void ", "")
            if k in res:
                avg_ns = float(r["AverageNs"])
                res[k]["avg_us"] = round(avg_ns / 1e3, 2)
                res[k]["algorithmic_GBps"] = round(known[k] / avg_ns, 1)
    res["factor_node_gather"] = res.get("k_node_gather", {}).get("factor")
    res["factor_slot_gather"] = res.get("k_slot_gather", {}).get("factor")
    res["factor_stream"] = res.get("k_stream", {}).get("factor")
    res["factor_qnode_gather"] = res.get("k_qnode_gather", {}).get("factor")
    # texel rows: FETCH_SIZE per touched line, against the 128-B lines touched
    tg = res.get("k_texel_gather")
    if tg:
        lines = tg["known_bytes"] / 16 * 2
        tg["fetch_bytes_per_line"] = round(tg["fetch_size_kb_per_dispatch"] * 1024.0 / lines, 1)
        if "avg_us" in tg:
            tg["lines_per_us"] = round(lines / tg["avg_us"], 1)
        res["factor_texel_gather"] = tg["factor"]
    Path(out_json).write_text(json.dumps(res, indent=1, sort_keys=True))
    print(json.dumps(res, indent=1, sort_keys=True))
    del trace_out


if __name__ == "__main__":
    main(sys.argv[1])
