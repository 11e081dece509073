"""Summarise tools/profile_pmc.sh output: per kernel, calls, average duration,
and per-dispatch averages of each PMC counter (FETCH_SIZE/WRITE_SIZE in KB as
rocprofv3 reports them).  Writes JSON + prints a table.

    python tools/pmc_summary.py <profile dir> <out.json> [config spp kernel [src_sha]]

With the optional workload fields the JSON carries a "_meta" record that
bench.py uses to attach the counter traffic to its roofline line.
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def short(name):
    return name.split("(")[0].replace("void ", "")


def main(d, out, meta=None):
    res = defaultdict(lambda: {"calls": 0, "dur_ns": 0.0, "counters": defaultdict(float), "dispatches": defaultdict(set)})
    for f in glob.glob(f"{d}/trace/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            res[k]["calls"] += 1
            res[k]["dur_ns"] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for f in glob.glob(f"{d}/*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            c = r["Counter_Name"]
            res[k]["counters"][c] += float(r["Counter_Value"])
            res[k]["dispatches"][c].add(r["Dispatch_Id"])
    table = {}
    for k, v in res.items():
        if v["calls"] == 0:
            continue
        row = {"calls": v["calls"], "avg_us": v["dur_ns"] / v["calls"] / 1e3}
        for c, tot in v["counters"].items():
            row[c + "_per_dispatch"] = tot / max(1, len(v["dispatches"][c]))
        table[k] = row
    if meta:
        table["_meta"] = meta
    json.dump(table, open(out, "w"), indent=1, sort_keys=True)
    for k, row in sorted(((k, r) for k, r in table.items() if k != "_meta"),
                         key=lambda kv: -kv[1]["calls"] * kv[1]["avg_us"]):
        print(k, {a: round(b, 1) for a, b in row.items()})


if __name__ == "__main__":
    meta = None
    if len(sys.argv) > 5:
        meta = {"config": sys.argv[3], "spp": int(sys.argv[4]), "kernel": sys.argv[5], "n_gpus": 1}
        if len(sys.argv) > 6:
            meta["src_sha"] = sys.argv[6]
    main(sys.argv[1], sys.argv[2], meta)
