#!/bin/bash
# One rocprofv3 counter pass over a bench.py run (GPU box):
#   tools/pmc_pass.sh <out_dir> "<counters>" <bench args...>
# Writes <out_dir>/summary.json (per-kernel per-dispatch averages) and drops
# the per-dispatch CSVs.  Each pass has its own time limit; counters only
# (no traces) so the pass is allowed on this pool.
set -euo pipefail
out=$(realpath -m "$1"); ctrs="$2"; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc $ctrs --output-format csv -d "$out/pmc" -o run -- \
    python3 "$root/bench.py" --no-cpu-baseline "$@" > "$out/pmc.log" 2>&1
python3 - "$out" <<'PY'
import csv, glob, json, sys
from collections import defaultdict
d = sys.argv[1]
acc = defaultdict(lambda: defaultdict(float)); disp = defaultdict(lambda: defaultdict(set))
for f in glob.glob(f"{d}/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k][r["Counter_Name"]].add(r["Dispatch_Id"])
res = {k: {c: v / max(1, len(disp[k][c])) for c, v in cs.items()} | {"dispatches": max(len(s) for s in disp[k].values())} for k, cs in acc.items()}
json.dump(res, open(f"{d}/summary.json", "w"), indent=1, sort_keys=True)
for k, v in res.items():
    if "pool" in k or "shade" in k:
        print(k, {a: round(b, 1) for a, b in v.items()})
PY
rm -rf "$out/pmc"
