#!/bin/bash
# rocprofv3 passes over one bench.py configuration (run on the GPU box):
#   tools/profile_bench.sh <out_dir> <config> <spp> <kernel> <bench args...>
# 1: kernel trace + stats; 2: FETCH_SIZE; 3: WRITE_SIZE; 4: SQ cycle counters;
# 5: L2 hit/miss.  Counter passes are separate runs with counters only (no
# --pmc together with traces).  Writes <out_dir>/summary.json (per-kernel
# per-dispatch averages, `_meta` with the source hash of the build) and
# <out_dir>/kernel_stats.csv; drops the per-dispatch CSVs.
set -euo pipefail
out=$(realpath -m "$1"); cfg="$2"; spp="$3"; kern="$4"; shift 4
root=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
B="$root/bench.py"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
    python3 "$B" --no-cpu-baseline --no-count "$@" > "$out/trace.log" 2>&1
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- \
    python3 "$B" --no-cpu-baseline --no-count "$@" > "$out/fetch.log" 2>&1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- \
    python3 "$B" --no-cpu-baseline --no-count "$@" > "$out/write.log" 2>&1
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD --output-format csv -d "$out/sq" -o run -- \
    python3 "$B" --no-cpu-baseline --no-count "$@" > "$out/sq.log" 2>&1
timeout -s KILL 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$out/tcc" -o run -- \
    python3 "$B" --no-cpu-baseline --no-count "$@" > "$out/tcc.log" 2>&1 || echo "tcc pass failed (rc $?)"
sha=$(cd "$root" && python3 -c "import bench; print(bench.src_sha())")
python3 "$root/tools/pmc_summary.py" "$out" "$out/summary.json" "$cfg" "$spp" "$kern" "$sha" > "$out/summary.txt"
cp "$out"/trace/run_kernel_stats.csv "$out/kernel_stats.csv"
# compact per-dispatch timeline of the wavefront kernels (order, kernel, us)
python3 - "$out" <<'PY'
import csv, glob, sys
d = sys.argv[1]
rows = []
for f in glob.glob(f"{d}/trace/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if k.startswith("k_"):
            rows.append((int(r["Start_Timestamp"]), k, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
rows.sort()
with open(f"{d}/dispatches.csv", "w") as o:
    o.write("start_us,kernel,us\n")
    t0 = rows[0][0] if rows else 0
    for s, k, us in rows:
        o.write(f'{(s - t0) / 1e3:.1f},"{k}",{us:.1f}\n')
PY
rm -rf "$out/trace" "$out/fetch" "$out/write" "$out/sq" "$out/tcc"
echo done
