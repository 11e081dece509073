#!/bin/bash
# rocprofv3 passes for one bench configuration (run on the GPU box):
#   tools/profile_pmc.sh <out_dir> <config> <spp> <kernel> <bench args...>
# 1: kernel trace + stats; 2: FETCH_SIZE; 3: WRITE_SIZE; 4: SQ cycle/instruction
# counters.  Counter passes are separate (no --pmc together with traces).
set -euo pipefail
out=$(realpath -m "$1"); cfg="$2"; spp="$3"; kern="$4"; shift 4
root=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
    python3 "$root/bench.py" --no-cpu-baseline "$@" > "$out/trace.log" 2>&1
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- \
    python3 "$root/bench.py" --no-cpu-baseline "$@" > "$out/fetch.log" 2>&1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- \
    python3 "$root/bench.py" --no-cpu-baseline "$@" > "$out/write.log" 2>&1
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD --output-format csv -d "$out/sq" -o run -- \
    python3 "$root/bench.py" --no-cpu-baseline "$@" > "$out/sq.log" 2>&1
# summarise on the box and drop the per-dispatch CSVs (they can exceed what
# gpurun copies back): keep the stats table, the JSON summary and the logs
python3 "$root/tools/pmc_summary.py" "$out" "$out/summary.json" "$cfg" "$spp" "$kern" > "$out/summary.txt"
cp "$out"/trace/run_kernel_stats.csv "$out/kernel_stats.csv"
rm -rf "$out/trace" "$out/fetch" "$out/write" "$out/sq"
echo done
