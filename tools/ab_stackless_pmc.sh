#!/bin/bash
# Occupancy counters of the any-hit kernels, default vs stackless (GPU box):
#   tools/ab_stackless_pmc.sh <out_dir>
# One SQ counter pass per arm (counters only, own time limit) over a 1-step
# bench; tools/pmc_pass.sh writes each arm's summary.json.
set -uo pipefail
out="$1"
root=$(cd "$(dirname "$0")/.." && pwd)
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
"$root/tools/pmc_pass.sh" "$out/default" "$C" --steps 1 --warmup 0 --no-count --no-verify && \
PT_HIP_LIB="$root/pathtracing_amd/_lib/variants/libpt_hip_sl7.so" \
    "$root/tools/pmc_pass.sh" "$out/stackless7" "$C" --steps 1 --warmup 0 --no-count --no-verify --any-stackless && \
"$root/tools/pmc_pass.sh" "$out/stackless8" "$C" --steps 1 --warmup 0 --no-count --no-verify --any-stackless
