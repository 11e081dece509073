#!/bin/bash
# A/B of the stackless any-hit traversal on C4 (GPU box):
#   tools/ab_stackless.sh <out_dir>
# default (LDS-stack any hit) / --any-stackless at 8 waves per SIMD / at 7
# (variant libpt_hip_sl7.so, PT_SL_WPE=7); one bench process each, own limit.
set -uo pipefail
out="$1"
root=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$root/$out"
cd "$root"
run() {  # tag lib args...
    local tag=$1 lib=$2; shift 2
    PT_HIP_LIB="$lib" timeout -k 10 400 python -u bench.py --no-cpu-baseline "$@" > "$out/$tag.json" 2> "$out/$tag.err"
    local rc=$?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernel_ms_per_step']; r=d['roofline']; s=r.get('shadow',{}); print(sys.argv[2], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', 'any', k['any'], 'ms/frame', s.get('kernel'), s.get('gpu_nodes_per_ray'), s.get('gpu_tris_per_ray'), 'verified', d.get('verified',{}).get('ok'))" "$out/$tag.json" "$tag" || true
    return $rc
}
run default pathtracing_amd/_lib/libpt_hip.so && \
run stackless8 pathtracing_amd/_lib/libpt_hip.so --any-stackless && \
run stackless7 pathtracing_amd/_lib/variants/libpt_hip_sl7.so --any-stackless
