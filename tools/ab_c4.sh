#!/bin/bash
# A/B of library variants on one bench configuration (GPU box):
#   tools/ab_c4.sh <out_dir> "<variant names>" <bench args...>
# variant "default" = pathtracing_amd/_lib/libpt_hip.so, else
# pathtracing_amd/_lib/variants/libpt_hip_<name>.so (tools/build_native.py --variant)
set -euo pipefail
out="$1"; vars="$2"; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$out"
for v in $vars; do
  if [ "$v" = default ]; then lib="$root/pathtracing_amd/_lib/libpt_hip.so"; else lib="$root/pathtracing_amd/_lib/variants/libpt_hip_$v.so"; fi
  PT_HIP_LIB="$lib" timeout -k 10 300 python3 "$root/bench.py" --no-cpu-baseline "$@" > "$out/$v.json" 2> "$out/$v.err"
  python3 -c "import json,sys; d=json.load(open('$out/$v.json')); r=d['roofline']; print('$v', d['value'], d['ms_per_step'], r.get('avg_launch_ms'), r.get('nodes_per_ray'), r.get('tris_per_ray'), r.get('shadow',{}).get('avg_launch_ms'))"
done
