#!/bin/bash
# A/B timing of library variants (tools/build_native.py --variant=...) on the
# GPU box:  tools/ab_bench.sh OUTDIR "bench args" variant1 variant2 ...
# One bench.py process per variant, each under its own time limit; stops at
# the first failure.  Variant "default" is pathtracing_amd/_lib/libpt_hip.so.
set -o pipefail
out=$1; args=$2; shift 2
mkdir -p "$out"
for v in "$@"; do
    if [ "$v" = default ]; then lib=pathtracing_amd/_lib/libpt_hip.so; else lib=pathtracing_amd/_lib/variants/libpt_hip_$v.so; fi
    tag=$(echo "$args" | tr -c 'a-zA-Z0-9' '_')
    PT_HIP_LIB=$lib timeout -k 10 300 python bench.py $args --no-cpu-baseline > "$out/${v}_$tag.json" 2> "$out/${v}_$tag.err" || { echo "FAIL $v $args"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], sys.argv[3], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/step', r['avg_launch_ms'], 'ms/closest')" "$out/${v}_$tag.json" "$v" "$args"
done
