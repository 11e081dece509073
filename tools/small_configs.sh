#!/bin/bash
# The small BASELINE configs on the GPU box: tools/small_configs.sh <out_dir>
set -uo pipefail
out="$1"
root=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$root/$out"
cd "$root"
for c in c1 c2 c3; do
    timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > "$out/$c.json" 2> "$out/$c.err" || { tail -3 "$out/$c.err"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['unit'], d['ms_per_step'], 'ms', 'verified', d.get('verified',{}).get('ok'))" "$out/$c.json" $c
done
