#!/bin/bash
# One rank's shard of the N-GPU C4 frame on one GPU (the driver's per-rank work):
#   tools/shard_proxy.sh <out_dir>
set -uo pipefail
out="$1"
root=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$root/$out"
cd "$root"
for s in 0/2 0/4 0/8; do
    tag=shard$(echo $s | tr -d /)
    timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-count --shard $s > "$out/$tag.json" 2> "$out/$tag.err" || { tail -3 "$out/$tag.err"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', 'verified', d.get('verified',{}).get('ok'))" "$out/$tag.json" $s
done
