#!/bin/bash
# Misc C4 bench probes (GPU box): tools/ab_misc.sh <out_dir>
# default / 768 M paths in flight / one rank's 1/8 shard (the N = 8 per-rank work)
set -uo pipefail
out="$1"
root=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$root/$out"
cd "$root"
run() {  # tag args...
    local tag=$1; shift
    timeout -k 10 500 python -u bench.py --no-cpu-baseline "$@" > "$out/$tag.json" 2> "$out/$tag.err"
    local rc=$?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', json.dumps(d['kernel_ms_per_step']), 'verified', d.get('verified',{}).get('ok'))" "$out/$tag.json" "$tag" || true
    return $rc
}
run default && run p768 --paths-in-flight 805306368 && run shard8 --shard 0/8
