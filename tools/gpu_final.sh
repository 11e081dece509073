#!/bin/bash
# The round's final GPU check of the current tree (GPU box):
#   tools/gpu_final.sh <out_dir>
# GPU suite, smoke, the default bench line, the same bench under
# torch.distributed.run at N = 1 (the driver's multi-rank launch).  Every step
# under its own time limit; stops at the first failure.
set -uo pipefail
out="$1"
root=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$root/$out"
cd "$root"
tools/gpu_check.sh "$out" tests || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.txt" 2>&1 || { tail -5 "$out/smoke.txt"; exit 1; }
tail -1 "$out/smoke.txt"
timeout -k 10 600 python -u bench.py > "$out/bench.json" 2> "$out/bench.err" || { tail -5 "$out/bench.err"; exit 1; }
cat "$out/bench.json"
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 1 > "$out/bench_torchrun.json" 2> "$out/bench_torchrun.err" || {
    tail -5 "$out/bench_torchrun.err"; exit 1; }
echo final ok
