#!/bin/bash
# One GPU-box check of the current tree (run through gpurun):
#   tools/gpu_check.sh <out_dir> [tests|bench|both] [pytest -k expr]
# The GPU test suite (its log, one line per test) and then, unless the suite
# ended in a crash, abort or time limit, one default bench.py line (C4).
# Every GPU step runs under its own time limit; nothing is retried.
set -uo pipefail
out="$1"; what="${2:-both}"; kexpr="${3:-}"
root=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$root/$out"
cd "$root"
rc=0
if [ -n "${PT_FIRST:-}" ] && [ "$what" != bench ]; then
    # the newest tests first, in their own process: a failure (or a fault)
    # there ends the call before the whole suite runs
    timeout -k 10 600 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread \
        -k "$PT_FIRST" > "$out/first.txt" 2>&1
    frc=$?
    tail -3 "$out/first.txt"
    if [ $frc -ne 0 ]; then echo "first tests rc=$frc"; exit $frc; fi
fi
if [ "$what" != bench ]; then
    args=(-u -m pytest tests -m gpu -v --maxfail=20 --timeout 300 --timeout-method thread)
    [ -n "$kexpr" ] && args+=(-k "$kexpr")
    timeout -k 10 1100 python "${args[@]}" > "$out/tests.txt" 2>&1
    rc=$?
    tail -3 "$out/tests.txt"
    echo "tests rc=$rc" | tee -a "$out/tests.txt"
    # 0 passed, 1 some failed: the GPU is fine; anything else (a crash, an
    # abort, the time limit) ends the call here
    if [ $rc -gt 1 ]; then exit $rc; fi
fi
if [ "$what" != tests ]; then
    timeout -k 10 900 python -u bench.py > "$out/bench.json" 2> "$out/bench.err"
    brc=$?
    tail -2 "$out/bench.err"
    cat "$out/bench.json"
    echo "bench rc=$brc"
    [ $brc -ne 0 ] && exit $brc
fi
exit $rc
