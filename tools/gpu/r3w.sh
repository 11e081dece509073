mkdir -p gpurun_out/r3w
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3w/smoke.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3w/tests.txt 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/r3w/tests.txt
[ $rc -eq 0 ] || exit $rc
bash tools/profile_bench.sh gpurun_out/r3w/prof c4 1024 "k_closest_pool<false, false, true>" --steps 1 --warmup 1 > gpurun_out/r3w/prof.log 2>&1 || exit $?
timeout -k 10 500 python bench.py > gpurun_out/r3w/bench.json 2> gpurun_out/r3w/bench.err
