mkdir -p gpurun_out/r3e
timeout -k 10 120 python -u tools/diag_lightcases.py lit_instances > gpurun_out/r3e/diag_light.txt 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3e/tests.txt 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/r3e/tests.txt
[ $rc -le 1 ] || exit $rc
bash tools/profile_bench.sh gpurun_out/r3e/prof c4 1024 "k_closest_pool<false, false, true>" --steps 1 --warmup 1 > gpurun_out/r3e/prof.log 2>&1 || exit $?
timeout -k 10 500 python bench.py > gpurun_out/r3e/bench.json 2> gpurun_out/r3e/bench.err
