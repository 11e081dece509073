# final r03 build record: smoke, GPU tests, rocprofv3 trace + counter passes, default bench
# (the counter summary is placed under profiles/ on the box first, so the bench line carries it)
mkdir -p gpurun_out/r3fd
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3fd/smoke.txt 2>&1 || exit $?
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3fd/tests.txt 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/r3fd/tests.txt
[ $rc -eq 0 ] || exit $rc
bash tools/profile_bench.sh gpurun_out/r3fd/prof c4 1024 "k_closest_pool<false, false, true>" --steps 1 --warmup 1 > gpurun_out/r3fd/prof.log 2>&1 || exit $?
cp gpurun_out/r3fd/prof/summary.json profiles/r03_c4_pmc.json || exit $?
timeout -k 10 500 python bench.py > gpurun_out/r3fd/bench.json 2> gpurun_out/r3fd/bench.err
