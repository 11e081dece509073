# HEAD build record: smoke, GPU tests, default bench (traffic from the build-matched counter profile)
mkdir -p gpurun_out/r3fa
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3fa/smoke.txt 2>&1 || exit $?
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3fa/tests.txt 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/r3fa/tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/r3fa/bench.json 2> gpurun_out/r3fa/bench.err
