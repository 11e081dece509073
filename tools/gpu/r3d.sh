mkdir -p gpurun_out/r3d
timeout -k 10 300 python -u tools/bitdiff.py gpurun_out/r3d/bd.json --c4 > gpurun_out/r3d/bd.txt 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3d/tests.txt 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/r3d/tests.txt
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r3d/bench.json 2> gpurun_out/r3d/bench.err
