mkdir -p gpurun_out/r3k
V=pathtracing_amd/_lib/variants/libpt_hip_wide.so
PT_HIP_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "pool_and_simple or trace_matches or sanmiguel" > gpurun_out/r3k/tests_wide.txt 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/r3k/tests_wide.txt
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3k/bench_base.json 2> gpurun_out/r3k/bench_base.err || exit $?
PT_HIP_LIB=$V timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 > gpurun_out/r3k/bench_wide.json 2> gpurun_out/r3k/bench_wide.err
