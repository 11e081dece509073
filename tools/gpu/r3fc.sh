# A/B: refill threshold of the overlapped pool kernels (swept at r02 on the one-step kernels: 16)
mkdir -p gpurun_out/r3fc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3fc/bench_base.json 2> gpurun_out/r3fc/bench_base.err || exit $?
for v in rf8 rf12 rf24; do
export PT_HIP_LIB=pathtracing_amd/_lib/variants/libpt_hip_$v.so
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3fc/smoke_$v.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3fc/bench_$v.json 2> gpurun_out/r3fc/bench_$v.err || exit $?
done
unset PT_HIP_LIB
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "overlapped or full_size" > gpurun_out/r3fc/tests_ovl.txt 2>&1
