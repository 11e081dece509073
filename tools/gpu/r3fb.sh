# A/B: k_shade block size / waves per SIMD (1024 x 4 waves spills 33 VGPRs; 3 waves fit 157 VGPRs)
mkdir -p gpurun_out/r3fb
timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3fb/bench_base.json 2> gpurun_out/r3fb/bench_base.err || exit $?
for v in ovl sh512w3 sh256w3; do
export PT_HIP_LIB=pathtracing_amd/_lib/variants/libpt_hip_$v.so
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3fb/smoke_$v.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3fb/bench_$v.json 2> gpurun_out/r3fb/bench_$v.err || exit $?
done
