# A/B: overlapped traversal variants (ray index in LDS, node-first vs primitive-first, shadow waves)
mkdir -p gpurun_out/r3t
timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3t/bench_base.json 2> gpurun_out/r3t/bench_base.err || exit $?
for v in specE specH specK specL; do
PT_HIP_LIB=pathtracing_amd/_lib/variants/libpt_hip_$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3t/bench_$v.json 2> gpurun_out/r3t/bench_$v.err || exit $?
done
