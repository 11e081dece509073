mkdir -p gpurun_out/r3m
for v in wpe6 wpe0; do
PT_HIP_LIB=pathtracing_amd/_lib/variants/libpt_hip_$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3m/bench_$v.json 2> gpurun_out/r3m/bench_$v.err || exit $?
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3m/bench_base.json 2> gpurun_out/r3m/bench_base.err
