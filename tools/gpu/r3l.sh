mkdir -p gpurun_out/r3l
V=pathtracing_amd/_lib/variants/libpt_hip_notex.so
PT_HIP_LIB=$V timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3l/bench_notex.json 2> gpurun_out/r3l/bench_notex.err
