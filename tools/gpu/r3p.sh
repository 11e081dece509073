# pool-kernel iteration statistics (PT_ITER_STATS diagnostics build)
mkdir -p gpurun_out/r3p
PT_HIP_LIB=pathtracing_amd/_lib/variants/libpt_hip_iters.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --spp 256 --steps 1 --warmup 0 > gpurun_out/r3p/bench.json 2> gpurun_out/r3p/bench.err
