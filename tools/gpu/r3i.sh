mkdir -p gpurun_out/r3i
timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 3 --spp 128 > gpurun_out/r3i/bench_spp128.json 2> gpurun_out/r3i/bench_spp128.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 3 --spp 256 > gpurun_out/r3i/bench_spp256.json 2> gpurun_out/r3i/bench_spp256.err
