# A/B: overlapped traversal with a two-deep leaf queue (specF/G) vs one (specE) vs base
mkdir -p gpurun_out/r3s
timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3s/bench_base.json 2> gpurun_out/r3s/bench_base.err || exit $?
for v in specE specF specG; do
PT_HIP_LIB=pathtracing_amd/_lib/variants/libpt_hip_$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3s/bench_$v.json 2> gpurun_out/r3s/bench_$v.err || exit $?
done
PT_HIP_LIB=pathtracing_amd/_lib/variants/libpt_hip_itersF.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --spp 256 --steps 1 --warmup 0 > gpurun_out/r3s/iters.json 2> gpurun_out/r3s/iters.err
