# A/B: overlapped traversal (PT_SPEC) at 6/7 waves vs the committed kernels
mkdir -p gpurun_out/r3q
timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3q/bench_base.json 2> gpurun_out/r3q/bench_base.err || exit $?
for v in specD specE specA; do
export PT_HIP_LIB=pathtracing_amd/_lib/variants/libpt_hip_$v.so
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3q/smoke_$v.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3q/bench_$v.json 2> gpurun_out/r3q/bench_$v.err || exit $?
done
