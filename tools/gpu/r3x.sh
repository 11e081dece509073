# A/B: cluster order in memory (breadth-first; children together + depth-first subtrees)
mkdir -p gpurun_out/r3x
timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3x/bench_base.json 2> gpurun_out/r3x/bench_base.err || exit $?
for v in order1 order2; do
export PT_HIP_LIB=pathtracing_amd/_lib/variants/libpt_hip_$v.so
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3x/smoke_$v.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3x/bench_$v.json 2> gpurun_out/r3x/bench_$v.err || exit $?
done
