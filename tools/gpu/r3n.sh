# A/B: wave-uniform step scheduling in the pool traversal (PT_SCHED) vs off,
# and the node-cost constant
mkdir -p gpurun_out/r3n
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3n/smoke.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3n/bench_base.json 2> gpurun_out/r3n/bench_base.err || exit $?
for v in sched0 schedn120 schedn300; do
PT_HIP_LIB=pathtracing_amd/_lib/variants/libpt_hip_$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3n/bench_$v.json 2> gpurun_out/r3n/bench_$v.err || exit $?
done
