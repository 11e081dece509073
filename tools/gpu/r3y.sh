# A/B: 64-B primitive slots (no slot spans two sectors / lines) vs 48-B
mkdir -p gpurun_out/r3y
timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3y/bench_base.json 2> gpurun_out/r3y/bench_base.err || exit $?
for v in geom64; do
export PT_HIP_LIB=pathtracing_amd/_lib/variants/libpt_hip_$v.so
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3y/smoke_$v.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3y/bench_$v.json 2> gpurun_out/r3y/bench_$v.err || exit $?
done
