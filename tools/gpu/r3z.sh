# A/B: entry-distance cull in the overlapped closest-hit kernel (16 / 14 LDS entries)
mkdir -p gpurun_out/r3z
timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3z/bench_base.json 2> gpurun_out/r3z/bench_base.err || exit $?
for v in ent ent20; do
export PT_HIP_LIB=pathtracing_amd/_lib/variants/libpt_hip_$v.so
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3z/smoke_$v.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 > gpurun_out/r3z/bench_$v.json 2> gpurun_out/r3z/bench_$v.err || exit $?
done
