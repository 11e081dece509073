# A/B: LDS stack entries of the closest-hit pool kernel only (the any-hit kernel keeps 20: at 7 waves its blocks fill the LDS)
mkdir -p gpurun_out/r3fe
timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3fe/bench_base.json 2> gpurun_out/r3fe/bench_base.err || exit $?
for v in lc24 lc26; do
export PT_HIP_LIB=pathtracing_amd/_lib/variants/libpt_hip_$v.so
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3fe/smoke_$v.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3fe/bench_$v.json 2> gpurun_out/r3fe/bench_$v.err || exit $?
done
