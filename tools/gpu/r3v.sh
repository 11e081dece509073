# A/B: overlapped traversal with the rare primitive work outside the step loop
# (7 waves without hot-path spills) vs the committed build (6 waves)
mkdir -p gpurun_out/r3v
timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3v/bench_base.json 2> gpurun_out/r3v/bench_base.err || exit $?
for v in specM specN specO; do
export PT_HIP_LIB=pathtracing_amd/_lib/variants/libpt_hip_$v.so
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3v/smoke_$v.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3v/bench_$v.json 2> gpurun_out/r3v/bench_$v.err || exit $?
done
