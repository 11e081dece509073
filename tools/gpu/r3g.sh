mkdir -p gpurun_out/r3g
V=pathtracing_amd/_lib/variants/libpt_hip_lds1.so
PT_HIP_LIB=$V timeout -k 10 300 python -u tools/bitdiff.py gpurun_out/r3g/bd_lds1.json > gpurun_out/r3g/bd_lds1.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3g/bench_base.json 2> gpurun_out/r3g/bench_base.err || exit $?
PT_HIP_LIB=$V timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3g/bench_lds1.json 2> gpurun_out/r3g/bench_lds1.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3g/bench_base2.json 2> gpurun_out/r3g/bench_base2.err
