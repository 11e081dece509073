mkdir -p gpurun_out/r3f
V=pathtracing_amd/_lib/variants/libpt_hip_lds.so
PT_HIP_LIB=$V timeout -k 10 300 python -u tools/bitdiff.py gpurun_out/r3f/bd_lds.json > gpurun_out/r3f/bd_lds.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3f/bench_base.json 2> gpurun_out/r3f/bench_base.err || exit $?
PT_HIP_LIB=$V timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3f/bench_lds.json 2> gpurun_out/r3f/bench_lds.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --steps 2 > gpurun_out/r3f/bench_base2.json 2> gpurun_out/r3f/bench_base2.err
timeout -k 10 400 python3 tools/fetch_calib.py gpurun_out/r3f/fetch_calib.json > gpurun_out/r3f/fetch_calib.log 2>&1
