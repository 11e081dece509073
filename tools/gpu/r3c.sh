mkdir -p gpurun_out/r3c
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3c/tests.txt 2>&1 || echo "TESTS FAILED rc=$?" >> gpurun_out/r3c/tests.txt
timeout -k 10 300 python -u tools/bitdiff.py gpurun_out/r3c/bd_base.json --c4 > gpurun_out/r3c/bd_base.txt 2>&1 &&
PT_HIP_LIB=pathtracing_amd/_lib/variants/libpt_hip_nocontract.so timeout -k 10 300 python -u tools/bitdiff.py gpurun_out/r3c/bd_nocontract.json --c4 > gpurun_out/r3c/bd_nocontract.txt 2>&1 &&
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r3c/bench.json 2> gpurun_out/r3c/bench.err
