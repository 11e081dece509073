set -o pipefail
mkdir -p gpurun_out/r4a
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r4a/gpu_tests.txt 2>&1
echo "tests rc=$?" >> gpurun_out/r4a/gpu_tests.txt
timeout -k 10 500 python bench.py --steps 3 --warmup 1 > gpurun_out/r4a/bench.json 2> gpurun_out/r4a/bench.err || exit $?
timeout -k 10 300 python bench.py --shard 0/8 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r4a/shard8.json 2> gpurun_out/r4a/shard8.err || exit $?
timeout -k 10 300 python bench.py --shard 0/2 --steps 2 --warmup 1 --no-cpu-baseline --no-count > gpurun_out/r4a/shard2.json 2> gpurun_out/r4a/shard2.err
