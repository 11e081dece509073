# overlapped traversal: iteration statistics and VALU counters (specE build)
set -e
mkdir -p gpurun_out/r3r
R=$GRAFT_REPO_ROOT
PT_HIP_LIB=pathtracing_amd/_lib/variants/libpt_hip_itersE.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-count --spp 256 --steps 1 --warmup 0 > gpurun_out/r3r/iters.json 2> gpurun_out/r3r/iters.err
cd /tmp && export TMPDIR=/tmp
L=$R/pathtracing_amd/_lib/variants/libpt_hip_specE.so
PT_HIP_LIB=$L timeout -s KILL 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/r3r/specE/sq -o run -- python3 $R/bench.py --no-cpu-baseline --no-count --spp 128 --steps 1 --warmup 0 > $R/gpurun_out/r3r/specE.sq.log 2>&1
PT_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r3r/specE/trace -o run -- python3 $R/bench.py --no-cpu-baseline --no-count --spp 128 --steps 1 --warmup 0 > $R/gpurun_out/r3r/specE.tr.log 2>&1
python3 $R/tools/pmc_summary.py $R/gpurun_out/r3r/specE $R/gpurun_out/r3r/specE.json > $R/gpurun_out/r3r/specE.txt
rm -rf $R/gpurun_out/r3r/specE
