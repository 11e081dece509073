# VALU issue share of the traversal kernels: one counter pass + one trace pass
# per build (committed scheduling off = sched0 variant, and PT_SCHED=1)
set -e
mkdir -p gpurun_out/r3o
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 -L > $R/gpurun_out/r3o/counters.txt 2>&1 || true
for v in sched0 base; do
  if [ $v = base ]; then L=$R/pathtracing_amd/_lib/libpt_hip.so; else L=$R/pathtracing_amd/_lib/variants/libpt_hip_$v.so; fi
  PT_HIP_LIB=$L timeout -s KILL 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/r3o/$v/sq -o run -- python3 $R/bench.py --no-cpu-baseline --no-count --spp 128 --steps 1 --warmup 0 > $R/gpurun_out/r3o/$v.sq.log 2>&1
  PT_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r3o/$v/trace -o run -- python3 $R/bench.py --no-cpu-baseline --no-count --spp 128 --steps 1 --warmup 0 > $R/gpurun_out/r3o/$v.tr.log 2>&1
  python3 $R/tools/pmc_summary.py $R/gpurun_out/r3o/$v $R/gpurun_out/r3o/$v.json > $R/gpurun_out/r3o/$v.txt
  rm -rf $R/gpurun_out/r3o/$v
done
