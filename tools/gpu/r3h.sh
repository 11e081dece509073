mkdir -p gpurun_out/r3h
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
V=$R/pathtracing_amd/_lib/variants/libpt_hip_lds1.so
C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES"
timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "k_shade" --output-format csv -d $R/gpurun_out/r3h/base -o run -- python3 $R/bench.py --no-cpu-baseline --no-count --steps 1 --warmup 0 > $R/gpurun_out/r3h/base.log 2>&1 || exit $?
PT_HIP_LIB=$V timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "k_shade" --output-format csv -d $R/gpurun_out/r3h/lds1 -o run -- python3 $R/bench.py --no-cpu-baseline --no-count --steps 1 --warmup 0 > $R/gpurun_out/r3h/lds1.log 2>&1
