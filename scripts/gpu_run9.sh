set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/exp_conv1.py > gpurun_out/exp9.log 2>&1; grep slots gpurun_out/exp9.log
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc9a -o run -- python $GRAFT_REPO_ROOT/scripts/bench_kernels.py --only conv1_fwd --iters 2 > $GRAFT_REPO_ROOT/gpurun_out/pmc9a.log 2>&1; echo "pmc a rc=$?"
timeout -k 10 300 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc9b -o run -- python $GRAFT_REPO_ROOT/scripts/bench_kernels.py --only conv1_fwd --iters 2 > $GRAFT_REPO_ROOT/gpurun_out/pmc9b.log 2>&1; echo "pmc b rc=$?"
