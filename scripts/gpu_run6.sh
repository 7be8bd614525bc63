set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/bench_kernels.py > gpurun_out/kbench6.log 2>&1; echo "kbench rc=$?"; cat gpurun_out/kbench6.log | grep op
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc6a -o run -- python $GRAFT_REPO_ROOT/scripts/bench_kernels.py --iters 3 > $GRAFT_REPO_ROOT/gpurun_out/pmc6a.log 2>&1; echo "pmc a rc=$?"
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc6b -o run -- python $GRAFT_REPO_ROOT/scripts/bench_kernels.py --iters 3 > $GRAFT_REPO_ROOT/gpurun_out/pmc6b.log 2>&1; echo "pmc b rc=$?"
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc6c -o run -- python $GRAFT_REPO_ROOT/scripts/bench_kernels.py --iters 3 > $GRAFT_REPO_ROOT/gpurun_out/pmc6c.log 2>&1; echo "pmc c rc=$?"
ls $GRAFT_REPO_ROOT/gpurun_out/pmc6a
