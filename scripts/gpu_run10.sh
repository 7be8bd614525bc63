set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc10 -o run -- python $GRAFT_REPO_ROOT/scripts/bench_kernels.py --iters 2 > $GRAFT_REPO_ROOT/gpurun_out/pmc10.log 2>&1; echo "pmc rc=$?"
