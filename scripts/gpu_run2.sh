set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -m gpu -x -q -s > gpurun_out/pytest_gpu2.log 2>&1
echo "pytest rc=$?"; grep -E "passed|failed|per-segment" gpurun_out/pytest_gpu2.log
timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/bench2.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench2.log; exit 1; }
tail -2 gpurun_out/bench2.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-graphs > gpurun_out/bench2_nograph.log 2>&1; echo "nograph rc=$?"; tail -1 gpurun_out/bench2_nograph.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof2 -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 30 --warmup 5 --no-graphs > $GRAFT_REPO_ROOT/gpurun_out/prof2.log 2>&1; echo "prof rc=$?"
find $GRAFT_REPO_ROOT/gpurun_out/prof2 -name "*stats*" | head
