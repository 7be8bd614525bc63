set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_conv.py tests/test_gpu_kernels.py -m gpu -q -s > gpurun_out/pytest_gpu4.log 2>&1
echo "pytest rc=$?"; grep -E "passed|failed|per-segment|Error|error" gpurun_out/pytest_gpu4.log | head -30
timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/bench4.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench3.log; exit 1; }
tail -1 gpurun_out/bench4.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof4 -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 30 --warmup 5 --no-graphs > $GRAFT_REPO_ROOT/gpurun_out/prof4.log 2>&1; echo "prof rc=$?"
