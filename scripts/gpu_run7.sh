set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_conv.py -m gpu -q -x > gpurun_out/pytest_gpu7.log 2>&1
rc=$?; echo "pytest conv rc=$rc"; grep -E "passed|failed|Error" gpurun_out/pytest_gpu7.log | head -20
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_gpu7.log; exit 1; }
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu7b.log 2>&1 || { echo "all gpu failed"; tail -30 gpurun_out/pytest_gpu7b.log; exit 1; }
tail -1 gpurun_out/pytest_gpu7b.log
timeout -k 10 300 python scripts/bench_kernels.py > gpurun_out/kbench7.log 2>&1; grep op gpurun_out/kbench7.log
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench7.log 2>&1; tail -1 gpurun_out/bench7.log
