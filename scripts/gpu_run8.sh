set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_conv.py -m gpu -q -x -k "conv1 or switch" > gpurun_out/pytest_gpu8.log 2>&1
rc=$?; echo "pytest conv1 rc=$rc"; tail -3 gpurun_out/pytest_gpu8.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_gpu8.log; exit 1; }
timeout -k 10 300 python scripts/bench_kernels.py --only conv1_fwd,conv1_wgrad > gpurun_out/kbench8.log 2>&1; grep op gpurun_out/kbench8.log
