set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu5.log 2>&1
echo "pytest rc=$?"; grep -E "passed|failed|Error" gpurun_out/pytest_gpu5.log | head -20; tail -5 gpurun_out/pytest_gpu5.log
