# Full GPU test suite on one MI355X (run through gpurun), then the headline bench.
# Usage: bash scripts/gpu_suite.sh TAG [pytest selection, default: tests]
set -o pipefail
TAG=${1:-suite}; SEL=${2:-tests}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest $SEL -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"
grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_$TAG.log | grep -v PASSED | head -20
tail -2 gpurun_out/pytest_$TAG.log
exit $rc
