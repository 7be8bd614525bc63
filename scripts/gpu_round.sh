# One gpurun call: GPU test suite, driver-style bench (20/5), forced-DP bench and the
# CU-stealing proxy. Every GPU step has its own time limit; the first failure ends the call.
# Usage: bash scripts/gpu_round.sh TAG [pytest selection, default: tests]
set -o pipefail
TAG=${1:-round}; SEL=${2:-tests}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
cat gpurun_out/bench_$TAG.json
timeout -k 10 180 python -u bench.py --gpus 1 --steps 200 --warmup 20 --force-dp --no-bf16-extra > gpurun_out/bench_dp_$TAG.json 2> gpurun_out/bench_dp_$TAG.err || exit 1
cat gpurun_out/bench_dp_$TAG.json
timeout -k 10 240 python -u scripts/bench_cu_steal.py > gpurun_out/steal_$TAG.jsonl 2> gpurun_out/steal_$TAG.err || exit 1
cat gpurun_out/steal_$TAG.jsonl
