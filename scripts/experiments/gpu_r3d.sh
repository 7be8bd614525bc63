# Full GPU suite + driver-style bench (optimizer-launch pack tail), then scripts/experiments/gpu_r3c.sh.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_r3d.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/pytest_r3d.log | head -5; tail -1 gpurun_out/pytest_r3d.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r3d.json 2> gpurun_out/bench_r3d.err || exit 1
cat gpurun_out/bench_r3d.json
timeout -k 10 180 python -u bench.py --gpus 1 --steps 400 --warmup 40 --no-bf16-extra > gpurun_out/bench_r3d_400.json 2>> gpurun_out/bench_r3d.err || exit 1
cat gpurun_out/bench_r3d_400.json
bash scripts/experiments/gpu_r3c.sh
