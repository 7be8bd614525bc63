set -o pipefail
mkdir -p gpurun_out
python -c "from apex_dqn_amd.ops import build; build.build_all()" > gpurun_out/build17.log 2>&1 &&
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu17.log 2>&1 &&
timeout -k 10 200 python scripts/bench_kernels.py --iters 50 > gpurun_out/kern17.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 300 --warmup 30 > gpurun_out/bench17.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/pytest_gpu17.log; cat gpurun_out/kern17.log; tail -2 gpurun_out/bench17.log; exit $rc
