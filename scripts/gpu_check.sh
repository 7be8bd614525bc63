# One GPU verification pass (run through gpurun): build, GPU tests, kernel
# microbenchmarks, the headline bench.  Usage: bash scripts/gpu_check.sh TAG
set -o pipefail
TAG=${1:-check}
mkdir -p gpurun_out
python -c "from apex_dqn_amd.ops import build; build.build_all()" > gpurun_out/build_$TAG.log 2>&1 &&
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_$TAG.log 2>&1 &&
timeout -k 10 200 python scripts/bench_kernels.py --iters 50 > gpurun_out/kern_$TAG.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 300 --warmup 30 > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; cat gpurun_out/kern_$TAG.log; tail -1 gpurun_out/bench_$TAG.log
exit $rc
