# Build -> GPU tests -> bench x2 -> kernel trace + one-step timeline (run through gpurun).
# Usage: bash scripts/gpu_iter.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-iter}
K=${2:-}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "from apex_dqn_amd.ops import build; build.build_all()" > gpurun_out/build_$TAG.log 2>&1 || { tail gpurun_out/build_$TAG.log; exit 1; }
if [ -n "$K" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/pytest_$TAG.log 2>&1
else
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
fi
rc=$?; tail -5 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 600 --warmup 50 > gpurun_out/bench_${TAG}_$i.log 2>&1 || { tail gpurun_out/bench_${TAG}_$i.log; exit 1; }
  cut -c1-230 gpurun_out/bench_${TAG}_$i.log | tail -1
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_step -o run -- python $R/bench.py --steps 200 --warmup 20 > $R/gpurun_out/${TAG}_step.log 2>&1 || exit 1
cd $R
python scripts/prof_summary.py gpurun_out/${TAG}_step --steps 220 --top 30 > gpurun_out/${TAG}_step.md 2>&1
python scripts/step_timeline.py gpurun_out/${TAG}_step/run_kernel_trace.csv > gpurun_out/${TAG}_timeline.txt 2>&1
cat gpurun_out/${TAG}_timeline.txt
