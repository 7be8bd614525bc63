# Kernel trace of the headline bench + per-kernel summary + one-step timeline (run through gpurun).
# Usage: bash scripts/gpu_trace.sh TAG [extra bench.py args, e.g. "--dtype bf16"]
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=$1; EXTRA=${2:-}
mkdir -p gpurun_out; export TMPDIR=/tmp
python -c "from apex_dqn_amd.ops import build; build.build_all()" > gpurun_out/build_$TAG.log 2>&1 || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_step -o run -- python $R/bench.py --steps 200 --warmup 20 --no-bf16-extra $EXTRA > $R/gpurun_out/${TAG}_step.log 2>&1 || exit 1
cd $R
python scripts/prof_summary.py gpurun_out/${TAG}_step --steps 220 --top 30 > gpurun_out/${TAG}_step.md 2>&1
python scripts/step_timeline.py gpurun_out/${TAG}_step/run_kernel_trace.csv > gpurun_out/${TAG}_timeline.txt 2>&1
cat gpurun_out/${TAG}_timeline.txt
