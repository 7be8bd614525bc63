set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
python -c "from apex_dqn_amd.ops import build; build.build_all()" > gpurun_out/build20.log 2>&1 &&
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu20.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 300 --warmup 30 > gpurun_out/bench20.log 2>&1 &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof20s -o run -- python $R/bench.py --steps 100 --warmup 20 > $R/gpurun_out/prof20s.log 2>&1
rc=$?; echo "rc=$rc"; cd $R
python scripts/prof_summary.py gpurun_out/prof20s --steps 120 --top 30 > gpurun_out/prof20s.md 2>&1
tail -3 gpurun_out/pytest_gpu20.log; tail -1 gpurun_out/bench20.log; cat gpurun_out/prof20s.md; exit $rc
