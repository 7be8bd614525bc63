# grad_finalize with all 16 partial loads in flight: tests, tree A/B both precisions.
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_split.py tests/test_gpu_trajectory.py tests/test_gpu_kernels.py -k "whole_step or trajectory or wgrad or finalize or norm" \
  > gpurun_out/pytest_r3t.log 2>&1 || { tail -30 gpurun_out/pytest_r3t.log; exit 1; }
tail -1 gpurun_out/pytest_r3t.log
bash scripts/experiments/ab_trees.sh gfin _abtree > /dev/null || exit 1
cat gpurun_out/abt_gfin.log; grep grad_finalize gpurun_out/trace_gfin_*.md
bash scripts/experiments/ab_trees.sh gfinbf _abtree --dtype bf16 > /dev/null || exit 1
cat gpurun_out/abt_gfinbf.log; grep grad_finalize gpurun_out/trace_gfinbf_*.md
