# conv1 epilogue: permlane16 swap + one 16-B LDS store per lane: tests, tree A/B both precisions.
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_split.py tests/test_gpu_runtime.py -k "conv12 or optimizer_stores or work_queue or whole_step or actor_q" \
  > gpurun_out/pytest_r3s.log 2>&1 || { tail -30 gpurun_out/pytest_r3s.log; exit 1; }
tail -1 gpurun_out/pytest_r3s.log
bash scripts/experiments/ab_trees.sh swp _abtree > /dev/null || exit 1
cat gpurun_out/abt_swp.log; grep conv12 gpurun_out/trace_swp_*.md
bash scripts/experiments/ab_trees.sh swpbf _abtree --dtype bf16 > /dev/null || exit 1
cat gpurun_out/abt_swpbf.log; grep conv12 gpurun_out/trace_swpbf_*.md
