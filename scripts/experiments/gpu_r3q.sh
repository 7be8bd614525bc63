# Scratch-free fused forward (frame slots as vector values; bf16 copy-out rounds) + actors on
# the fused forward: tests, tree A/B in both precisions, e2e.
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread tests/test_gpu_split.py tests/test_gpu_runtime.py -k "conv12 or optimizer_stores or work_queue or whole_step or actor or loop" \
  > gpurun_out/pytest_r3q.log 2>&1 || { tail -30 gpurun_out/pytest_r3q.log; exit 1; }
grep "actor q-values\|passed\|failed" gpurun_out/pytest_r3q.log | tail -4
bash scripts/experiments/ab_trees.sh c12scratch _abtree > /dev/null || exit 1
cat gpurun_out/abt_c12scratch.log; grep conv12 gpurun_out/trace_c12scratch_*.md
bash scripts/experiments/ab_trees.sh c12scratchbf _abtree --dtype bf16 > /dev/null || exit 1
cat gpurun_out/abt_c12scratchbf.log; grep conv12 gpurun_out/trace_c12scratchbf_*.md
timeout -k 10 300 python -u main.py --params-file configs/pong_1gpu.json --mode gpu --learner-steps 8000 \
    --set Runtime.ckpt_dir= --set Runtime.log_every=500 \
    --metrics gpurun_out/r3_e2e_pong_fp32_actor_c12.jsonl > gpurun_out/r3_e2e_c12.log 2>&1 || { tail -20 gpurun_out/r3_e2e_c12.log; exit 1; }
python scripts/e2e_summary.py gpurun_out/r3_e2e_pong_fp32_actor_c12.jsonl | tail -1
