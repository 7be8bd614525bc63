# Split conv2 data gradient with the copy-out overlapped: tests, tree A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_split.py tests/test_gpu_conv.py -k "dgrad or image_resident or work_queue or whole_step" \
  > gpurun_out/pytest_r3u.log 2>&1 || { tail -30 gpurun_out/pytest_r3u.log; exit 1; }
tail -1 gpurun_out/pytest_r3u.log
bash scripts/experiments/ab_trees.sh dgov _abtree > /dev/null || exit 1
cat gpurun_out/abt_dgov.log; grep conv2_dgrad gpurun_out/trace_dgov_*.md
