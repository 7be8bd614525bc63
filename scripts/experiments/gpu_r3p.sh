# Spill-free split conv2 data gradient (two pixel-tile passes): tests, then a tree A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_split.py -k "dgrad or image_resident or work_queue or whole_step" \
  > gpurun_out/pytest_r3p.log 2>&1 || { tail -30 gpurun_out/pytest_r3p.log; exit 1; }
tail -1 gpurun_out/pytest_r3p.log
bash scripts/experiments/ab_trees.sh dgradsplit _abtree
grep conv2_dgrad gpurun_out/trace_dgradsplit_*.md
