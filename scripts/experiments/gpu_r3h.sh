# Optimizer-written conv12 fragments: GPU tests (bit identity vs the pack launch, the split
# suite, runtime graph / resume tests), then a same-box A/B vs the pack launch and forced DP.
set -o pipefail
R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p $R/gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_split.py -k optimizer_stores \
  > gpurun_out/pytest_r3h.log 2>&1 || { tail -30 gpurun_out/pytest_r3h.log; exit 1; }
tail -3 gpurun_out/pytest_r3h.log
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_runtime.py tests/test_gpu_trajectory.py tests/test_gpu_kernels.py \
  > gpurun_out/pytest_r3h_rt.log 2>&1 || { tail -30 gpurun_out/pytest_r3h_rt.log; exit 1; }
tail -3 gpurun_out/pytest_r3h_rt.log
AB_STEPS=600 AB_WARMUP=50 bash scripts/ab.sh optfrags "APEX_OPT_FRAGS=1 :: --no-bf16-extra" "APEX_OPT_FRAGS=0 :: --no-bf16-extra" \
  "APEX_OPT_FRAGS=1 :: --no-bf16-extra --force-dp" "APEX_OPT_FRAGS=0 :: --no-bf16-extra --force-dp"
