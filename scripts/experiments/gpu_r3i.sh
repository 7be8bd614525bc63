# bf16 fused conv1 -> conv2 forward: GPU tests (fused bf16 kernel vs fp64 and the separate
# kernels, optimizer fragment stores, whole-step / trajectory oracles), then a same-box A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p $R/gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread tests/test_gpu_split.py -k "bf16 or optimizer_stores or conv12 or whole_step" \
  > gpurun_out/pytest_r3i.log 2>&1 || { tail -40 gpurun_out/pytest_r3i.log; exit 1; }
grep "bf16 conv2 output\|passed\|failed" gpurun_out/pytest_r3i.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_trajectory.py tests/test_gpu_runtime.py \
  > gpurun_out/pytest_r3i_rt.log 2>&1 || { tail -40 gpurun_out/pytest_r3i_rt.log; exit 1; }
tail -2 gpurun_out/pytest_r3i_rt.log
AB_STEPS=600 AB_WARMUP=50 bash scripts/ab.sh c12bf16 "APEX_CONV12_BF16=1 :: --dtype bf16 --no-bf16-extra" "APEX_CONV12_BF16=0 :: --dtype bf16 --no-bf16-extra"
