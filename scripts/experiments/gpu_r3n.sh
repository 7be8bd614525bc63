# Peeled optimizer fragment stores (75 VGPRs): bit-identity tests, A/B vs the pack launch;
# actor relaunch A/B on one box.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_split.py -k "optimizer_stores or rmsprop" \
  > gpurun_out/pytest_r3n.log 2>&1 || { tail -30 gpurun_out/pytest_r3n.log; exit 1; }
tail -1 gpurun_out/pytest_r3n.log
AB_STEPS=600 AB_WARMUP=50 bash scripts/ab.sh optfrags2 "APEX_OPT_FRAGS=1 :: --no-bf16-extra" "APEX_OPT_FRAGS=0 :: --no-bf16-extra" \
  "APEX_OPT_FRAGS=1 :: --dtype bf16 --no-bf16-extra" "APEX_OPT_FRAGS=0 :: --dtype bf16 --no-bf16-extra"
for v in 0 1; do
  APEX_ACTOR_RELAUNCH=$v timeout -k 10 300 python -u main.py --params-file configs/pong_1gpu.json --mode gpu --learner-steps 8000 \
    --set Runtime.ckpt_dir= --set Runtime.log_every=500 \
    --metrics gpurun_out/r3_e2e_relaunch$v.jsonl > gpurun_out/r3_e2e_r$v.log 2>&1 || { tail -20 gpurun_out/r3_e2e_r$v.log; exit 1; }
  echo "relaunch=$v $(python scripts/e2e_summary.py gpurun_out/r3_e2e_relaunch$v.jsonl | tail -1)"
done
