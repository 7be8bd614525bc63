# Lock-step learning parity on the final tree (fake_ale_target, 3 seeds; fp32 / bf16 / torch).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u scripts/learning_parity.py --env fake_ale_target --seeds 1,2,3 --variants fp32,bf16,torch \
    --steps 3000 --lockstep --out gpurun_out/r3_learning_parity_lockstep_final.json > gpurun_out/r3_lp_final.log 2>&1 || { tail -20 gpurun_out/r3_lp_final.log; exit 1; }
tail -3 gpurun_out/r3_lp_final.log
