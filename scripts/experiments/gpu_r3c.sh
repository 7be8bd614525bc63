# Multi-seed learning parity (fp32 split / bf16 / torch learner) on two envs, and the
# end-to-end loop with bf16 actor inference (Runtime.actor_precision) for comparison.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u main.py --params-file configs/pong_1gpu.json --mode gpu --learner-steps 8000 \
    --set Runtime.ckpt_dir= --set Runtime.log_every=500 --set Runtime.actor_precision=bf16 \
    --metrics gpurun_out/r3_e2e_pong_fp32_bf16actors.jsonl > gpurun_out/r3_e2e_b.log 2>&1 || { tail -20 gpurun_out/r3_e2e_b.log; exit 1; }
python scripts/e2e_summary.py gpurun_out/r3_e2e_pong_fp32_bf16actors.jsonl | tail -2
timeout -k 10 900 python -u scripts/learning_parity.py --env fake_ale_target --seeds 1,2,3 --variants fp32,bf16,torch \
    --steps 6000 --out gpurun_out/r3_learning_parity_fake_ale_target.json > gpurun_out/r3_lp_fake.log 2>&1 || { tail -20 gpurun_out/r3_lp_fake.log; exit 1; }
tail -1 gpurun_out/r3_lp_fake.log
timeout -k 10 900 python -u scripts/learning_parity.py --env synthetic --seeds 1,2,3 --variants fp32,bf16,torch \
    --steps 6000 --out gpurun_out/r3_learning_parity_synthetic.json > gpurun_out/r3_lp_syn.log 2>&1 || { tail -20 gpurun_out/r3_lp_syn.log; exit 1; }
tail -1 gpurun_out/r3_lp_syn.log
