# Actor inference as a HIP graph + pipelined actor groups: GPU tests, actor-step breakdown
# (pipeline 2 and 1), e2e loop (default fp32-class actors).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_runtime.py -k "pipelined or actor_q or loop" \
  > gpurun_out/pytest_r3l.log 2>&1 || { tail -30 gpurun_out/pytest_r3l.log; exit 1; }
tail -1 gpurun_out/pytest_r3l.log
timeout -k 10 240 python -u scripts/diag_e2e_actor.py --steps 4000 > gpurun_out/diag_e2e_pipe.log 2>&1 || { tail -20 gpurun_out/diag_e2e_pipe.log; exit 1; }
tail -n 8 gpurun_out/diag_e2e_pipe.log
timeout -k 10 240 python -u scripts/diag_e2e_actor.py --steps 4000 --set Runtime.actor_pipeline=1 > gpurun_out/diag_e2e_p1.log 2>&1 || { tail -20 gpurun_out/diag_e2e_p1.log; exit 1; }
tail -n 8 gpurun_out/diag_e2e_p1.log
timeout -k 10 300 python -u main.py --params-file configs/pong_1gpu.json --mode gpu --learner-steps 8000 \
    --set Runtime.ckpt_dir= --set Runtime.log_every=500 \
    --metrics gpurun_out/r3_e2e_pong_fp32_pipelined.jsonl > gpurun_out/r3_e2e_p.log 2>&1 || { tail -20 gpurun_out/r3_e2e_p.log; exit 1; }
python scripts/e2e_summary.py gpurun_out/r3_e2e_pong_fp32_pipelined.jsonl | tail -2
timeout -k 10 300 python -u main.py --params-file configs/pong_1gpu.json --mode gpu --learner-steps 8000 \
    --set Runtime.ckpt_dir= --set Runtime.log_every=500 --set Runtime.actor_pipeline=1 \
    --metrics gpurun_out/r3_e2e_pong_fp32_graph_p1.jsonl > gpurun_out/r3_e2e_p1.log 2>&1 || { tail -20 gpurun_out/r3_e2e_p1.log; exit 1; }
python scripts/e2e_summary.py gpurun_out/r3_e2e_pong_fp32_graph_p1.jsonl | tail -2
