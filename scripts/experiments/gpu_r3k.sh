# Actor-step time breakdown of the end-to-end loop (fp32-class actors, then bf16 actors).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u scripts/diag_e2e_actor.py --steps 4000 > gpurun_out/diag_e2e_fp32.log 2>&1 || { tail -20 gpurun_out/diag_e2e_fp32.log; exit 1; }
timeout -k 10 240 python -u scripts/diag_e2e_actor.py --steps 4000 --set Runtime.actor_precision=bf16 > gpurun_out/diag_e2e_bf16.log 2>&1 || { tail -20 gpurun_out/diag_e2e_bf16.log; exit 1; }
tail -9 gpurun_out/diag_e2e_fp32.log gpurun_out/diag_e2e_bf16.log
