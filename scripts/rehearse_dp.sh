# Rehearse the multi-rank bench on ONE GPU (run through gpurun): 2 ranks over gloo
# (RCCL refuses two ranks on one device) through the exact torchrun launch the
# driver uses for N>1 -- DP step segments, bucketed all-reduces, IS-normaliser
# MIN all-reduce, eviction cadence, max-over-ranks timing.  Numbers are NOT a
# scaling measurement (both ranks share one GPU and gloo stages through the host).
# Usage: bash scripts/rehearse_dp.sh [N]   (N ranks, default 2)
set -o pipefail
N=${1:-2}
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus $N --steps 60 --warmup 10 --dist-backend gloo > gpurun_out/rehearse_dp.log 2>&1
rc=$?; tail -3 gpurun_out/rehearse_dp.log; exit $rc
