# Phase timing (in-kernel probes) and wall time of the fused conv1 -> conv2 forward, split and bf16.
set -o pipefail
mkdir -p gpurun_out
for v in "" "--bf16"; do
  echo "== split/bf16 flag: '$v' probe" >> gpurun_out/probe_c12.log
  timeout -k 10 120 python -u scripts/probe_conv12.py --probe $v >> gpurun_out/probe_c12.log 2>&1 || exit 1
  echo "== '$v' wall" >> gpurun_out/probe_c12.log
  timeout -k 10 120 python -u scripts/probe_conv12.py $v >> gpurun_out/probe_c12.log 2>&1 || exit 1
done
cat gpurun_out/probe_c12.log
