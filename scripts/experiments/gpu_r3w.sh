# Kernel trace of the forced data-parallel step.
set -o pipefail
bash scripts/gpu_trace.sh r3wdp "--force-dp" > /dev/null || exit 1
cat gpurun_out/r3wdp_timeline.txt
