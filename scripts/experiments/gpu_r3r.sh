# Full GPU suite on the current tree, then the fp32 step's LDS / MFMA counters.
set -o pipefail
bash scripts/gpu_suite.sh r3r || exit 1
bash scripts/pmc_step.sh r3rpmc > /dev/null || exit 1
head -20 gpurun_out/pmc_r3rpmc.md
