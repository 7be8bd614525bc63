# Per-kernel LDS / MFMA counters of the fp32 learner step (one rocprofv3 counter pass over
# a short bench run; run through gpurun).  Usage: bash scripts/pmc_step.sh [TAG] [bench args]
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; export TMPDIR=/tmp; TAG=${1:-step}; EXTRA=${2:-}
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d $R/gpurun_out/pmc_${TAG} -o run -- python3 $R/bench.py --steps 30 --warmup 10 --no-bf16-extra --prep-warm 0 $EXTRA > $R/gpurun_out/pmc_${TAG}.log 2>&1 || exit 1
cd $R && python scripts/pmc_summary.py gpurun_out/pmc_${TAG} > gpurun_out/pmc_${TAG}.md 2>&1
cat gpurun_out/pmc_${TAG}.md | head -40
