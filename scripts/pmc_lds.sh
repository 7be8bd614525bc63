# LDS bank-conflict counters of the learner's image-resident conv kernels (bf16 path),
# one counter pass of scripts/bench_kernels.py (run through gpurun).
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; export TMPDIR=/tmp; TAG=${1:-lds}
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $R/gpurun_out/pmc_${TAG} -o run -- python3 $R/scripts/bench_kernels.py --iters 2 > $R/gpurun_out/pmc_${TAG}.log 2>&1 || exit 1
cd $R && python scripts/pmc_summary.py gpurun_out/pmc_${TAG} > gpurun_out/pmc_${TAG}.md 2>&1
