set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; export TMPDIR=/tmp
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fc -o run -- python3 $R/scripts/bench_split_gemm.py > $R/gpurun_out/pmc_fc.log 2>&1 || exit 1
cd $R && python scripts/pmc_summary.py gpurun_out/pmc_fc > gpurun_out/pmc_fc.md 2>&1
