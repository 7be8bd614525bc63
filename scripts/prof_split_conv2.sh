set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; export TMPDIR=/tmp
cd $R && timeout -k 10 120 python scripts/bench_split_conv2.py > gpurun_out/split_c2.log 2>&1 || exit 1
cd /tmp
for ONLY in fwd dgrad; do
export ONLY
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_${ONLY}_a -o run -- python3 $R/scripts/bench_split_conv2.py > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_${ONLY}_b -o run -- python3 $R/scripts/bench_split_conv2.py > /dev/null 2>&1 || exit 1
done
cd $R; python scripts/pmc_summary.py gpurun_out/pmc_fwd_a gpurun_out/pmc_fwd_b gpurun_out/pmc_dgrad_a gpurun_out/pmc_dgrad_b > gpurun_out/pmc_split.md 2>&1
