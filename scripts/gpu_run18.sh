set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
python -c "from apex_dqn_amd.ops import build; build.build_all()" > gpurun_out/build18.log 2>&1 || exit 1
cd /tmp
ONLY=conv3_wgrad,conv2_wgrad,conv1_wgrad,fc_wgrad,conv2_wgrad@1024,conv2_wgrad@256
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof18k -o run -- python $R/scripts/bench_kernels.py --iters 10 --only $ONLY > $R/gpurun_out/prof18k.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $R/gpurun_out/pmc18a -o run -- python $R/scripts/bench_kernels.py --iters 2 --only $ONLY > $R/gpurun_out/pmc18a.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY --kernel-trace --output-format csv -d $R/gpurun_out/pmc18b -o run -- python $R/scripts/bench_kernels.py --iters 2 --only $ONLY > $R/gpurun_out/pmc18b.log 2>&1
rc=$?; echo "rc=$rc"; cd $R
python scripts/prof_summary.py gpurun_out/prof18k --top 20 > gpurun_out/prof18k.md 2>&1
cat gpurun_out/prof18k.md; tail -3 gpurun_out/pmc18b.log; exit $rc
