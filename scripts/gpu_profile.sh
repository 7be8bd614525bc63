# rocprofv3 evidence (run through gpurun): a kernel trace of the bench step and
# per-kernel counters of the GEMM microbenchmarks (counters in their own run,
# never combined with runtime/sys traces).  Usage: bash scripts/gpu_profile.sh TAG
set -o pipefail
TAG=${1:-prof}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "from apex_dqn_amd.ops import build; build.build_all()" > gpurun_out/build_$TAG.log 2>&1 || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_step -o run -- python3 $R/bench.py --steps 200 --warmup 20 > $R/gpurun_out/${TAG}_step.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_pmc_a -o run -- python3 $R/scripts/bench_kernels.py --iters 2 > $R/gpurun_out/${TAG}_pmc_a.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_pmc_b -o run -- python3 $R/scripts/bench_kernels.py --iters 2 > $R/gpurun_out/${TAG}_pmc_b.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_pmc_c -o run -- python3 $R/scripts/bench_kernels.py --iters 2 > $R/gpurun_out/${TAG}_pmc_c.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_pmc_d -o run -- python3 $R/scripts/bench_kernels.py --iters 2 > $R/gpurun_out/${TAG}_pmc_d.log 2>&1
rc=$?; echo "rc=$rc"; cd $R
python scripts/prof_summary.py gpurun_out/${TAG}_step --steps 220 --top 30 > gpurun_out/${TAG}_step.md 2>&1
python scripts/pmc_summary.py gpurun_out/${TAG}_pmc_a gpurun_out/${TAG}_pmc_b gpurun_out/${TAG}_pmc_c gpurun_out/${TAG}_pmc_d > gpurun_out/${TAG}_pmc.md 2>&1
cat gpurun_out/${TAG}_step.md gpurun_out/${TAG}_pmc.md
exit $rc
