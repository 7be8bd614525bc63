set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
python -c "from apex_dqn_amd.ops import build; build.build_all()" > gpurun_out/build13.log 2>&1 || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof13k -o run -- python $R/scripts/bench_kernels.py --iters 20 > $R/gpurun_out/prof13k.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof13s -o run -- python $R/bench.py --steps 200 --warmup 20 > $R/gpurun_out/prof13s.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $R/gpurun_out/pmc13 -o run -- python $R/scripts/bench_kernels.py --iters 2 > $R/gpurun_out/pmc13.log 2>&1
rc=$?; echo "rc=$rc"; cd $R
python scripts/prof_summary.py gpurun_out/prof13k --top 40 > gpurun_out/prof13k.md 2>&1
python scripts/prof_summary.py gpurun_out/prof13s --steps 220 --top 40 > gpurun_out/prof13s.md 2>&1
cat gpurun_out/prof13k.md; cat gpurun_out/prof13s.md; exit $rc
