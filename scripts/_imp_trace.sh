set -o pipefail
R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/imp6 -o run -- python $R/bench.py --network impala --steps 60 --warmup 10 > $R/gpurun_out/imp6.log 2>&1 || exit 1
cd $R
python scripts/prof_summary.py gpurun_out/imp6 --steps 70 --top 40 > gpurun_out/imp6.md 2>&1
python scripts/step_timeline.py gpurun_out/imp6/run_kernel_trace.csv "void sconv_fwd_kernel" > gpurun_out/imp6_timeline.txt 2>&1
cat gpurun_out/imp6.md
