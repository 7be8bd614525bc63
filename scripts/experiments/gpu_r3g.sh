# Final round-3 profiles on the committed code: fp32 step trace + timeline, HBM bytes and
# LDS / MFMA counters of the fp32 step, IMPALA fp32 trace, driver-style bench + forced DP.
set -o pipefail
R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p $R/gpurun_out
timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r3g.json 2> gpurun_out/bench_r3g.err || exit 1
cat gpurun_out/bench_r3g.json
timeout -k 10 180 python -u bench.py --gpus 1 --steps 400 --warmup 40 --force-dp --no-bf16-extra > gpurun_out/bench_dp_r3g.json 2>> gpurun_out/bench_r3g.err || exit 1
timeout -k 10 180 python -u bench.py --gpus 1 --steps 400 --warmup 40 --no-bf16-extra > gpurun_out/bench_400_r3g.json 2>> gpurun_out/bench_r3g.err || exit 1
cat gpurun_out/bench_dp_r3g.json gpurun_out/bench_400_r3g.json
bash scripts/gpu_trace.sh r3gfp32 > /dev/null || exit 1
bash scripts/pmc_step_bytes.sh r3gbytes || exit 1
bash scripts/pmc_step.sh r3gpmc > /dev/null || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r3gimpala_fp32 -o run -- python $R/bench.py --network impala --dtype fp32 --steps 40 --warmup 10 --no-bf16-extra > $R/gpurun_out/r3gimpala_fp32.log 2>&1 || exit 1
cd $R && python scripts/prof_summary.py gpurun_out/r3gimpala_fp32 --steps 50 --top 40 > gpurun_out/r3gimpala_fp32.md 2>&1
timeout -k 10 240 python -u bench.py --network impala --steps 60 --warmup 10 > gpurun_out/bench_impala_r3g.json 2>> gpurun_out/bench_r3g.err || exit 1
cat gpurun_out/bench_impala_r3g.json
