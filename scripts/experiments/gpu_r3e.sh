# Round-3 profiles: fp32 / bf16 step traces + timelines, per-kernel HBM bytes, LDS / MFMA
# counters of the fp32 step, IMPALA fp32 (split) and bf16 step traces.
set -o pipefail
R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p $R/gpurun_out
bash scripts/gpu_trace.sh r3fp32 || exit 1
bash scripts/gpu_trace.sh r3bf16 "--dtype bf16" > /dev/null || exit 1
bash scripts/pmc_step_bytes.sh r3bytes || exit 1
bash scripts/pmc_step.sh r3pmc > /dev/null || exit 1
for dt in fp32 bf16; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r3impala_$dt -o run -- python $R/bench.py --network impala --dtype $dt --steps 40 --warmup 10 --no-bf16-extra > $R/gpurun_out/r3impala_$dt.log 2>&1 || exit 1
  cd $R && python scripts/prof_summary.py gpurun_out/r3impala_$dt --steps 50 --top 40 > gpurun_out/r3impala_$dt.md 2>&1
done
head -12 gpurun_out/r3impala_fp32.md

timeout -k 10 180 python -u bench.py --gpus 1 --steps 200 --warmup 20 --force-dp --no-bf16-extra > gpurun_out/bench_dp_r3e.json 2> gpurun_out/bench_dp_r3e.err || exit 1
cat gpurun_out/bench_dp_r3e.json
