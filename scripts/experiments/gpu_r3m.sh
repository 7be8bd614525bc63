# Relaunch-after-append actor pipeline: tests + e2e; then the headline bench (driver-style),
# fp32 and bf16 step traces of the current code.
set -o pipefail
R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p $R/gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_runtime.py -k "pipelined or actor_q or loop" \
  > gpurun_out/pytest_r3m.log 2>&1 || { tail -30 gpurun_out/pytest_r3m.log; exit 1; }
tail -1 gpurun_out/pytest_r3m.log
timeout -k 10 300 python -u main.py --params-file configs/pong_1gpu.json --mode gpu --learner-steps 8000 \
    --set Runtime.ckpt_dir= --set Runtime.log_every=500 \
    --metrics gpurun_out/r3_e2e_pong_fp32_pipelined2.jsonl > gpurun_out/r3_e2e_p2.log 2>&1 || { tail -20 gpurun_out/r3_e2e_p2.log; exit 1; }
python scripts/e2e_summary.py gpurun_out/r3_e2e_pong_fp32_pipelined2.jsonl | tail -2
timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r3m.json 2> gpurun_out/bench_r3m.err || exit 1
cat gpurun_out/bench_r3m.json
timeout -k 10 180 python -u bench.py --gpus 1 --steps 400 --warmup 40 > gpurun_out/bench_400_r3m.json 2>> gpurun_out/bench_r3m.err || exit 1
cat gpurun_out/bench_400_r3m.json
bash scripts/gpu_trace.sh r3mfp32 > /dev/null || exit 1
bash scripts/gpu_trace.sh r3mbf16 "--dtype bf16" > /dev/null || exit 1
head -16 gpurun_out/r3mbf16_timeline.txt
