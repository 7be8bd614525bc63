# Final round-3 numbers on the committed tree: driver-style bench, 400/40, step trace.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_final_20.json 2> gpurun_out/bench_final.err || exit 1
tail -1 gpurun_out/bench_final_20.json
timeout -k 10 180 python -u bench.py --gpus 1 --steps 400 --warmup 40 > gpurun_out/bench_final_400.json 2>> gpurun_out/bench_final.err || exit 1
tail -1 gpurun_out/bench_final_400.json
bash scripts/gpu_trace.sh r3final > /dev/null || exit 1
head -16 gpurun_out/r3final_timeline.txt
