# IMPALA split kernels + work-queue tests, headline bench (queue off), IMPALA fp32 bench,
# CU-steal proxy with the queue on (forced-DP learner) and off.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_impala_split.py tests/test_impala.py tests/test_gpu_split.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r3b.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed|impala split step" gpurun_out/pytest_r3b.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r3b.json 2> gpurun_out/bench_r3b.err || exit 1
cat gpurun_out/bench_r3b.json
timeout -k 10 240 python -u bench.py --network impala --steps 60 --warmup 10 > gpurun_out/bench_impala_r3b.json 2> gpurun_out/bench_impala_r3b.err || exit 1
cat gpurun_out/bench_impala_r3b.json
timeout -k 10 240 python -u bench.py --network impala --steps 40 --warmup 10 --graph-impala --no-bf16-extra > gpurun_out/bench_impala_graph_r3b.json 2> gpurun_out/bench_impala_graph_r3b.err || exit 1
cat gpurun_out/bench_impala_graph_r3b.json
APEX_WORK_QUEUE=1 timeout -k 10 240 python -u scripts/bench_cu_steal.py > gpurun_out/steal_wq_r3b.jsonl 2> gpurun_out/steal_wq_r3b.err || exit 1
cat gpurun_out/steal_wq_r3b.jsonl
APEX_WORK_QUEUE=0 timeout -k 10 240 python -u scripts/bench_cu_steal.py > gpurun_out/steal_static_r3b.jsonl 2> gpurun_out/steal_static_r3b.err || exit 1
cat gpurun_out/steal_static_r3b.jsonl
