# Final check: full GPU suite, then the driver-style bench on the committed tree.
set -o pipefail
bash scripts/gpu_suite.sh r3ab || exit 1
timeout -k 10 180 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r3ab.json 2> gpurun_out/bench_r3ab.err || exit 1
tail -1 gpurun_out/bench_r3ab.json | cut -c1-300
timeout -k 10 180 python -u bench.py --gpus 1 --steps 400 --warmup 40 > gpurun_out/bench_r3ab_400.json 2>> gpurun_out/bench_r3ab.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/bench_r3ab_400.json').read().strip().splitlines()[-1]); print(d['value'], d.get('value_bf16'))"
