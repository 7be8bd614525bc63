# Forced data-parallel step (world 1, RCCL process group) in both precisions vs single rank.
set -o pipefail
mkdir -p gpurun_out
for a in "" "--force-dp"; do
  timeout -k 10 200 python -u bench.py --steps 400 --warmup 40 $a > gpurun_out/bench_r3v$a.json 2>> gpurun_out/bench_r3v.err || { tail -20 gpurun_out/bench_r3v.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_r3v$a.json').read().strip().splitlines()[-1]); print('$a', d['value'], d.get('value_bf16'), d['config']['parallelism'], d['config'].get('dp_collectives'))"
done
