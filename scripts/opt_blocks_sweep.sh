# fp32 step rate vs the optimizer launch shape (APEX_OPT_THREADS x APEX_OPT_BLOCKS;
# default 512 x 512, tuned on the bf16 step)
set -o pipefail
out=gpurun_out/opt_blocks_sweep.log; : > $out
for rep in 1 2; do
for v in "512 512" "1024 256" "1024 512" "512 1024" "256 2048" "512 768"; do
  set -- $v
  r=$(APEX_OPT_THREADS=$1 APEX_OPT_BLOCKS=$2 timeout -k 10 200 python bench.py --steps 400 --warmup 40 --no-bf16-extra 2>/dev/null | tail -1) || { echo "FAIL $v" >> $out; exit 1; }
  echo "threads=$1 blocks=$2 => $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $out
done; done
cat $out
