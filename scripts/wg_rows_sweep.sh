# fp32 step rate vs the split-K rows of the conv3 / conv2 weight gradients
# (APEX_WG_ROWS3 / APEX_WG_ROWS2; 0 = ops/conv.py default, tuned on the bf16 step)
set -o pipefail
out=gpurun_out/wg_rows_sweep.log; : > $out
for rep in 1 2; do
for v in "0 0" "256 0" "320 0" "0 512" "0 576" "${WG_EXTRA:-0 0}"; do
  set -- $v
  r=$(APEX_WG_ROWS3=$1 APEX_WG_ROWS2=$2 timeout -k 10 200 python bench.py --steps 400 --warmup 40 --no-bf16-extra 2>/dev/null | tail -1) || { echo "FAIL $v" >> $out; exit 1; }
  echo "rows3=$1 rows2=$2 => $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $out
done; done
cat $out
