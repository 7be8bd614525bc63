set -o pipefail
out=gpurun_out/warm_ab.log; : > $out
for rep in 1 2; do
for v in "--steps 20 --warmup 5 --prep-warm 0" "--steps 20 --warmup 5 --prep-warm 4" "--steps 400 --warmup 40 --prep-warm 0" "--steps 20 --warmup 5 --prep-warm 20"; do
  r=$(timeout -k 10 200 python bench.py $v --no-bf16-extra 2>/dev/null | tail -1) || { echo "FAIL $v" >> $out; exit 1; }
  echo "$v => $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("prep_warm_replays"))')" >> $out
done; done
cat $out
