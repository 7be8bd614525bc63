# A/B bench variants in one GPU call: each argument is one variant,
# "VAR=1 VAR2=x :: --bench-flag ..." (env before ::, bench flags after).
# Usage: bash scripts/ab.sh TAG "variant1" "variant2" ...   (each run twice, interleaved)
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
python -c "from apex_dqn_amd.ops import build; build.build_all()" > gpurun_out/build_$TAG.log 2>&1 || exit 1
out=gpurun_out/ab_$TAG.log
: > $out
for rep in 1 2; do
  for v in "$@"; do
    envs="${v%%::*}"; flags="${v#*::}"; [ "$envs" = "$v" ] && flags=""
    r=$(env $envs timeout -k 10 200 python bench.py --steps ${AB_STEPS:-600} --warmup ${AB_WARMUP:-50} $flags 2>/dev/null | tail -1) || { echo "FAIL $v" >> $out; exit 1; }
    echo "$v => $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $out
  done
done
cat $out
