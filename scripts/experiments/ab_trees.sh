# A/B of two source trees (prebuilt in-tree): bench twice each, interleaved, then a kernel
# trace of each.  Usage: bash scripts/experiments/ab_trees.sh TAG OTHER_TREE [bench flags]
set -o pipefail
TAG=$1; OTHER=$2; shift 2
R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp
mkdir -p $R/gpurun_out
out=$R/gpurun_out/abt_$TAG.log; : > $out
for rep in 1 2; do
  for t in "$R" "$R/$OTHER"; do
    r=$(cd $t && timeout -k 10 200 python bench.py --steps 400 --warmup 40 --no-bf16-extra "$@" 2>/dev/null | tail -1) || { echo "FAIL $t" >> $out; exit 1; }
    echo "$t => $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $out
  done
done
cat $out
for t in "$R" "$R/$OTHER"; do
  n=$(basename $t)
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trace_${TAG}_$n -o run -- python $t/bench.py --steps 200 --warmup 20 --no-bf16-extra "$@" > $R/gpurun_out/trace_${TAG}_$n.log 2>&1 || exit 1
  cd $R && python scripts/prof_summary.py gpurun_out/trace_${TAG}_$n --steps 220 --top 30 > gpurun_out/trace_${TAG}_$n.md 2>&1
done
