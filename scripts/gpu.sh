# One parameterised runner for GPU work (run through gpurun).  Every GPU step has its
# own time limit and writes under gpurun_out/; chain steps with && so the first failure
# ends the call.
#
#   bash scripts/gpu.sh build                          # content-addressed build check (no recompiles expected)
#   bash scripts/gpu.sh test TAG [SEL] [-k EXPR]       # pytest -m gpu (default SEL: tests)
#   bash scripts/gpu.sh bench TAG [bench.py args]      # one bench.py run -> gpurun_out/bench_TAG.json
#   bash scripts/gpu.sh sweep TAG [sweep args]         # scripts/bench_batch_sweep.py (step time vs rows per rank)
#   bash scripts/gpu.sh trace TAG [bench.py args]      # rocprofv3 kernel trace + per-kernel table + one-step timeline
#   bash scripts/gpu.sh pmc TAG COUNTERS [bench args]  # one rocprofv3 --pmc pass (<= 8 SQ counters), summarised
#   bash scripts/gpu.sh ab TAG "ENV=1 :: --flag" ...   # interleaved A/B of bench variants (each twice)
#   bash scripts/gpu.sh steal TAG                      # CU-steal proxy of the DP step (scripts/bench_cu_steal.py)
#   bash scripts/gpu.sh e2e TAG [main.py --set args]   # actor + learner loop, Pong-shaped config
#   bash scripts/gpu.sh py TAG SCRIPT [args]           # any python script under a 300 s limit
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
cmd=$1; shift
case "$cmd" in
build)
  timeout -k 10 900 python -c "
from apex_dqn_amd.ops import build
stale = [w for w in ('runtime', 'comm', 'kernels', 'kernels_debug') if build.library_stale(w)]
print('stale libraries before build:', stale)
build.build_all()" > gpurun_out/build.log 2>&1
  rc=$?; cat gpurun_out/build.log; exit $rc ;;
test)
  TAG=$1; shift; SEL=${1:-tests}; [ $# -gt 0 ] && shift
  timeout -k 10 1000 python -u -m pytest $SEL -m gpu -x -v --timeout 240 --timeout-method thread \
      -p no:cacheprovider "$@" > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"
  grep -E "FAILED|ERROR" gpurun_out/pytest_$TAG.log | head -20
  tail -2 gpurun_out/pytest_$TAG.log; exit $rc ;;
bench)
  TAG=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
  rc=$?; cat gpurun_out/bench_$TAG.json; [ $rc -eq 0 ] || tail -20 gpurun_out/bench_$TAG.err; exit $rc ;;
sweep)
  TAG=$1; shift
  timeout -k 10 900 python -u scripts/bench_batch_sweep.py --out gpurun_out/sweep_$TAG.json "$@" \
      > gpurun_out/sweep_$TAG.log 2>&1
  rc=$?; cat gpurun_out/sweep_$TAG.log | tail -30; exit $rc ;;
trace)
  TAG=$1; shift
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_step -o run -- \
      python3 $R/bench.py --steps 200 --warmup 20 --no-bf16-extra "$@" > $R/gpurun_out/${TAG}_step.log 2>&1 || exit 1
  cd $R
  python scripts/prof_summary.py gpurun_out/${TAG}_step --steps 220 --top 40 > gpurun_out/${TAG}_step.md 2>&1
  python scripts/step_timeline.py gpurun_out/${TAG}_step/run_kernel_trace.csv > gpurun_out/${TAG}_timeline.txt 2>&1
  cat gpurun_out/${TAG}_timeline.txt | head -60 ;;
pmc)
  TAG=$1; CNT=$2; shift 2
  cd /tmp
  timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d $R/gpurun_out/${TAG}_pmc -o run -- \
      python3 $R/bench.py --steps 50 --warmup 10 --no-bf16-extra "$@" > $R/gpurun_out/${TAG}_pmc.log 2>&1 || exit 1
  cd $R
  python scripts/pmc_summary.py gpurun_out/${TAG}_pmc > gpurun_out/${TAG}_pmc.md 2>&1; head -40 gpurun_out/${TAG}_pmc.md ;;
ab)
  TAG=$1; shift
  out=gpurun_out/ab_$TAG.log; : > $out
  for rep in 1 2; do
    for v in "$@"; do
      envs="${v%%::*}"; flags="${v#*::}"; [ "$envs" = "$v" ] && flags=""
      r=$(env $envs timeout -k 10 150 python bench.py --steps ${AB_STEPS:-600} --warmup ${AB_WARMUP:-50} $flags \
          2>>gpurun_out/ab_$TAG.err | tail -1) || { echo "FAIL $v" >> $out; cat $out; exit 1; }
      echo "$v => $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("value_bf16"))')" >> $out
    done
  done
  cat $out ;;
steal)
  TAG=$1
  timeout -k 10 300 python -u scripts/bench_cu_steal.py > gpurun_out/steal_$TAG.jsonl 2> gpurun_out/steal_$TAG.err
  rc=$?; cat gpurun_out/steal_$TAG.jsonl; exit $rc ;;
e2e)
  TAG=$1; shift
  timeout -k 10 400 python -u main.py --params-file configs/pong_1gpu.json --mode gpu \
      --learner-steps ${E2E_STEPS:-8000} --metrics gpurun_out/e2e_$TAG.jsonl --set Runtime.log_every=500 "$@" \
      > gpurun_out/e2e_$TAG.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/e2e_$TAG.log; exit $rc; }
  python scripts/e2e_summary.py gpurun_out/e2e_$TAG.jsonl ;;
py)
  TAG=$1; shift
  timeout -k 10 300 python -u "$@" > gpurun_out/py_$TAG.log 2>&1
  rc=$?; tail -40 gpurun_out/py_$TAG.log; exit $rc ;;
*)
  echo "unknown step: $cmd"; exit 2 ;;
esac
