# HBM bytes per kernel of the learner step (rocprofv3 counters, run through gpurun):
# FETCH_SIZE / WRITE_SIZE (KB per dispatch) + L2 hit/miss, eager steps (no graphs: the
# counter passes serialise dispatches anyway).  Usage: bash scripts/pmc_step_bytes.sh TAG [bench args]
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=$1; EXTRA=${2:-}
mkdir -p $R/gpurun_out; export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --kernel-trace --output-format csv -d $R/gpurun_out/pmc_${TAG}_a -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-graphs --no-bf16-extra $EXTRA > $R/gpurun_out/pmc_${TAG}_a.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE TCC_MISS_sum --kernel-trace --output-format csv -d $R/gpurun_out/pmc_${TAG}_b -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-graphs --no-bf16-extra $EXTRA > $R/gpurun_out/pmc_${TAG}_b.log 2>&1 || exit 1
cd $R && python scripts/pmc_summary.py gpurun_out/pmc_${TAG}_a gpurun_out/pmc_${TAG}_b > gpurun_out/pmc_${TAG}.md 2>&1
