# Effective shader clock per kernel of the learner step: GRBM_GUI_ACTIVE (GPU-busy
# cycles) over the traced kernel duration.  Usage: bash scripts/pmc_clock.sh TAG [bench args]
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=$1; EXTRA=${2:-}
mkdir -p $R/gpurun_out; export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $R/gpurun_out/pmc_clk_${TAG} -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-graphs --no-bf16-extra $EXTRA > $R/gpurun_out/pmc_clk_${TAG}.log 2>&1 || exit 1
