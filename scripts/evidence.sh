# Round-end evidence on one GPU (run through gpurun): driver-command bench, longer bench,
# emulated W = 2 / 4 / 8 rank steps with the single-rank step at the same rows, the step's
# PMC pass (LDS conflicts / MFMA busy; EV_NO_PMC=1 skips it), IMPALA, forced DP at world 1.  Each GPU step under its own limit, chained.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/ev; export TMPDIR=/tmp
b() { timeout -k 10 300 python -u bench.py "$@"; }
b --gpus 1 --steps 20 --warmup 5 > gpurun_out/ev/bench_20_5.json 2> gpurun_out/ev/bench_20_5.err && \
b --steps 200 --warmup 20 > gpurun_out/ev/bench_200.json 2> gpurun_out/ev/bench_200.err && \
for W in 2 4 8; do
  b --steps 400 --warmup 40 --emulate-world $W --no-bf16-extra > gpurun_out/ev/emu_w$W.json 2>> gpurun_out/ev/emu.err || exit 1
  rows=$(python -c "import json; print(json.load(open('gpurun_out/ev/emu_w$W.json'))['config']['per_rank_rows'])")
  b --steps 400 --warmup 40 --batch $rows --no-bf16-extra > gpurun_out/ev/single_rows$rows.json 2>> gpurun_out/ev/emu.err || exit 1
  b --steps 400 --warmup 40 --emulate-world $W --no-bf16-extra --dtype bf16 > gpurun_out/ev/emu_w${W}_bf16.json 2>> gpurun_out/ev/emu.err || exit 1
done && \
b --steps 200 --warmup 20 --network impala > gpurun_out/ev/bench_impala.json 2> gpurun_out/ev/bench_impala.err && \
b --steps 400 --warmup 40 --force-dp --no-bf16-extra > gpurun_out/ev/bench_forced_dp.json 2> gpurun_out/ev/bench_forced_dp.err && \
{ [ -n "$EV_NO_PMC" ] || { bash scripts/pmc_step.sh ev > /dev/null && python scripts/pmc_util.py gpurun_out/pmc_ev > gpurun_out/ev/pmc_lds_mfma.md; }; }
rc=$?; for f in gpurun_out/ev/*.json; do echo "$f $(python -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d.get('value_bf16'))")"; done; exit $rc
