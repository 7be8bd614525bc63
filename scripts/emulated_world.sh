# bench.py --emulate-world W for W = 2, 4, 8 (fp32 + bf16 extra) and the single-rank step
# at the same per-rank rows; summarised into gpurun_out/emulated_world.json.  Run through gpurun.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
: > gpurun_out/emulated_world.jsonl
for W in 8 4 2; do
  timeout -k 10 300 python -u bench.py --emulate-world $W --steps ${EMU_STEPS:-400} --warmup 20 \
      2>> gpurun_out/emulated_world.err | tail -1 >> gpurun_out/emulated_world.jsonl || exit 1
  rows=$(tail -1 gpurun_out/emulated_world.jsonl | python -c 'import json,sys; print(json.loads(sys.stdin.read())["config"]["per_rank_rows"])')
  timeout -k 10 300 python -u bench.py --batch $rows --steps ${EMU_STEPS:-400} --warmup 20 \
      2>> gpurun_out/emulated_world.err | tail -1 >> gpurun_out/emulated_world.jsonl || exit 1
done
timeout -k 10 300 python -u bench.py --steps ${EMU_STEPS:-400} --warmup 20 2>> gpurun_out/emulated_world.err \
    | tail -1 >> gpurun_out/emulated_world.jsonl || exit 1
python - <<'PY'
import json
rows = [json.loads(l) for l in open("gpurun_out/emulated_world.jsonl") if l.strip()]
out = {"note": "bench.py --emulate-world W: rank 0's share of a W-rank global-batch DP step on one MI355X "
               "(collectives = device copies of their true sizes; RCCL latency and xGMI time not included), "
               "next to the single-rank step at the same rows per rank and at 512 rows",
       "runs": []}
for r in rows:
    out["runs"].append({"emulated_world": r.get("emulated_world"), "per_rank_rows": r["config"]["per_rank_rows"],
                        "fp32_steps_per_s": r["value"], "fp32_us_per_step": round(1e3 * r["ms_per_step"], 1),
                        "bf16_steps_per_s": r.get("value_bf16"),
                        "bf16_us_per_step": round(1e3 * r["ms_per_step_bf16"], 1) if r.get("ms_per_step_bf16") else None,
                        "dp_shard_update": r["config"].get("dp_shard_update"),
                        "dp_fc_exchange": r["config"].get("dp_fc_exchange"),
                        "rank0_rows_drawn_per_step": r.get("rank0_rows_drawn_per_step"),
                        "dp_graphs": r.get("dp_graphs")})
json.dump(out, open("gpurun_out/emulated_world.json", "w"), indent=1)
for x in out["runs"]:
    print(x)
PY
