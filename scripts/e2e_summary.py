"""Second-half mean learner grad-steps/s and env frames/s of a main.py metrics JSONL."""
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if '"kind": "learner"' in l]
h = rows[len(rows) // 2:]
k1 = [r for r in h if "grad_steps_per_s" in r]
print(json.dumps({"n_log": len(rows), "second_half_grad_steps_per_s": sum(r["grad_steps_per_s"] for r in k1) / max(1, len(k1)),
                  "second_half_env_frames_per_s": sum(r.get("env_frames_per_s", 0) for r in k1) / max(1, len(k1)),
                  "last_step": rows[-1]["step"]}))
