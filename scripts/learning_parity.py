"""Learning-curve parity of the learner variants: the same config, seeds and step budget
trained with
  fp32   Runtime.dtype = fp32 on the HIP kernels (split hi/lo operands, the reference's
         precision),
  bf16   Runtime.dtype = bf16 on the HIP kernels,
  torch  the torch-autograd learner on MIOpen / hipBLASLt in fp32 (use_hip_kernels off),
on
  synthetic        Atari-shaped frames, reward 1 when the action matches the hidden state
                   drawn in the frame (random policy ~1/A per step),
  fake_ale_target  the full DQN wrapper stack (frame skip 4 + max-pool, no-op starts,
                   episodic life, reward clipping, 84x84 gray) over FakeALE in target
                   mode: reward only while the block is in the right third of the screen.
Mean episode return per log interval; the summary is the second-half mean per run and
its mean / std over seeds per variant.  Usage (one GPU):
    python scripts/learning_parity.py --env fake_ale_target --seeds 1,2,3 --out profiles/x.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


VARIANTS = {"fp32": {"dtype": "fp32"}, "bf16": {"dtype": "bf16"},
            "torch": {"dtype": "fp32", "use_hip_kernels": False}}


def run(variant: str, steps: int, seed: int, async_actors: bool, env: str = "synthetic"):
    import torch
    from apex_dqn_amd.config import ApexConfig
    from apex_dqn_amd.runtime.gpu_loop import train_frames
    from apex_dqn_amd.utils.metrics import MetricsLogger

    class Mem(MetricsLogger):
        def __init__(self):
            self.rows = []

        def log(self, kind, **kw):
            self.rows.append(dict(kind=kind, **kw))

        def episode(self, *a, **k):
            pass

        def close(self):
            pass

    cfg = ApexConfig.from_dict({
        "env_conf": {"state_shape": [4, 84, 84], "action_dim": 6,
                     "name": "SyntheticPong" if env == "synthetic" else "FakeALE"},
        "Actor": {"num_actors": 128, "T": 10 ** 9, "num_steps": 3, "epsilon": 0.4, "alpha": 7, "gamma": 0.99,
                  "n_step_transition_batch_size": 128, "Q_network_sync_freq": 200},
        "Learner": {"remove_old_xp_freq": 100, "q_target_sync_freq": 1000, "min_replay_mem_size": 20000,
                    "replay_sample_size": 512},
        "Replay_Memory": {"soft_capacity": 200000, "priority_exponent": 0.6, "importance_sampling_exponent": 0.4},
        "Runtime": {**VARIANTS[variant], "seed": seed, "log_every": 250, "lr": 1e-4, "env_backend": env}})
    m = Mem()
    out = train_frames(cfg, torch.device("cuda", 0), steps, metrics=m, async_actors=async_actors)
    curve = [(r["step"], r["mean_return"], r["loss"]) for r in m.rows if r["kind"] == "learner"]
    half = [c[1] for c in curve[len(curve) // 2:]]
    isw = [r.get("is_weight_mean") for r in m.rows if r["kind"] == "learner"]
    return {"variant": variant, "env": env, "seed": seed, "curve": curve, "is_weight_mean_last": isw[-1] if isw else None, "final_mean_return": curve[-1][1] if curve else None,
            "mean_return_second_half": sum(half) / max(len(half), 1),
            "episodes": len(out["episodes"]), "actor_steps": out["actor_steps"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=6000)
    ap.add_argument("--seeds", default="3")
    ap.add_argument("--variants", default="fp32,bf16")
    ap.add_argument("--env", default="synthetic", choices=["synthetic", "fake_ale_target"])
    ap.add_argument("--lockstep", action="store_true", help="alternate actor / learner (deterministic schedule)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import numpy as np
    res = []
    for seed in [int(x) for x in a.seeds.split(",")]:
        for v in a.variants.split(","):
            r = run(v, a.steps, seed, not a.lockstep, a.env)
            res.append(r)
            print(json.dumps({"variant": v, "seed": seed, "second_half": r["mean_return_second_half"],
                              "final": r["final_mean_return"], "is_weight_mean": r["is_weight_mean_last"]}),
                  flush=True)
    per = {}
    for v in a.variants.split(","):
        xs = [r["mean_return_second_half"] for r in res if r["variant"] == v]
        per[v] = {"mean": float(np.mean(xs)), "std": float(np.std(xs)), "runs": xs}
    summary = {"what": f"learning-curve parity ({a.variants}) on {a.env}", "steps": a.steps, "seeds": a.seeds,
               "summary": per, "runs": res}
    print(json.dumps(per), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()
