"""Learning-curve parity of the two learner precisions on the synthetic Atari env
(reward 1 when the action matches the hidden state drawn in the frame, random
policy ~1/A per step): the same config, seed and step budget trained with
Runtime.dtype = fp32 (split hi/lo operands, the reference's precision) and bf16,
mean episode return per log interval.  Usage (one GPU):
    python scripts/learning_parity.py [--steps 6000] [--out profiles/r2_learning_parity.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(dtype: str, steps: int, seed: int, async_actors: bool):
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
        "env_conf": {"state_shape": [4, 84, 84], "action_dim": 6, "name": "SyntheticPong"},
        "Actor": {"num_actors": 128, "T": 10 ** 9, "num_steps": 3, "epsilon": 0.4, "alpha": 7, "gamma": 0.99,
                  "n_step_transition_batch_size": 128, "Q_network_sync_freq": 200},
        "Learner": {"remove_old_xp_freq": 100, "q_target_sync_freq": 1000, "min_replay_mem_size": 20000,
                    "replay_sample_size": 512},
        "Replay_Memory": {"soft_capacity": 200000, "priority_exponent": 0.6, "importance_sampling_exponent": 0.4},
        "Runtime": {"dtype": dtype, "seed": seed, "log_every": 250, "lr": 1e-4}})
    m = Mem()
    out = train_frames(cfg, torch.device("cuda", 0), steps, metrics=m, async_actors=async_actors)
    curve = [(r["step"], r["mean_return"], r["loss"]) for r in m.rows if r["kind"] == "learner"]
    half = [c[1] for c in curve[len(curve) // 2:]]
    return {"dtype": dtype, "curve": curve, "final_mean_return": curve[-1][1] if curve else None,
            "mean_return_second_half": sum(half) / max(len(half), 1),
            "episodes": len(out["episodes"]), "actor_steps": out["actor_steps"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=6000)
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--lockstep", action="store_true", help="alternate actor / learner (deterministic schedule)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    res = [run(dt, a.steps, a.seed, not a.lockstep) for dt in ("fp32", "bf16")]
    summary = {"what": "learning-curve parity fp32 (split) vs bf16 on SyntheticPong (A=6, random ~ 1/6 reward "
                       "per step)", "steps": a.steps, "seed": a.seed, "runs": res}
    print(json.dumps({r["dtype"]: r["mean_return_second_half"] for r in res}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()
