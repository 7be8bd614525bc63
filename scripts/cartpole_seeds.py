#!/usr/bin/env python
"""CartPole learning over seeds for both IS-weight normalisations:
the CPU inline loop (C++ CartPole dynamics, MLP dueling DQN, host prioritized replay)
for each Runtime.is_normalise in (batch_max, global_min) and each seed, recording the
last-20-episode mean return and the mean IS weight the updates were scaled by
(the weight multiplies the loss, so it is the factor on the effective learning rate).
Random policy ~22.  Usage (CPU):
    python scripts/cartpole_seeds.py --seeds 1,2,3 --updates 2500 --out profiles/r3_cartpole_seeds.json
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def cfg_for(mode: str, seed: int):
    from apex_dqn_amd.config import ApexConfig
    return ApexConfig.from_dict({
        "env_conf": {"state_shape": [4], "action_dim": 2, "name": "CartPole-v1"},
        "Actor": {"num_actors": 4, "num_steps": 3, "Q_network_sync_freq": 50, "n_step_transition_batch_size": 8},
        "Learner": {"min_replay_mem_size": 300, "replay_sample_size": 64, "q_target_sync_freq": 100,
                    "remove_old_xp_freq": 50},
        "Replay_Memory": {"soft_capacity": 5000},
        "Runtime": {"lr": 1e-3, "log_every": 100, "seed": seed, "is_normalise": mode}})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", default="1,2,3")
    ap.add_argument("--updates", type=int, default=2500)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    from apex_dqn_amd.replay import host_replay
    from apex_dqn_amd.runtime.loops import train_inline
    seen = []
    orig = host_replay.PrioritizedReplay.sample

    def sample(self, *args, **kw):      # record the IS weights every update used
        out = orig(self, *args, **kw)
        seen.append(float(np.mean(out["weights"])))
        return out

    host_replay.PrioritizedReplay.sample = sample
    runs = []
    for mode in ("batch_max", "global_min"):
        for seed in [int(s) for s in a.seeds.split(",")]:
            torch.manual_seed(seed)
            seen.clear()
            out = train_inline(cfg_for(mode, seed), a.updates, actor_steps_per_update=1)
            r = {"is_normalise": mode, "seed": seed, "mean_return_last20": out["mean_return_last"],
                 "episodes": len(out["episodes"]), "is_weight_mean": float(np.mean(seen)) if seen else None}
            runs.append(r)
            print(json.dumps(r), flush=True)
    summ = {}
    for mode in ("batch_max", "global_min"):
        rs = [r for r in runs if r["is_normalise"] == mode]
        summ[mode] = {"return_mean": float(np.mean([r["mean_return_last20"] for r in rs])),
                      "return_std": float(np.std([r["mean_return_last20"] for r in rs])),
                      "is_weight_mean": float(np.mean([r["is_weight_mean"] for r in rs]))}
    print(json.dumps(summ), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"what": "CartPole-v1 inline learning, 3 seeds x IS normalisation; random policy ~22",
                       "updates": a.updates, "summary": summ, "runs": runs}, f, indent=1)


if __name__ == "__main__":
    main()
