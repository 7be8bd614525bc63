#!/usr/bin/env python
"""Why does a learner variant not learn on fake_ale_target?  Runs the GPU loop (lock-step
actors, deterministic) for each variant and prints: the replay's reward statistics, the
actors' action histogram, q-value spread, episode returns, and the learner's loss /
|delta| -- side by side for the HIP (fp32 split) and torch-autograd learners.
    python scripts/diag_fake_ale.py [--steps 1500]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=1500)
    ap.add_argument("--variants", default="fp32,torch")
    ap.add_argument("--env", default="fake_ale_target")
    a = ap.parse_args()
    from apex_dqn_amd.actors import gpu_actor
    from apex_dqn_amd.config import ApexConfig
    from apex_dqn_amd.runtime.gpu_loop import train_frames
    V = {"fp32": {"dtype": "fp32"}, "bf16": {"dtype": "bf16"}, "torch": {"dtype": "fp32", "use_hip_kernels": False}}
    for v in a.variants.split(","):
        acts, qs = [], []
        orig = gpu_actor.GpuActorGroup.policy

        def policy(self, payload):
            q, act = orig(self, payload)
            acts.append(act.copy())
            qs.append(q.copy())
            return q, act

        gpu_actor.GpuActorGroup.policy = policy
        try:
            cfg = ApexConfig.from_dict({
                "env_conf": {"state_shape": [4, 84, 84], "action_dim": 6, "name": "FakeALE"},
                "Actor": {"num_actors": 128, "T": 10 ** 9, "num_steps": 3, "epsilon": 0.4, "alpha": 7, "gamma": 0.99,
                          "n_step_transition_batch_size": 128, "Q_network_sync_freq": 200},
                "Learner": {"remove_old_xp_freq": 100, "q_target_sync_freq": 1000, "min_replay_mem_size": 20000,
                            "replay_sample_size": 512},
                "Replay_Memory": {"soft_capacity": 200000, "priority_exponent": 0.6,
                                  "importance_sampling_exponent": 0.4},
                "Runtime": {**V[v], "seed": 1, "log_every": 0, "lr": 1e-4, "env_backend": a.env}})
            torch.manual_seed(1)
            out = train_frames(cfg, torch.device("cuda", 0), a.steps, async_actors=False)
        finally:
            gpu_actor.GpuActorGroup.policy = orig
        L, rp = out["learner"], out.get("replay") or out["learner"].replay
        n = int(rp.size()) if hasattr(rp, "size") else 0
        rew = rp.rew[:max(n, 1)].float().cpu().numpy()
        A = np.concatenate(acts[-50:]) if acts else np.zeros(1)
        Q = np.concatenate(qs[-50:]) if qs else np.zeros((1, 6))
        rets = [r for (_, _, r) in out["episodes"]]
        m = L.last_metrics()
        print(f"[{v}] learner={L.kind} replay={n} reward!=0 {np.mean(rew != 0):.3f} mean {rew.mean():.3f} | "
              f"actions(last 50 steps) {np.bincount(A.astype(int), minlength=6) / max(A.size, 1)} | "
              f"q mean {Q.mean():.3f} spread(max-min over a) {np.mean(Q.max(1) - Q.min(1)):.4f} | "
              f"episodes {len(rets)} return(last 50) {np.mean(rets[-50:]) if rets else float('nan'):.2f} | "
              f"loss {m.get('loss')} td {m.get('td_abs_mean', m.get('td_abs'))} isw {m.get('is_weight_mean')}",
              flush=True)


if __name__ == "__main__":
    main()
