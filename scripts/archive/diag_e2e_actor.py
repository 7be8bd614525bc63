#!/usr/bin/env python
"""Where does the end-to-end actor step's time go?  Runs the GPU loop (async actor thread,
the Pong-shaped config) and accumulates wall time per actor-step component -- policy
(inference kernels + the host wait for q / actions), env step, frame ingest, n-step
builder, replay insert -- and prints them with the learner's update rate.
    python scripts/diag_e2e_actor.py [--steps 3000] [--set Runtime.actor_precision=bf16]
"""
import argparse
import json
import os
import sys
import time
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--params", default="configs/pong_1gpu.json")
    ap.add_argument("--set", action="append", default=[])
    a = ap.parse_args()
    from apex_dqn_amd.actors import gpu_actor
    from apex_dqn_amd.config import ApexConfig
    from apex_dqn_amd.runtime.gpu_loop import train_frames
    with open(a.params) as f:
        d = json.load(f)
    d.setdefault("Runtime", {}).update({"ckpt_dir": "", "log_every": 0})
    for kv in a.set:
        k, v = kv.split("=", 1)
        sec, key = k.split(".", 1)
        try:
            v = json.loads(v)
        except ValueError:
            pass
        d.setdefault(sec, {})[key] = v
    cfg = ApexConfig.from_dict(d)
    T = defaultdict(float)
    N = defaultdict(int)
    G = gpu_actor.GpuActorGroup

    def timed(name, fn):
        def w(*args, **kw):
            t = time.perf_counter()
            r = fn(*args, **kw)
            T[name] += time.perf_counter() - t
            N[name] += 1
            return r
        return w

    orig = {k: getattr(G, k) for k in ("policy", "_ingest", "step", "launch_policy", "finish_step")}
    G.policy = timed("policy", orig["policy"])
    G._ingest = timed("ingest", orig["_ingest"])
    G.step = timed("group_step", orig["step"])
    G.launch_policy = timed("launch_policy", orig["launch_policy"])
    G.finish_step = timed("finish_step", orig["finish_step"])
    env_t = {}

    orig_reset = G.reset

    def reset(self):
        if self.env not in env_t:
            self.env.step = timed("env_step", self.env.step)
            self.builder.step = timed("nstep_builder", self.builder.step)
            env_t[self.env] = True
        if "insert" not in env_t:
            self.replay.insert = timed("replay_insert", self.replay.insert)
            env_t["insert"] = True
        return orig_reset(self)

    G.reset = reset
    torch.manual_seed(0)
    t0 = time.time()
    out = train_frames(cfg, torch.device("cuda", 0), a.steps)
    wall = time.time() - t0
    steps = out["actor_steps"]
    E = out["actors"].E
    groups = getattr(out["actors"], "groups", [out["actors"]])
    print(json.dumps({"learner_steps": a.steps, "wall_s": round(wall, 2), "actor_steps": steps, "E": E,
                      "groups": len(groups),
                      "env_frames_per_s_incl_fill": round(steps * E / wall)}))
    for k in sorted(T, key=lambda k: -T[k]):
        print(f"{k:15s} calls {N[k]:7d}  total {T[k]:8.2f} s  per call {1e3 * T[k] / max(N[k], 1):7.3f} ms")


if __name__ == "__main__":
    main()
