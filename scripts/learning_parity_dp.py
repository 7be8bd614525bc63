"""Learning-curve parity of the sharded global-batch DP update (learner/dp_step.py).

The round-3 single-rank parity runs (scripts/learning_parity.py --env fake_ale_target
--lockstep: 3,000 updates, 3 seeds, fp32 89.9 +- 1.2 / bf16 90.5 +- 3.0 / torch
90.6 +- 3.6, profiles/r3_learning_parity_fake_ale_target_lockstep_final_tree.json)
re-run with W data-parallel ranks rehearsed on ONE GPU (gloo carries the collectives;
RCCL refuses two ranks on one device): the same config -- 128 fake-ALE actors in total
(128 / W per rank, the epsilon ladder interleaved over the ranks), one global prioritized
replay of the same capacity sharded over the ranks, 512-sample global batches (each rank
computes its rows), the sharded fc update, the factored exchange, lock-step actors (one
actor-group step per update on every rank, so env frames per update match the
single-rank runs).  Rank 0 logs the mean episode return of its envs and the loss.

    python scripts/learning_parity_dp.py --world 2 --seeds 1,2,3 --out gpurun_out/parity_dp_w2.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, world, path, q, steps, seed, variant):
    import torch
    from apex_dqn_amd.config import ApexConfig
    from apex_dqn_amd.parallel.dist import Comm
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

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comm = Comm.init(rank, world, f"file://{path}", backend="gloo", device=dev)
    cfg = ApexConfig.from_dict({
        "env_conf": {"state_shape": [4, 84, 84], "action_dim": 6, "name": "FakeALE"},
        "Actor": {"num_actors": 128, "T": 10 ** 9, "num_steps": 3, "epsilon": 0.4, "alpha": 7, "gamma": 0.99,
                  "n_step_transition_batch_size": 128, "Q_network_sync_freq": 200},
        "Learner": {"remove_old_xp_freq": 100, "q_target_sync_freq": 1000, "min_replay_mem_size": 20000,
                    "replay_sample_size": 512},
        "Replay_Memory": {"soft_capacity": 200000, "priority_exponent": 0.6, "importance_sampling_exponent": 0.4},
        "Runtime": {"dtype": variant, "seed": seed, "log_every": 250, "lr": 1e-4, "env_backend": "fake_ale_target",
                    "async_actors": False}})
    m = Mem() if rank == 0 else None
    t0 = time.time()
    out = train_frames(cfg, dev, steps, comm=comm, metrics=m, actor_steps_per_update=1, async_actors=False)
    L = out["learner"]
    res = None
    if rank == 0:
        curve = [(r["step"], r["mean_return"], r["loss"], r.get("valid_rows")) for r in m.rows if r["kind"] == "learner"]
        half = [c[1] for c in curve[len(curve) // 2:]]
        res = {"world": world, "variant": variant, "seed": seed, "curve": curve,
               "final_mean_return": curve[-1][1] if curve else None,
               "mean_return_second_half": sum(half) / max(len(half), 1),
               "episodes_rank0": len(out["episodes"]), "actor_steps": out["actor_steps"],
               "rows_per_rank": int(L.B), "sharded_fc_update": bool(getattr(L, "_shard", False)),
               "fc_exchange": "factors" if getattr(L, "_fc_factors", False) else "allreduce",
               "rows_resized": int(getattr(L, "rows_resized", 0)), "wall_s": round(time.time() - t0, 1)}
    q.put((rank, res))
    comm.shutdown()


def run_one(world, steps, seed, variant):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    path = os.path.join(tempfile.mkdtemp(), "store")
    ps = [ctx.Process(target=worker, args=(r, world, path, q, steps, seed, variant)) for r in range(world)]
    for p in ps:
        p.start()
    got = {}
    import queue
    t0 = time.time()
    while len(got) < world:
        try:
            r, res = q.get(timeout=50)
            got[r] = res
        except queue.Empty:
            # (a heartbeat: a GPU command that prints nothing for minutes is taken for hung)
            print(f"  ... world {world} seed {seed}: {time.time() - t0:.0f} s", flush=True)
            if time.time() - t0 > 1800:
                raise SystemExit("timed out")
            if any(p.exitcode not in (None, 0) for p in ps):
                raise SystemExit("a rank died")
    for p in ps:
        p.join(timeout=120)
        if p.exitcode != 0:
            raise SystemExit(f"rank exited with {p.exitcode}")
    return got[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--seeds", default="1,2,3")
    ap.add_argument("--variant", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import numpy as np
    res = []
    for seed in [int(x) for x in a.seeds.split(",")]:
        r = run_one(a.world, a.steps, seed, a.variant)
        res.append(r)
        print(json.dumps({k: r[k] for k in ("world", "seed", "mean_return_second_half", "final_mean_return",
                                            "rows_per_rank", "sharded_fc_update", "wall_s")}), flush=True)
        if a.out:
            with open(a.out, "w") as f:
                json.dump({"partial": True, "runs": res}, f)
    xs = [r["mean_return_second_half"] for r in res]
    summary = {"what": f"learning-curve parity of the sharded global-batch DP update, W = {a.world} ranks on one "
                       f"GPU (gloo), fake_ale_target, lock-step, {a.variant}",
               "steps": a.steps, "seeds": a.seeds,
               "summary": {"mean": float(np.mean(xs)), "std": float(np.std(xs)), "runs": xs},
               "single_rank_reference": "profiles/r3_learning_parity_fake_ale_target_lockstep_final_tree.json: "
                                        "fp32 89.85 +- 1.22 (88.9 / 89.1 / 91.6), bf16 90.5 +- 3.0, torch 90.6 +- 3.6",
               "runs": res}
    print(json.dumps(summary["summary"]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()
