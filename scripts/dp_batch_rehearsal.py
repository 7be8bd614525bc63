"""How often does the global-batch DP draw shrink below replay_sample_size?

A 2-rank end-to-end rehearsal on ONE GPU (gloo carries the collectives; RCCL refuses two
ranks on one device): actor groups on the fake-ALE emulator behind the full Atari
wrapper stack, the interleaved epsilon ladder over both ranks, one global prioritized
replay sharded over the ranks, the global-batch DP learner (runtime/gpu_loop.py, lock-step
actors).  Every update's global batch M (the rows both ranks drew) and the largest
shard's share of the priority mass are recorded, with the adaptive row buffer
(``Runtime.dp_rows_adaptive``) off and on.

    python scripts/dp_batch_rehearsal.py --updates 3000 --out gpurun_out/dp_batch_M.jsonl
"""
import argparse
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, world, path, q, updates, adaptive, slack):
    import numpy as np
    import torch
    from apex_dqn_amd.config import ApexConfig
    from apex_dqn_amd.learner.fused_learner import FusedNatureLearner
    from apex_dqn_amd.parallel.dist import Comm
    from apex_dqn_amd.replay.gpu_replay import SHARD_STATS
    from apex_dqn_amd.runtime.gpu_loop import train_frames
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comm = Comm.init(rank, world, f"file://{path}", backend="gloo", device=dev)
    cfg = ApexConfig.from_dict({
        "env_conf": {"state_shape": [4, 84, 84], "action_dim": 6, "name": "PongNoFrameskip-v4"},
        "Actor": {"num_actors": 64 * world, "T": 10 ** 9, "n_step_transition_batch_size": 64, "Q_network_sync_freq": 400},
        "Learner": {"remove_old_xp_freq": 100, "q_target_sync_freq": 2500, "min_replay_mem_size": 6000,
                    "replay_sample_size": 512},
        "Replay_Memory": {"soft_capacity": 60000},
        "Runtime": {"env_backend": "fake_ale", "async_actors": False, "log_every": 0, "seed": 11,
                    "dp_rows_adaptive": adaptive, "dp_batch_slack": slack}})
    rec = []
    orig = FusedNatureLearner.step

    def step(self):
        before = int(self.valid_rows_total.item())
        orig(self)
        rows = int(self.valid_rows_total.item()) - before
        T = self.replay.shard_stats.double().reshape(self.world, SHARD_STATS)[:, 0].cpu().numpy()
        rec.append((rows, float(T.max() / max(T.sum(), 1e-30)), int(self.B)))
    FusedNatureLearner.step = step
    out = train_frames(cfg, dev, updates, comm=comm, actor_steps_per_update=1)
    L = out["learner"]
    q.put((rank, rec, int(getattr(L, "rows_resized", 0))))
    comm.shutdown()


def run(updates, adaptive, slack, world=2):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with tempfile.TemporaryDirectory() as td:
        procs = [ctx.Process(target=worker, args=(r, world, os.path.join(td, "store"), q, updates, adaptive, slack))
                 for r in range(world)]
        for p in procs:
            p.start()
        res = sorted([q.get(timeout=1800) for _ in range(world)])
        for p in procs:
            p.join(timeout=120)
            assert p.exitcode == 0, p.exitcode
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--updates", type=int, default=3000)
    ap.add_argument("--slack", type=float, default=0.125)
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--modes", default="off,on", help="adaptive row buffer off / on")
    ap.add_argument("--out", default="gpurun_out/dp_batch_M.jsonl")
    args = ap.parse_args()
    import threading
    import time
    import numpy as np

    def beat():
        t0 = time.time()
        while True:
            time.sleep(30)
            print(f"... {time.time() - t0:.0f} s", flush=True)
    threading.Thread(target=beat, daemon=True).start()
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as f:
        for adaptive in [m == "on" for m in args.modes.split(",")]:
            res = run(args.updates, adaptive, args.slack, args.world)
            n = min(len(r[1]) for r in res)
            M = np.array([sum(r[1][i][0] for r in res) for i in range(n)])
            share = np.array([res[0][1][i][1] for i in range(n)])
            rows = np.array([res[0][1][i][2] for i in range(n)])
            vals, cnt = np.unique(M, return_counts=True)
            row = {"adaptive": adaptive, "world": args.world, "replay_sample_size": 512, "dp_batch_slack": args.slack,
                   "updates": int(n), "M_hist": {str(int(v)): int(c) for v, c in zip(vals, cnt)},
                   "frac_M_below_512": float((M < 512).mean()), "M_min": int(M.min()), "M_mean": float(M.mean()),
                   "max_shard_share": {"p50": float(np.percentile(share, 50)), "p99": float(np.percentile(share, 99)),
                                       "max": float(share.max())},
                   "rows_per_rank": {"first": int(rows[0]), "last": int(rows[-1])},
                   "row_buffer_resizes": int(res[0][2])}
            f.write(json.dumps(row) + "\n")
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
