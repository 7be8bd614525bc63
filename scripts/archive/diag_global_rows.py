#!/usr/bin/env python
"""Diagnostic (torchrun, gloo, ranks may share one GPU): per-step rows of the
global-batch draw on bench.py's synthetic replay -- each rank's rows with IS weight > 0
and valid generation, and M / per-rank counts from the host mirror of the draw
(replay/gpu_replay.py global_draw) on the same gathered statistics."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from apex_dqn_amd.parallel.dist import Comm  # noqa: E402
from apex_dqn_amd.replay.gpu_replay import SHARD_STATS, global_draw  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)) % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    comm = Comm.from_env(backend="gloo", device=dev)
    args = bench.parser().parse_args(["--gpus", str(world), "--replay", "20000", "--dist-backend", "gloo"])
    replay = bench.make_replay(args, dev, rank)
    cfg, L = bench.make_learner(args, "fp32", dev, comm, rank, replay, "global")
    for t in range(30):
        if L._sample_ver != replay.version:
            L._sample()
        torch.cuda.synchronize()
        st = replay.shard_stats.double().cpu().numpy().reshape(world, SHARD_STATS)
        mir = [int(global_draw(st, r, L.B, replay.shard_seed, int(replay.ctr.item()), replay.shard_mcap)[1].sum())
               for r in range(world)]
        mine = torch.tensor(np.concatenate([st.reshape(-1), [float(replay.ctr.item())]]), dtype=torch.float64)
        allv = [torch.zeros_like(mine) for _ in range(world)]
        torch.distributed.all_gather(allv, mine)
        same = all(torch.equal(allv[0], a) for a in allv[1:])
        w = L.S["weights"]
        rec = dict(t=t, rank=rank, w_pos=int((w > 0).sum()), gen_ok=int((L.S["gen"] >= 0).sum()), mirror=mir,
                   share=[round(float(x), 4) for x in st[:, 0] / st[:, 0].sum()], stats_equal=same,
                   T=[float(x) for x in st[:, 0]], ctr=int(replay.ctr.item()))
        print(json.dumps(rec), flush=True)
        L.step()
    comm.shutdown()


if __name__ == "__main__":
    main()
