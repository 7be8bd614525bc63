#!/usr/bin/env python
"""Ape-X launcher (reference ``main.py``: ``python main.py --params-file parameters.json``).

Modes (``--mode``, default ``auto``):
  gpu        one process per GPU (launch N>1 with torchrun); each rank runs an
             actor group + HBM replay shard + fused learner; data-parallel over RCCL.
  multiproc  the reference topology on CPU: N actor processes feed the learner
             process (CartPole / MLP configs).
  inline     actors, replay and learner in one process (debugging).
``auto`` picks ``gpu`` for image configs on a GPU host, else ``multiproc``.

Examples:
  python main.py                                   # reference parameters.json
  python main.py --params-file configs/cartpole.json
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 main.py --params-file configs/breakout_8gpu.json
  python main.py --set Learner.replay_sample_size=512 --set Runtime.learner_T=10000
"""
from __future__ import annotations

import argparse
import json
import os
import sys

# HIP maps every stream to one of GPU_MAX_HW_QUEUES hardware queues (4 by default); the
# learner's two step streams, the data-parallel collective / fork streams and the actor
# groups' streams exceed four, and a stream that shares a queue runs behind that queue's
# other work (actor inference queued behind the learner's step graphs starved the actors:
# profiles/r4_e2e_actor_streams_ab.txt).  Read when HIP initialises, so set before it.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def parse_args(argv=None):
    ap = argparse.ArgumentParser(prog="main.py")
    ap.add_argument("--params-file", default="parameters.json", type=str, metavar="PARAMSFILE",
                    help="Path to json file defining the parameters for the Actor, Learner and Replay memory")
    ap.add_argument("--set", action="append", default=[], metavar="Section.key=value",
                    help="override a config value (repeatable)")
    ap.add_argument("--mode", default="auto", choices=["auto", "gpu", "multiproc", "inline"])
    ap.add_argument("--learner-steps", type=int, default=None, help="overrides Runtime.learner_T")
    ap.add_argument("--metrics", default=None, help="JSONL metrics path (rank 0)")
    return ap.parse_args(argv)


def main(argv=None):
    args = parse_args(argv)
    import torch

    from apex_dqn_amd.config import ApexConfig
    from apex_dqn_amd.utils.metrics import MetricsLogger

    cfg = ApexConfig.load(args.params_file, args.set)
    steps = args.learner_steps or cfg.Runtime.learner_T
    rank = int(os.environ.get("RANK", "0"))
    if rank == 0:
        d = cfg.to_dict()
        print("Using the params:\n env_conf:{} \n actor_params:{} \n learner_params:{} \n, replay_params:{}"
              "\n runtime:{}".format(d["env_conf"], d["Actor"], d["Learner"], d["Replay_Memory"], d["Runtime"]))
    metrics = MetricsLogger(args.metrics or cfg.Runtime.metrics_path, rank=rank, echo=True)
    mode = args.mode
    image = len(cfg.env_conf.state_shape) == 3 and cfg.network in ("nature64", "nature32", "impala")
    if mode == "auto":
        mode = "gpu" if (torch.cuda.is_available() and image) else "multiproc"
    if mode == "gpu":
        from apex_dqn_amd.parallel.dist import Comm
        from apex_dqn_amd.runtime.gpu_loop import train_frames
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if torch.cuda.is_available():
            torch.cuda.set_device(local)
            device = torch.device("cuda", local)
        else:
            device = torch.device("cpu")
        comm = Comm.from_env(device=device)
        out = train_frames(cfg, device, steps, comm=comm, metrics=metrics)
        comm.shutdown()
    elif mode == "multiproc":
        from apex_dqn_amd.runtime.loops import train_multiprocess
        dev = "cuda" if torch.cuda.is_available() else "cpu"
        out = train_multiprocess(cfg, steps, device=dev, metrics=metrics)
    else:
        from apex_dqn_amd.runtime.loops import train_inline
        out = train_inline(cfg, steps, device="cuda" if torch.cuda.is_available() else "cpu", metrics=metrics)
    if rank == 0:
        print(json.dumps({"learner_steps": out["learner"].num_q_updates, "episodes": len(out["episodes"]),
                          "mean_return_last": out["mean_return_last"]}))
    metrics.close()


if __name__ == "__main__":
    main()
