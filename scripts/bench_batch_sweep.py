#!/usr/bin/env python
"""Per-rank learner step time vs rows per rank (one GPU): the cost model of the
global-batch (strong-scaling) DP mode.  With ``Runtime.batch_scope = "global"`` a
W-rank update of 512 samples computes ceil(512/W (1 + slack)) + 2 rows per rank
(``ApexConfig.dp_batch``: 290 / 146 / 74 at W = 2 / 4 / 8); this times the
single-rank step (bench.py's timing discipline) at those sizes and at the plain
powers of two, in both precisions, and writes one JSON document.

    python scripts/bench_batch_sweep.py --out gpurun_out/batch_sweep.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="64,74,128,146,256,290,512")
    ap.add_argument("--dtypes", default="fp32,bf16")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--out", default="gpurun_out/batch_sweep.json")
    a = ap.parse_args()
    from apex_dqn_amd.parallel.dist import Comm
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comm = Comm.from_env(backend="nccl", device=dev, force=False)
    base = ["--steps", str(a.steps), "--warmup", str(a.warmup)]
    args = bench_args(base)
    replay = bench.make_replay(args, dev, 0)
    rows = []
    for dt in a.dtypes.split(","):
        for B in [int(x) for x in a.batches.split(",")]:
            args = bench_args(base + ["--batch", str(B), "--dtype", dt])
            cfg, L = bench.make_learner(args, dt, dev, comm, 0, replay)
            r = bench.measure(cfg, L, replay, comm, args.warmup, args.steps, args.prep_warm)
            us = 1e6 * r["dt"] / args.steps
            rows.append({"dtype": dt, "rows": B, "us_per_step": round(us, 2), "steps_per_s": round(1e6 / us, 1),
                         "samples_per_s": round(B * 1e6 / us, 0),
                         "graph_captures_in_timed": r["graph_captures_in_timed"]})
            print(json.dumps(rows[-1]), flush=True)
            del L
            torch.cuda.empty_cache()
    doc = {"what": "single-rank fused learner step vs rows per rank (bench.py timing: warm graphs, "
                   "barrier + synchronize brackets)", "steps": a.steps, "warmup": a.warmup,
           "device": torch.cuda.get_device_name(dev), "time": time.strftime("%Y-%m-%d %H:%M:%S"), "rows": rows}
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(doc, f, indent=1)


def bench_args(argv):
    """bench.py's argument namespace for ``argv`` (its defaults otherwise)."""
    return bench.parser().parse_args(list(argv))


if __name__ == "__main__":
    main()
