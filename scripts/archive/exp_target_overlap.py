#!/usr/bin/env python
"""Experiment: can the target network's forward (B rows: conv12 -> conv3 -> fc) run
beside the learner's latency-bound backward?  Times, as captured HIP graphs replayed
back to back on one MI355X:

  bwd       the step's backward (fc dgrad .. grad_finalize, ``_seg2``)
  tgt       the target forward of B rows alone
  serial    both on one stream
  parallel  target forward on a second stream forked before the backward, joined after
  parallel_wq   the same with the persistent kernels' device-side work queues on

and prints one JSON line per variant (us per replay, mean of ``--reps`` replays)."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from apex_dqn_amd.config import ApexConfig  # noqa: E402
from apex_dqn_amd.learner.fused_learner import FusedNatureLearner  # noqa: E402
from apex_dqn_amd.ops import conv as C  # noqa: E402
from apex_dqn_amd.ops.switches import SW  # noqa: E402
from apex_dqn_amd.replay.gpu_replay import GpuReplayShard  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    B = a.batch
    cfg = ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 4, "name": "Synthetic"},
                                "Learner": {"replay_sample_size": B},
                                "Runtime": {"use_graphs": False, "presample": False, "dtype": a.dtype}})
    rp = GpuReplayShard(20000, 20000, 24000, 4, device=dev, seed=1)
    rng = np.random.default_rng(0)
    seqs = rp.append_frames(rng.integers(0, 255, (24000, 84, 84), dtype=np.uint8))
    K = 20000
    st = np.stack([seqs[i:i + 4] for i in range(K)])
    rp.insert(dict(S_t=st, S_tpn=st + 3, A_t=rng.integers(0, 4, K), R=rng.normal(size=K).astype(np.float32),
                   Gamma=np.full(K, 0.97, np.float32), priority=rng.random(K).astype(np.float32) + 0.01))
    L = FusedNatureLearner(cfg, dev, rp, backend="hip")
    for _ in range(3):
        L._step_body()
    torch.cuda.synchronize()
    ops, sp = L.ops, L.split
    T, Tb, Tl = L.T, L.Tb, L.Tl
    y2 = torch.zeros(B, 9, 9, 64, dtype=torch.bfloat16, device=dev)
    y2l = torch.zeros_like(y2) if sp else None
    y3 = torch.zeros(B, 7, 7, 64, dtype=torch.bfloat16, device=dev)
    y3l = torch.zeros_like(y3) if sp else None
    h = torch.zeros(B, 1024, dtype=torch.bfloat16, device=dev)
    hl = torch.zeros_like(h) if sp else None
    slots = L.slots[2 * B:].clone()
    c1, c2 = L._conv12_weights()

    def tgt():
        # all rows on the second (target) weight set: img_switch = 0
        w1, b1, w1b, b1b = c1
        w2, w2l, b2, w2b, w2bl, b2b = c2
        C.conv12_fused_fwd(ops.lib, ops.ws, rp.frames, slots, w1, b1, w2, w2l, b2, L.rt.obs_scale, y2, y2l,
                           copy_n=0, w1b=w1b, b1b=b1b, w2b=w2b, w2b_lo=w2bl, b2b=b2b, rows_first=0, pack_sets=0)
        C.conv_fwd(ops.lib, y2, Tb["w3"], T["b3"], 1, y3, **({"x_lo": y2l, "w_lo": Tl["w3"], "out_lo": y3l}
                                                             if sp else {}))
        C.dense_fwd128(ops.lib, ops.ws, y3.reshape(B, 3136), Tb["wfc"], T["bfc"], h, True, ksplit=2,
                       **({"x_lo": y3l.reshape(B, 3136), "w_lo": Tl["wfc"], "out_lo": hl} if sp else {}))

    def bwd():
        L._seg2()

    side = torch.cuda.Stream(dev)

    def par():
        ev = torch.cuda.Event()
        ev.record()
        side.wait_event(ev)
        with torch.cuda.stream(side):
            tgt()
        bwd()
        torch.cuda.current_stream(dev).wait_stream(side)

    def serial():
        tgt()
        bwd()

    def time_graph(fn):
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            fn()
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        for _ in range(10):
            g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            g.replay()
        torch.cuda.synchronize()
        return 1e6 * (time.perf_counter() - t0) / a.reps

    res = {}
    for name, fn in (("bwd", bwd), ("tgt", tgt), ("serial", serial), ("parallel", par)):
        res[name] = time_graph(fn)
        print(json.dumps({"variant": name, "B": B, "dtype": a.dtype, "us": round(res[name], 2)}), flush=True)
    SW.work_queue = "on"
    ops.ws.work_queue = True
    res["parallel_wq"] = time_graph(par)
    print(json.dumps({"variant": "parallel_wq", "B": B, "dtype": a.dtype, "us": round(res["parallel_wq"], 2)}),
          flush=True)
    res["serial_wq"] = time_graph(serial)
    print(json.dumps({"variant": "serial_wq", "B": B, "dtype": a.dtype, "us": round(res["serial_wq"], 2)}),
          flush=True)


if __name__ == "__main__":
    main()
