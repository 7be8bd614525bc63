"""Microbenchmark of the learner's optimizer launch at the NatureCNN size (3.33 M
parameters, fp32-class: hi / lo bf16 copies): clip + centered RMSprop alone, fused with
the next batch's draw (rmsprop_sample_kernel), and the draw alone (tree_sample) -- each
timed inside a HIP graph of repeated launches (scripts/bench_tree.py:timed).  Tells
whether the draw's blocks or the update's HBM traffic bound the fused launch."""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from bench_tree import timed  # noqa: E402
from apex_dqn_amd.ops.fused_ops import HipBackend  # noqa: E402
from apex_dqn_amd.replay.gpu_replay import GpuReplayShard  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    n = 3_336_392     # (the NatureCNN count rounded to 8: the lo plane stays 16-B aligned)
    B = int(os.environ.get("B", "512"))
    cap = 100000
    rp = GpuReplayShard(cap, cap, cap + 4096, 4, device=dev, seed=1)
    rng = np.random.default_rng(0)
    rp.frame_head = cap + 4096
    for s in range(0, cap, 16384):
        K = min(16384, cap - s)
        st = rng.integers(0, cap, size=K)[:, None] + np.arange(4)[None]
        rp.insert(dict(S_t=st, S_tpn=st + 3, A_t=rng.integers(0, 4, K), R=rng.normal(size=K).astype(np.float32),
                       Gamma=np.full(K, 0.97, np.float32), priority=rng.random(K).astype(np.float32) + 0.01))
    rp.rebuild()
    be = HipBackend()
    g = torch.Generator(device="cpu").manual_seed(0)
    p = torch.randn(n, generator=g).to(dev)
    gr = torch.randn(n, generator=g).to(dev) * 1e-3
    v, m = torch.zeros(n, device=dev), torch.zeros(n, device=dev)
    pbf = torch.zeros(2 * n, device=dev, dtype=torch.bfloat16)
    part, gn = torch.zeros(4096, dtype=torch.float64, device=dev), torch.zeros(1, device=dev)
    part[:2600] = 1e-6
    S = rp.alloc_sample_buffers(B)
    nxt2 = torch.zeros(B, 4, dtype=torch.int32, device=dev)
    args = (p, gr, v, m, pbf[:n], 2.5e-4, 0.95, 1.5e-7, 40.0, True, part, gn)
    kw = dict(norm_total=(part, 2600), pb_lo=pbf[n:])
    res = {
        "rmsprop_only_us": timed(lambda: be.optimizer(*args, **kw)),
        "rmsprop_sample_us": timed(lambda: be.optimizer(*args, sample=(rp, B, S, nxt2), **kw)),
        "tree_sample_only_us": timed(lambda: rp.sample(B, out=S, nxt2=nxt2)),
    }
    res.update(B=B, n=n, bytes_per_update=n * (4 * 4 + 3 * 4 + 2 * 2))
    res["rmsprop_only_TBps"] = round(res["bytes_per_update"] / res["rmsprop_only_us"] / 1e6, 2)
    print(json.dumps({k: (round(x, 2) if isinstance(x, float) else x) for k, x in res.items()}), flush=True)


if __name__ == "__main__":
    main()
