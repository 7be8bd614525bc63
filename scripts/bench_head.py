"""Microbenchmark of the dueling-head kernels at B=512 (A=4): ddqn_head, the
head with the fused priority write-back, head_wgrad -- each timed inside a HIP
graph of repeated launches (scripts/bench_tree.py:timed)."""
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
    B, A = int(os.environ.get("B", "512")), 4
    g = torch.Generator(device="cpu").manual_seed(0)
    Hon = torch.relu(torch.randn(2 * B, 1024, generator=g)).to(dev, torch.bfloat16)
    Htg = torch.relu(torch.randn(B, 1024, generator=g)).to(dev, torch.bfloat16)
    Hsrc, Htsrc = Hon.clone(), Htg.clone()

    def P():
        return {"wv": (torch.randn(512, generator=g) * 0.05).to(dev), "bv": torch.randn(1, generator=g).to(dev),
                "wa": (torch.randn(A, 512, generator=g) * 0.05).to(dev), "ba": torch.randn(A, generator=g).to(dev)}
    Pon, Ptg = P(), P()
    Psrc, Ptsrc = {k: v.clone() for k, v in Pon.items()}, {k: v.clone() for k, v in Ptg.items()}
    act = torch.randint(0, A, (B,), generator=g).to(dev, torch.int32)
    rew, gam, isw = torch.randn(B, device=dev), torch.full((B,), 0.97, device=dev), torch.rand(B, device=dev)
    td, loss = torch.zeros(B, device=dev), torch.zeros(B, device=dev)
    dH, dhead = torch.zeros(B, 1024, device=dev, dtype=torch.bfloat16), torch.zeros(B, A + 1, device=dev)
    zero = torch.zeros(2 * 512 + A * 512 + A + 1, device=dev)
    gr = {"wv": torch.zeros(512, device=dev), "bv": torch.zeros(1, device=dev),
          "wa": torch.zeros(A, 512, device=dev), "ba": torch.zeros(A, device=dev)}
    rp = GpuReplayShard(100000, 100000, 100100, 4, device=dev)
    rng = np.random.default_rng(0)
    rp.frame_head = 100100
    K = 100000
    st = rng.integers(0, 100000, size=K)[:, None] + np.arange(4)[None]
    rp.insert(dict(S_t=st, S_tpn=st + 3, A_t=rng.integers(0, A, K), R=rng.normal(size=K).astype(np.float32),
                   Gamma=np.full(K, 0.97, np.float32), priority=rng.random(K).astype(np.float32) + 0.01))
    rp.rebuild()
    S = rp.alloc_sample_buffers(B)
    rp.sample(B, out=S)
    be = HipBackend()
    args = (Hon, Htg, Pon, Ptg, act, rew, gam, isw, True, 1.0, 1.0 / B, td, loss, dH, dhead)
    for name, fn in [("head", lambda: be.head(*args, zero=zero)),
                     ("head_wgrad", lambda: be.head_wgrad(Hon, dhead, gr)),
                     ("head_wgrad_prio", lambda: be.head_wgrad(Hon, dhead, gr, prio=(rp, S["idx"], S["gen"], td))),
                     ("tree_update", lambda: rp.update_priorities(S["idx"], td, S["gen"])),
                     # the head right after a kernel that rewrote its inputs (as in the step,
                     # where the fc forward produces them): minus "rewrite" = in-step cost
                     ("rewrite", lambda: (Hon.copy_(Hsrc), Htg.copy_(Htsrc))),
                     ("rewrite+head", lambda: (Hon.copy_(Hsrc), Htg.copy_(Htsrc), be.head(*args, zero=zero))),
                     # ... and its head weights too (the optimizer rewrites them every step)
                     ("rewrite_all", lambda: (Hon.copy_(Hsrc), Htg.copy_(Htsrc), [Pon[k].copy_(Psrc[k]) for k in Pon],
                                              [Ptg[k].copy_(Ptsrc[k]) for k in Ptg])),
                     ("rewrite_all+head", lambda: (Hon.copy_(Hsrc), Htg.copy_(Htsrc), [Pon[k].copy_(Psrc[k]) for k in Pon],
                                                   [Ptg[k].copy_(Ptsrc[k]) for k in Ptg], be.head(*args, zero=zero)))]:
        print(json.dumps({"op": name, "B": B, "us": round(timed(fn), 2)}), flush=True)


if __name__ == "__main__":
    main()
