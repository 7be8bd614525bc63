"""Microbenchmark of the replay sum-tree kernels (tree_update variants, tree_sample)
on a 100k-leaf shard at B=512, timed inside a HIP graph of repeated launches.
Writes one JSON line per variant."""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from apex_dqn_amd.ops import _lib  # noqa: E402
from apex_dqn_amd.replay.gpu_replay import GpuReplayShard  # noqa: E402


def timed(fn, reps=20, iters=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return 1e3 * e0.elapsed_time(e1) / (iters * reps)


def main():
    dev = torch.device("cuda", 0)
    cap, B = 100000, 512
    rp = GpuReplayShard(cap, cap, cap + 4096, 4, device=dev, seed=1)
    rng = np.random.default_rng(0)
    rp.frame_head = cap + 4096
    for s in range(0, cap, 16384):
        K = min(16384, cap - s)
        base = rng.integers(0, cap, size=K)
        st = base[:, None] + np.arange(4)[None]
        rp.insert(dict(S_t=st, S_tpn=st + 3, A_t=rng.integers(0, 4, K), R=rng.normal(size=K).astype(np.float32),
                       Gamma=np.full(K, 0.97, np.float32), priority=rng.random(K).astype(np.float32) + 0.01))
    rp.rebuild()
    S = rp.alloc_sample_buffers(B)
    rp.sample(B, out=S)
    tds = [torch.rand(B, device=dev), torch.rand(B, device=dev)]
    flip = [0]
    lib = rp.lib
    out = []

    def upd(n, mode, dedupe, gen=True):
        def f():
            flip[0] ^= 1
            td = tds[flip[0]]
            _lib.check(lib.apex_tree_update(rp.tree_desc(), S["idx"].data_ptr(), td.data_ptr(), n, mode,
                                            rp.alpha, rp.eps, S["gen"].data_ptr() if gen else None,
                                            rp.gen.data_ptr(), dedupe, rp.ctr.data_ptr(),
                                            rp._stream()), "tree_update")
        return f
    for name, fn in [("update_full", upd(B, 1, 1)), ("update_nodedupe", upd(B, 1, 0)),
                     ("update_mode0", upd(B, 0, 1, False)), ("update_mode0_nodedupe", upd(B, 0, 0, False)),
                     ("update_n64", upd(64, 1, 1)), ("update_n1", upd(1, 1, 1)),
                     ("sample", lambda: rp.sample(B, out=S))]:
        out.append({"op": name, "us": round(timed(fn), 2)})
        print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
