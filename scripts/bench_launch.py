"""Cost of a kernel boundary inside a HIP graph on this GPU: a graph of N launches of a
trivial kernel (apex_fill16 over n 16-B elements, 2048 x 256 threads) is replayed and
timed; us per launch for several n, and the same for a 256-block grid via torch's
fill_ on a small tensor.  The learner step is ~15 back-to-back launches, so this
bounds what fusing launches can save."""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from apex_dqn_amd.ops import _lib  # noqa: E402


def per_launch(fn, n_launch=200, iters=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n_launch):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (iters * n_launch)


def main():
    lib = _lib.require_kernels()
    dev = torch.device("cuda", 0)
    buf = torch.zeros(64 << 20, dtype=torch.uint8, device=dev)
    res = {}
    for n16 in (1, 4096, 65536, 1 << 20):
        us = per_launch(lambda: _lib.check(lib.apex_fill16(buf.data_ptr(), n16, 0, _lib.stream_ptr()), "fill16"))
        res[f"fill16_{n16 * 16}B"] = round(us, 3)
        print(json.dumps({"kernel": "fill16", "bytes": n16 * 16, "us_per_launch": round(us, 3)}), flush=True)
    t = torch.zeros(256 * 64, device=dev)
    us = per_launch(lambda: t.fill_(1.0))
    res["torch_fill_64KB"] = round(us, 3)
    print(json.dumps({"kernel": "torch_fill", "bytes": t.numel() * 4, "us_per_launch": round(us, 3)}), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/launch_cost.json", "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
