#!/usr/bin/env python
"""fc GEMMs of the learner step: hand-written igemm kernels vs hipBLASLt (torch)
at the headline shapes -- decides whether the dense layers deserve another tile."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return 1e3 * e0.elapsed_time(e1) / iters


def main():
    from apex_dqn_amd.ops import _lib, conv as C
    lib = _lib.require_kernels()
    dev = torch.device("cuda", 0)
    bf = torch.bfloat16
    B = 512
    x = torch.relu(torch.randn(3 * B, 3136, device=dev)).to(bf)
    w = (torch.randn(1024, 3136, device=dev) * 0.02).to(bf)
    b = torch.randn(1024, device=dev) * 0.1
    h = torch.empty(3 * B, 1024, device=dev, dtype=bf)
    dh = (torch.randn(B, 1024, device=dev) * 0.01).to(bf)
    dx = torch.empty(B, 3136, device=dev, dtype=bf)
    gw = torch.empty(1024, 3136, device=dev)
    gb = torch.empty(1024, device=dev)
    bb = b.to(bf)
    res = {
        "fc_fwd_ours": timeit(lambda: C.dense_fwd(lib, x, w, b, h, True)),
        "fc_fwd_blas": timeit(lambda: torch.relu_(torch.addmm(bb, x, w.t(), out=h))),
        "fc_dgrad_ours": timeit(lambda: C.dense_dgrad(lib, dh, w, dx, x[:B])),
        "fc_dgrad_blas": timeit(lambda: torch.mm(dh, w, out=dx).mul_(x[:B] > 0)),
        "fc_wgrad_ours": timeit(lambda: C.dense_wgrad(lib, dh, x[:B], gw, gb)),
        "fc_wgrad_blas": timeit(lambda: (torch.mm(dh.t(), x[:B], out_dtype=torch.float32)
                                         if hasattr(torch, "_scaled_mm") else torch.mm(dh.t().float(), x[:B].float()))),
    }
    for k, v in res.items():
        print(json.dumps({"op": k, "us": round(v, 2)}))


if __name__ == "__main__":
    main()
