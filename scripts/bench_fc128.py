"""fc forward at the learner shape (1536 x 3136 -> 1024, online rows 0..1023, target
rows 1024..1535): the 64x64-tile LDS-DMA kernel of the step (``dense_fwd``) against
the 128x128-tile split-K kernel (``dense_fwd128``, ksplit 1..4), bf16 and split
(fp32-accurate) operands.  Reports us per call (graph-replayed) and the max relative
error against an fp64 reference of the same op."""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from bench_tree import timed  # noqa: E402
from apex_dqn_amd.ops import _lib, conv as C  # noqa: E402


def sp(t):
    hi = t.to(torch.bfloat16)
    return hi, (t - hi.float()).to(torch.bfloat16)


def main():
    dev = torch.device("cuda", 0)
    lib = _lib.require_kernels()
    torch.manual_seed(0)
    N, S = 1536, 1024
    x = torch.relu(torch.randn(N, 3136, device=dev))
    w, w2 = torch.randn(1024, 3136, device=dev) * 0.02, torch.randn(1024, 3136, device=dev) * 0.02
    b, b2 = torch.randn(1024, device=dev) * 0.1, torch.randn(1024, device=dev) * 0.1
    (xh, xl), (wh, wl), (w2h, w2l) = sp(x), sp(w), sp(w2)
    ws = C.Workspace()
    res = {}
    for split in (False, True):
        xs = (xh.double() + xl.double()) if split else xh.double()
        ws_ = (wh.double() + wl.double()) if split else wh.double()
        w2s = (w2h.double() + w2l.double()) if split else w2h.double()
        ref = torch.cat([xs[:S] @ ws_.T + b.double(), xs[S:] @ w2s.T + b2.double()]).clamp_min(0)
        o = [torch.zeros(N, 1024, device=dev, dtype=torch.bfloat16) for _ in range(2)]
        lo = dict(x_lo=xl, w_lo=wl, w2_lo=w2l, out_lo=o[1]) if split else {}
        cases = {"t64": lambda: C.dense_fwd(lib, xh, wh, b, o[0], True, None, w2h, b2, S, **lo)}
        for k in (1, 2, 3, 4):
            for lw in (False, True):
                cases[f"t128_k{k}{'_lw' if lw else ''}"] = (
                    lambda k=k, lw=lw: C.dense_fwd128(lib, ws, xh, wh, b, o[0], True, w2h, b2, S, k, lw, **lo))
        for name, fn in cases.items():
            for t in o:
                t.zero_()
            fn()
            torch.cuda.synchronize()
            got = o[0].double() + (o[1].double() if split else 0)
            err = float(((got - ref).abs() / (ref.abs() + 1e-2)).max())
            us = timed(fn)
            r = {"split": split, "kernel": name, "us": round(us, 2), "max_rel_err": err}
            print(json.dumps(r), flush=True)
            res[f"{'split' if split else 'bf16'}_{name}"] = r
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/fc128.json", "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
