"""Generic implicit-GEMM forward/dgrad kernels at the learner shapes: the register-
staged kernel (tile hint 2 = 64-row, 1 = 128-row tiles) against the LDS-DMA staged
kernel (hint 3, the launcher default), bf16 and split (fp32-accurate) operands.
Every kernel runs the same MFMA sequence per accumulator, so the outputs must agree
bit for bit; the script reports the max |difference| next to the times."""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from bench_tree import timed  # noqa: E402
from apex_dqn_amd.ops import _lib, conv as C  # noqa: E402
from apex_dqn_amd.ops.switches import SW  # noqa: E402


def sp(t):
    hi = t.to(torch.bfloat16)
    return hi, (t - hi.float()).to(torch.bfloat16)


def main():
    dev = torch.device("cuda", 0)
    lib = _lib.require_kernels()
    torch.manual_seed(0)
    N, B = 1536, 512
    x = torch.relu(torch.randn(N, 3136, device=dev))
    w, w2 = torch.randn(1024, 3136, device=dev) * 0.02, torch.randn(1024, 3136, device=dev) * 0.02
    b, b2 = torch.randn(1024, device=dev), torch.randn(1024, device=dev)
    (xh, xl), (wh, wl), (w2h, w2l) = sp(x), sp(w), sp(w2)
    x3 = torch.relu(torch.randn(N, 9, 9, 64, device=dev))
    w3, w32 = torch.randn(64, 3, 3, 64, device=dev) * 0.04, torch.randn(64, 3, 3, 64, device=dev) * 0.04
    (x3h, x3l), (w3h, w3l), (w32h, w32l) = sp(x3), sp(w3), sp(w32)
    dH = torch.randn(B, 1024, device=dev) * 0.01
    (dHh, dHl) = sp(dH)
    y3 = torch.relu(torch.randn(B, 3136, device=dev)).to(torch.bfloat16)
    dy3 = torch.randn(B, 7, 7, 64, device=dev)
    (d3h, d3l) = sp(dy3)
    y2 = torch.relu(torch.randn(B, 9, 9, 64, device=dev)).to(torch.bfloat16)
    dy2 = torch.randn(B, 9, 9, 64, device=dev)
    (d2h, d2l) = sp(dy2)
    wc2 = torch.randn(64, 4, 4, 64, device=dev) * 0.03
    (wc2h, wc2l) = sp(wc2)
    y1 = torch.relu(torch.randn(B, 20, 20, 64, device=dev)).to(torch.bfloat16)

    def outs(*shape):
        return [torch.zeros(*shape, device=dev, dtype=torch.bfloat16) for _ in range(2)]

    SW.conv3_dgrad_img = False
    SW.conv2_dgrad_img = False
    cases = {
        "fc_fwd": (outs(N, 1024), lambda o, s: C.dense_fwd(
            lib, xh, wh, b, o[0], True, None, w2h, b2, 1024,
            **(dict(x_lo=xl, w_lo=wl, w2_lo=w2l, out_lo=o[1]) if s else {}))),
        "fc_dgrad": (outs(B, 3136), lambda o, s: C.dense_dgrad(
            lib, dHh, wh, o[0], y3, **(dict(dh_lo=dHl, w_lo=wl, out_lo=o[1]) if s else {}))),
        "conv3_fwd": (outs(N, 7, 7, 64), lambda o, s: C.conv_fwd(
            lib, x3h, w3h, b, 1, o[0], w32h, b2, 1024,
            **(dict(x_lo=x3l, w_lo=w3l, w2_lo=w32l, out_lo=o[1]) if s else {}))),
        "conv3_dgrad": (outs(B, 9, 9, 64), lambda o, s: C.conv3_dgrad(
            lib, d3h, w3h, y2, o[0], **(dict(dy_lo=d3l, w_lo=w3l, out_lo=o[1]) if s else {}))),
        "conv2_dgrad": (outs(B, 20, 20, 64), lambda o, s: C.conv2_dgrad(
            lib, d2h, wc2h, y1, o[0], **(dict(dy_lo=d2l, w_lo=wc2l, out_lo=o[1]) if s else {}))),
    }
    res = {}
    for split in (False, True):
        for name, (o, fn) in cases.items():
            r = {"op": name, "split": split}
            ref = None
            for hint in (2, 1, 4, 5):
                C._HINTS["tile"], C._HINTS["order"] = hint, 0
                for t in o:
                    t.zero_()
                fn(o, split)
                torch.cuda.synchronize()
                got = [t.clone() for t in o]
                if ref is None:
                    ref = got
                else:
                    r[f"maxdiff_h{hint}"] = max(float((a.float() - c.float()).abs().max()) for a, c in zip(got, ref))
                r[f"us_h{hint}"] = round(timed(lambda: fn(o, split)), 2)
            if name in ("conv3_dgrad", "conv2_dgrad") and not (name == "conv3_dgrad" and split):
                SW.conv3_dgrad_img = SW.conv2_dgrad_img = True      # image-resident kernels
                C._HINTS["tile"] = 0
                r["us_img"] = round(timed(lambda: fn(o, split)), 2)
                SW.conv3_dgrad_img = SW.conv2_dgrad_img = False
            print(json.dumps(r), flush=True)
            res[f"{name}_{'split' if split else 'bf16'}"] = r
    C._HINTS["tile"] = C._HINTS["order"] = 0
    SW.conv3_dgrad_img = True
    SW.conv2_dgrad_img = True
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/dma_gemm.json", "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
