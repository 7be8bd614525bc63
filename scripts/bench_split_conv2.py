"""Split-mode (fp32-accurate) conv2 kernels at the learner shapes: image-resident
forward / data gradient (csrc/conv2_img.hip) vs the generic implicit GEMM, and the
per-image cost slope (N sweep at a fixed grid) that separates fixed overheads
(weight fragments, first plane) from the per-image work."""
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
    N = 1536
    x = torch.relu(torch.randn(N, 20, 20, 64, device=dev))
    w = torch.randn(64, 4, 4, 64, device=dev) * 0.03
    w2 = torch.randn(64, 4, 4, 64, device=dev) * 0.03
    b, b2 = torch.randn(64, device=dev), torch.randn(64, device=dev)
    (xh, xl), (wh, wl), (w2h, w2l) = sp(x), sp(w), sp(w2)
    oh = torch.empty(N, 9, 9, 64, device=dev, dtype=torch.bfloat16)
    ol = torch.empty_like(oh)
    fl = 3 * 2.0 * N * 81 * 64 * 1024
    only = os.environ.get("ONLY", "")
    if not only:
        SW.conv2_img = False
        us = timed(lambda: C.conv_fwd(lib, xh, wh, b, 2, oh, w2h, b2, 1024, x_lo=xl, w_lo=wl, w2_lo=w2l, out_lo=ol))
        print(json.dumps({"op": "conv2_fwd_split_igemm", "us": round(us, 2), "tflops_eff": round(fl / us / 1e6, 1)}),
              flush=True)
    for pack in (False, True):
        SW.c2f_pack = pack
        for n in ((256, 512, 1024, 1536) if not only else (1536,)):
            if only and only != "fwd":
                break
            us = timed(lambda: C.conv2_img_fwd(lib, xh[:n], wh, b, oh[:n], w2h, b2, 2 * n // 3, x_lo=xl[:n],
                                               w_lo=wl, w2_lo=w2l, out_lo=ol[:n]))
            print(json.dumps({"op": "conv2_fwd_split_img", "packed_w": pack, "images": n, "us": round(us, 2),
                              "tflops_eff": round(3 * 2.0 * n * 81 * 64 * 1024 / us / 1e6, 1)}), flush=True)
    B = 512
    dy = torch.randn(B, 9, 9, 64, device=dev)
    dyh, dyl = sp(dy)
    y1 = torch.relu(torch.randn(B, 20, 20, 64, device=dev)).to(torch.bfloat16)
    dxh = torch.empty(B, 20, 20, 64, device=dev, dtype=torch.bfloat16)
    dxl = torch.empty_like(dxh)
    if not only:
        SW.conv2_dgrad_img = False
        us = timed(lambda: C.conv2_dgrad(lib, dyh, wh, y1, dxh, dy_lo=dyl, w_lo=wl, out_lo=dxl))
        print(json.dumps({"op": "conv2_dgrad_split_igemm", "us": round(us, 2)}), flush=True)
    for n in ((256, 512) if not only else (512,)):
        if only and only != "dgrad":
            break
        us = timed(lambda: C.conv2_dgrad_img(lib, dyh[:n], wh, y1[:n], dxh[:n], dy_lo=dyl[:n], w_lo=wl,
                                             out_lo=dxl[:n]))
        print(json.dumps({"op": "conv2_dgrad_split_img", "images": n, "us": round(us, 2)}), flush=True)


if __name__ == "__main__":
    main()
