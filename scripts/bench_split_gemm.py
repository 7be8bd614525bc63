"""Split-mode (fp32-accurate) generic implicit-GEMM kernels at the learner shapes
with the tile-shape hint swept (0 = launcher default, 1 = 128-row tiles, 2 = 64-row)."""
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
    x = torch.relu(torch.randn(N, 3136, device=dev))
    w, w2 = torch.randn(1024, 3136, device=dev) * 0.02, torch.randn(1024, 3136, device=dev) * 0.02
    b, b2 = torch.randn(1024, device=dev), torch.randn(1024, device=dev)
    (xh, xl), (wh, wl), (w2h, w2l) = sp(x), sp(w), sp(w2)
    oh = torch.empty(N, 1024, device=dev, dtype=torch.bfloat16)
    ol = torch.empty_like(oh)
    x3 = torch.relu(torch.randn(N, 9, 9, 64, device=dev))
    w3, w32 = torch.randn(64, 3, 3, 64, device=dev) * 0.04, torch.randn(64, 3, 3, 64, device=dev) * 0.04
    (x3h, x3l), (w3h, w3l), (w32h, w32l) = sp(x3), sp(w3), sp(w32)
    o3h = torch.empty(N, 7, 7, 64, device=dev, dtype=torch.bfloat16)
    o3l = torch.empty_like(o3h)
    B = 512
    dH = torch.randn(B, 1024, device=dev) * 0.01
    (dHh, dHl) = sp(dH)
    y3 = torch.relu(torch.randn(B, 3136, device=dev)).to(torch.bfloat16)
    dxh = torch.empty(B, 3136, device=dev, dtype=torch.bfloat16)
    dxl = torch.empty_like(dxh)
    dy3 = torch.randn(B, 7, 7, 64, device=dev)
    (d3h, d3l) = sp(dy3)
    y2 = torch.relu(torch.randn(B, 9, 9, 64, device=dev)).to(torch.bfloat16)
    e2h = torch.empty(B, 9, 9, 64, device=dev, dtype=torch.bfloat16)
    e2l = torch.empty_like(e2h)
    SW.conv3_dgrad_img = False
    for hint, order in ((0, 0), (1, 0), (2, 0), (2, 1), (2, 2), (1, 1), (1, 2)):
        C._HINTS["tile"], C._HINTS["order"] = hint, order
        r = {"hint": hint, "order": order}
        r["fc_fwd"] = timed(lambda: C.dense_fwd(lib, xh, wh, b, oh, True, None, w2h, b2, 1024, x_lo=xl, w_lo=wl,
                                                 w2_lo=w2l, out_lo=ol))
        r["conv3_fwd"] = timed(lambda: C.conv_fwd(lib, x3h, w3h, b, 1, o3h, w32h, b2, 1024, x_lo=x3l, w_lo=w3l,
                                                  w2_lo=w32l, out_lo=o3l))
        r["conv3_dgrad"] = timed(lambda: C.conv3_dgrad(lib, d3h, w3h, y2, e2h, dy_lo=d3l, w_lo=w3l, out_lo=e2l))
        print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
    C._HINTS["tile"] = C._HINTS["order"] = 0


if __name__ == "__main__":
    main()
