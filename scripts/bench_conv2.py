"""conv2 forward at the learner shape (3B = 1536 images, 20x20x64 -> 9x9x64):
image-resident kernel (csrc/conv2_img.hip, several grid sizes) vs the generic
implicit GEMM (csrc/conv_mfma.hip igemm_fwd)."""
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


def main():
    dev = torch.device("cuda", 0)
    N = int(os.environ.get("N", "1536"))
    lib = _lib.require_kernels()
    x = torch.relu(torch.randn(N, 20, 20, 64, device=dev)).to(torch.bfloat16)
    w = (torch.randn(64, 4, 4, 64, device=dev) * 0.03).to(torch.bfloat16)
    w2 = (torch.randn(64, 4, 4, 64, device=dev) * 0.03).to(torch.bfloat16)
    b, b2 = torch.randn(64, device=dev), torch.randn(64, device=dev)
    out = torch.empty(N, 9, 9, 64, device=dev, dtype=torch.bfloat16)
    fl = 2.0 * N * 81 * 64 * 1024
    SW.conv2_img = False
    us = timed(lambda: C.conv_fwd(lib, x, w, b, 2, out, w2, b2, 2 * N // 3))
    print(json.dumps({"op": "conv2_fwd_igemm", "us": round(us, 2), "tflops": round(fl / us / 1e6, 1)}), flush=True)
    B = N // 2       # 768: the per-image sweep below uses 256 / 512 / 768 of them
    dy = torch.randn(B, 9, 9, 64, device=dev).to(torch.bfloat16)
    y1 = torch.relu(torch.randn(B, 20, 20, 64, device=dev)).to(torch.bfloat16)
    dx = torch.empty(B, 20, 20, 64, device=dev, dtype=torch.bfloat16)
    fl2 = 2.0 * B * 400 * 64 * 256
    SW.conv2_dgrad_img = False
    us = timed(lambda: C.conv2_dgrad(lib, dy, w, y1, dx))
    print(json.dumps({"op": "conv2_dgrad_igemm", "us": round(us, 2), "tflops": round(fl2 / us / 1e6, 1)}), flush=True)
    for nimg in (256, 512, 768):
        us = timed(lambda: C.conv2_dgrad_img(lib, dy[:nimg], w, y1[:nimg], dx[:nimg], grid=256))
        print(json.dumps({"op": "conv2_dgrad_img_n", "images": nimg, "us": round(us, 2)}), flush=True)
    for grid in (256, 512):
        us = timed(lambda: C.conv2_dgrad_img(lib, dy, w, y1, dx, grid=grid))
        print(json.dumps({"op": "conv2_dgrad_img", "grid": grid, "us": round(us, 2),
                          "tflops": round(fl2 / us / 1e6, 1)}), flush=True)
    dy3 = torch.randn(B, 7, 7, 64, device=dev).to(torch.bfloat16)
    w3 = (torch.randn(64, 3, 3, 64, device=dev) * 0.04).to(torch.bfloat16)
    y2 = torch.relu(torch.randn(B, 9, 9, 64, device=dev)).to(torch.bfloat16)
    dx2 = torch.empty(B, 9, 9, 64, device=dev, dtype=torch.bfloat16)
    SW.conv3_dgrad_img = False
    us = timed(lambda: C.conv3_dgrad(lib, dy3[:512], w3, y2[:512], dx2[:512]))
    print(json.dumps({"op": "conv3_dgrad_igemm", "images": 512, "us": round(us, 2)}), flush=True)
    for g3 in (256, 128, 512):
        us = timed(lambda: C.conv3_dgrad_img(lib, dy3[:512], w3, y2[:512], dx2[:512], grid=g3))
        print(json.dumps({"op": "conv3_dgrad_img", "images": 512, "grid": g3, "us": round(us, 2)}), flush=True)
    for grid in (256, 128, 512, 768):
        us = timed(lambda: C.conv2_img_fwd(lib, x, w, b, out, w2, b2, 2 * N // 3, grid=grid))
        print(json.dumps({"op": "conv2_fwd_img", "grid": grid, "us": round(us, 2),
                          "tflops": round(fl / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
