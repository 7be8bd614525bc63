#!/usr/bin/env python
"""Per-kernel microbenchmark of the learner's GEMM-shaped ops at the headline
shapes (B=512, 3B=1536 forward rows).  Prints one JSON line per op with time
and achieved TFLOP/s.  Use under rocprofv3 for counters:
    rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 ... -- python scripts/bench_kernels.py --iters 5
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--B", type=int, default=512)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    from apex_dqn_amd.ops import _lib, conv as C
    lib = _lib.require_kernels()
    dev = torch.device("cuda", 0)
    B = a.B
    N3 = 3 * B
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)

    def rn(*s, scale=1.0):
        return (torch.randn(*s, device=dev, generator=g) * scale).to(bf)

    ring = torch.randint(0, 256, (20000, 84, 84), device=dev, dtype=torch.uint8, generator=g)
    slots = torch.randint(0, 20000, (N3, 4), device=dev, dtype=torch.int32, generator=g)
    w1, w1t = rn(64, 4, 8, 8, scale=0.05), rn(64, 4, 8, 8, scale=0.05)
    w2, w2t = rn(64, 4, 4, 64, scale=0.03), rn(64, 4, 4, 64, scale=0.03)
    w3, w3t = rn(64, 3, 3, 64, scale=0.04), rn(64, 3, 3, 64, scale=0.04)
    wfc, wfct = rn(1024, 3136, scale=0.02), rn(1024, 3136, scale=0.02)
    bias = torch.randn(1024, device=dev) * 0.1
    y1 = torch.relu(rn(N3, 20, 20, 64))
    y2 = torch.relu(rn(N3, 9, 9, 64))
    y3 = torch.relu(rn(N3, 7, 7, 64))
    h = torch.empty(N3, 1024, device=dev, dtype=bf)
    dH = rn(B, 1024, scale=0.01)
    dY3 = rn(B, 7, 7, 64)
    dY2 = rn(B, 9, 9, 64)
    dY1 = rn(B, 20, 20, 64)
    ws = C.Workspace()
    gw = torch.empty(1024 * 3136, device=dev)
    gb = torch.empty(1024, device=dev)
    F = lambda n: 2.0 * n  # noqa: E731
    ops = {
        "conv1_fwd": (lambda: C.conv1_s2d_fwd(lib, ws, ring, slots, w1, bias[:64], 1 / 255., y1, w1t, bias[:64], 2 * B),
                      F(N3 * 400 * 64 * 256)),
        "conv2_fwd": (lambda: C.conv_fwd(lib, y1, w2, bias[:64], 2, y2, w2t, bias[:64], 2 * B), F(N3 * 81 * 64 * 1024)),
        "conv3_fwd": (lambda: C.conv_fwd(lib, y2, w3, bias[:64], 1, y3, w3t, bias[:64], 2 * B), F(N3 * 49 * 64 * 576)),
        "fc_fwd": (lambda: C.dense_fwd(lib, y3.reshape(N3, 3136), wfc, bias, h, True, None, wfct, bias, 2 * B),
                   F(N3 * 1024 * 3136)),
        "fc_dgrad": (lambda: C.dense_dgrad(lib, dH, wfc, dY3.reshape(B, 3136), y3[:B].reshape(B, 3136)),
                     F(B * 3136 * 1024)),
        "fc_wgrad": (lambda: C.dense_wgrad(lib, dH, y3[:B].reshape(B, 3136), gw.view(1024, 3136), gb),
                     F(B * 3136 * 1024)),
        "conv3_dgrad": (lambda: C.conv3_dgrad(lib, dY3, w3, y2[:B], dY2), F(B * 81 * 64 * 576)),
        "conv3_wgrad": (lambda: C.conv_wgrad(lib, ws, dY3, y2[:B], 3, 1, gw[:64 * 576].view(64, 3, 3, 64), gb[:64]),
                        F(B * 49 * 64 * 576)),
        "conv2_dgrad": (lambda: C.conv2_dgrad(lib, dY2, w2, y1[:B], dY1), F(B * 400 * 64 * 256)),
        "conv2_wgrad": (lambda: C.conv_wgrad(lib, ws, dY2, y1[:B], 4, 2, gw[:64 * 1024].view(64, 4, 4, 64), gb[:64]),
                        F(B * 81 * 64 * 1024)),
        "conv1_wgrad": (lambda: C.conv1_wgrad_ring(lib, ws, dY1, ring, slots[:B], 1 / 255., gw[:64 * 256].view(64, 4, 8, 8),
                                                   gb[:64]), F(B * 400 * 64 * 256)),
    }
    # split-size variants of the weight-gradient kernels (rows of the reduction per block)
    for tr in (128, 256, 512, 1024):
        ops[f"conv3_wgrad@{tr}"] = (lambda tr=tr: C.conv_wgrad(lib, ws, dY3, y2[:B], 3, 1, gw[:64 * 576].view(64, 3, 3, 64),
                                                              gb[:64], target_rows=tr), F(B * 49 * 64 * 576))
        ops[f"conv2_wgrad@{tr}"] = (lambda tr=tr: C.conv_wgrad(lib, ws, dY2, y1[:B], 4, 2, gw[:64 * 1024].view(64, 4, 4, 64),
                                                              gb[:64], target_rows=tr), F(B * 81 * 64 * 1024))
    ops["conv1_wgrad@tiled"] = (lambda: C.conv1_wgrad_ring_tiled(lib, ws, dY1, ring, slots[:B], 1 / 255.,
                                                                 gw[:64 * 256].view(64, 4, 8, 8), gb[:64]),
                                F(B * 400 * 64 * 256))
    for gr in (128, 512):
        ops[f"conv1_wgrad@g{gr}"] = (lambda gr=gr: C.conv1_wgrad_ring(lib, ws, dY1, ring, slots[:B], 1 / 255.,
                                                                     gw[:64 * 256].view(64, 4, 8, 8), gb[:64],
                                                                     grid=gr), F(B * 400 * 64 * 256))
    # launch-shape sweep of the forward-family GEMMs (tile 1: BM=128, 2: BM=64; order 1: M fastest, 2: N fastest)
    for tile in (1, 2):
        for order in (1, 2):
            for nm in ("fc_fwd", "fc_dgrad", "conv3_fwd", "conv2_fwd", "conv3_dgrad", "conv2_dgrad"):
                fn, fl = ops[nm]
                ops[f"{nm}@t{tile}o{order}"] = ((lambda fn=fn, tile=tile, order=order:
                                                (C.set_launch_hints(tile, order), fn(), C.set_launch_hints())), fl)
    total = 0.0
    for name, (fn, flops) in ops.items():
        if a.only and name not in a.only.split(","):
            continue
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = 1e3 * e0.elapsed_time(e1) / a.iters
        if "@" not in name:
            total += us
        print(json.dumps({"op": name, "us": round(us, 2), "tflops": round(flops / us / 1e6, 1)}), flush=True)
    print(json.dumps({"op": "TOTAL", "us": round(total, 1)}))


if __name__ == "__main__":
    main()
