#!/usr/bin/env python
"""Phase timing of the fused conv1 -> conv2 kernel (csrc/conv12_fused.hip) from its
in-kernel s_memtime probes (diagnostic library, PROBE in csrc/mfma_common.h), plus
wall time of the release kernel for a few variants (copy_n, grid).
Phases per image: conv1 (MFMA loop), wait+barrier+copy-out, conv2 (MFMA loop),
tail (reduction, y2 epilogue, barriers, next DMA issue)."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def setup(B, dev):
    g = torch.Generator(device=dev).manual_seed(0)
    N = 3 * B
    ring = torch.randint(0, 256, (20000, 84, 84), device=dev, dtype=torch.uint8, generator=g)
    slots = torch.randint(0, 20000, (N, 4), device=dev, dtype=torch.int32, generator=g)
    w1 = torch.randn(64, 4, 8, 8, device=dev, generator=g) * 0.05
    w2 = torch.randn(64, 4, 4, 64, device=dev, generator=g) * 0.03
    w2h = w2.to(torch.bfloat16)
    w2l = (w2 - w2h.float()).to(torch.bfloat16)
    b = torch.randn(64, device=dev, generator=g) * 0.1
    y1 = torch.empty(B, 20, 20, 64, device=dev, dtype=torch.bfloat16)
    y1l = torch.empty_like(y1)
    y2 = torch.empty(N, 9, 9, 64, device=dev, dtype=torch.bfloat16)
    y2l = torch.empty_like(y2)
    w3 = torch.randn(64, 3, 3, 64, device=dev, generator=g) * 0.04
    w3h = w3.to(torch.bfloat16)
    w3l = (w3 - w3h.float()).to(torch.bfloat16)
    y3 = torch.empty(N, 7, 7, 64, device=dev, dtype=torch.bfloat16)
    return dict(ring=ring, slots=slots, w1=w1, w2h=w2h, w2l=w2l, b=b, y1=y1, y1l=y1l, y2=y2, y2l=y2l, N=N,
                w3h=w3h, w3l=w3l, y3=y3, y3l=torch.empty_like(y3))


def launch(lib, C, ws, t, B, copy=True, grid=0, probe=None, bf16=False, split=0, conv3=False):
    lo = (lambda k: None) if bf16 else (lambda k: t[k])      # noqa: E731
    C.conv12_fused_fwd(lib, ws, t["ring"], t["slots"], t["w1"], t["b"], t["w2h"], lo("w2l"), t["b"], 1 / 255.0,
                       t["y2"], lo("y2l"), y1=t["y1"], y1_lo=lo("y1l"), copy_n=B if copy else 0, w1b=t["w1"],
                       b1b=t["b"], w2b=t["w2h"], w2b_lo=lo("w2l"), b2b=t["b"], rows_first=2 * B, grid=grid,
                       probe=probe, probe_split=split,
                       **(dict(c3=(t["w3h"], lo("w3l"), t["b"], t["w3h"], lo("w3l"), t["b"]), y3=t["y3"],
                               y3_lo=lo("y3l")) if conv3 else {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=512)
    ap.add_argument("--probe", action="store_true")
    ap.add_argument("--split", type=int, default=0, help="probe: wait for the first frames before the weights")
    ap.add_argument("--conv3", action="store_true", help="conv3 fused too (c3)")
    ap.add_argument("--bf16", action="store_true", help="the bf16 learner's one-plane kernel")
    a = ap.parse_args()
    if a.probe:
        os.environ["APEX_DEBUG_BOUNDS"] = "1"
    from apex_dqn_amd.ops import _lib, conv as C
    lib = _lib.require_kernels()
    dev = torch.device("cuda", 0)
    t = setup(a.B, dev)
    ws = C.Workspace()
    if a.probe:
        buf = torch.zeros(4 * 4 * 16 * 4, dtype=torch.int64, device=dev)
        for _ in range(3):
            launch(lib, C, ws, t, a.B, bf16=a.bf16)
        buf.zero_()
        launch(lib, C, ws, t, a.B, probe=buf, bf16=a.bf16, split=a.split, conv3=a.conv3)
        torch.cuda.synchronize()
        st = buf.cpu().numpy().reshape(4, 4, 16, 4)
        p13 = st[:, :, 13, :]        # fused conv3 of image 0 (--conv3): y2 -> LDS, MFMA loop, epilogue
        if np.all(p13 > 0):
            print(json.dumps({"conv3_y2_to_lds": int(np.median(p13[:, :, 1] - p13[:, :, 0])),
                              "conv3_mfma_loop": int(np.median(p13[:, :, 2] - p13[:, :, 1])),
                              "conv3_epilogue": int(np.median(p13[:, :, 3] - p13[:, :, 2]))}))
        p14 = st[:, :, 14, :]        # prologue: dma issue, [frames landed], weights landed
        print(json.dumps({"split": a.split, "entry_to_dma_issue": int(np.median(p14[:, :, 0] - st[:, :, 15, 0])),
                          "dma_issue": int(np.median(p14[:, :, 1] - p14[:, :, 0])),
                          "to_before_weights": int(np.median(p14[:, :, 2] - p14[:, :, 1])),
                          "weights": int(np.median(p14[:, :, 3] - p14[:, :, 2])),
                          "barrier_to_conv1": int(np.median(st[:, :, 0, 0] - p14[:, :, 3]))}))
        names = ["conv1", "wait_copy", "conv2"]
        sp = st[:, :, 15, :]          # kernel entry / exit stamps (csrc/conv12_fused.hip)
        last = max(it for it in range(13) if np.all(st[:, :, it, 0] > 0))
        print(json.dumps({"prologue_to_conv1_it0": int(np.median(st[:, :, 0, 0] - sp[:, :, 0])),
                          "last_conv2_end_to_exit": int(np.median(sp[:, :, 1] - st[:, :, last, 3])),
                          "block_wall_us_realtime": float(np.median(sp[:, :, 3] - sp[:, :, 2])) / 100.0,
                          "entry_skew_us": float(sp[:, :, 2].max() - sp[:, :, 2].min()) / 100.0}))
        for it in range(13):
            row = st[:, :, it, :]
            if not np.all(row > 0):
                continue
            rec = {"it": it}
            for k in range(1, 4):
                rec[names[k - 1]] = int(np.median(row[:, :, k] - row[:, :, k - 1]))
            if it + 1 < 16 and np.all(st[:, :, it + 1, 0] > 0):
                rec["tail"] = int(np.median(st[:, :, it + 1, 0] - row[:, :, 3]))
            print(json.dumps(rec))
        return
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for name, kw in (("copy", dict(copy=True)), ("nocopy", dict(copy=False)), ("copy_g240", dict(copy=True, grid=240))):
        for _ in range(5):
            launch(lib, C, ws, t, a.B, bf16=a.bf16, **kw)
        ts = []
        for _ in range(20):
            ev[0].record()
            launch(lib, C, ws, t, a.B, bf16=a.bf16, **kw)
            ev[1].record()
            torch.cuda.synchronize()
            ts.append(ev[0].elapsed_time(ev[1]) * 1e3)
        print(json.dumps({"variant": name, "us_median": round(float(np.median(ts)), 1),
                          "us_min": round(float(np.min(ts)), 1)}))


if __name__ == "__main__":
    main()
