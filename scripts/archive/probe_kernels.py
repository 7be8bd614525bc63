#!/usr/bin/env python
"""Phase timing of the persistent image-resident kernels from in-kernel
s_memtime probes (``PROBE`` in csrc/mfma_common.h).

For each probed kernel, prints per-iteration phase durations (shader clocks,
median over the waves of the first PROBE_BLOCKS workgroups): where a persistent
workgroup's time goes (waiting for its DMA, converting, MFMA loop, barriers).
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["APEX_DEBUG_BOUNDS"] = "1"   # the diagnostic library carries the PROBE stamps

PROBE_BLOCKS, PROBE_ITERS = 4, 16


def phases(buf: torch.Tensor, nw: int, names, waves=None):
    t = buf.cpu().numpy().astype(np.int64).reshape(PROBE_BLOCKS, nw, PROBE_ITERS, 4)
    if waves is not None:
        t = t[:, waves]
    out = []
    for it in range(PROBE_ITERS):
        row = t[:, :, it, :]
        if not np.all(row > 0):
            continue
        rec = {"it": it}
        for k in range(1, 4):
            d = row[:, :, k] - row[:, :, k - 1]
            rec[names[k - 1]] = int(np.median(d))
            rec[names[k - 1] + "_max"] = int(d.max())
        if it + 1 < PROBE_ITERS and np.all(t[:, :, it + 1, 0] > 0):
            rec["tail"] = int(np.median(t[:, :, it + 1, 0] - row[:, :, 3]))
        out.append(rec)
    total = t[:, :, :, :].max() - t[t > 0].min()
    return out, int(total)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=512)
    a = ap.parse_args()
    from apex_dqn_amd.ops import _lib, conv as C
    lib = _lib.require_kernels()
    dev = torch.device("cuda", 0)
    B = a.B
    N3 = 3 * B
    g = torch.Generator(device=dev).manual_seed(0)
    bf = torch.bfloat16
    ring = torch.randint(0, 256, (100000, 84, 84), device=dev, dtype=torch.uint8, generator=g)
    slots = torch.randint(0, 100000, (N3, 4), device=dev, dtype=torch.int32, generator=g)
    w1 = (torch.randn(64, 4, 8, 8, device=dev, generator=g) * 0.05).to(bf)
    w1t = (torch.randn(64, 4, 8, 8, device=dev, generator=g) * 0.05).to(bf)
    bias = torch.randn(64, device=dev) * 0.1
    y1 = torch.empty(N3, 20, 20, 64, device=dev, dtype=bf)
    ws = C.Workspace()
    probe = torch.zeros(PROBE_BLOCKS * 8 * PROBE_ITERS * 4, dtype=torch.int64, device=dev)
    run = lambda p=None: C.conv1_s2d_fwd(lib, ws, ring, slots, w1, bias, 1 / 255., y1, w1t, bias, 2 * B,  # noqa
                                         probe=p)
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        run()
    e1.record()
    torch.cuda.synchronize()
    run(probe)
    torch.cuda.synchronize()
    print(json.dumps({"kernel": "conv1_s2d_fwd", "us": e0.elapsed_time(e1) / 20 * 1e3}))
    for grp, waves, names in (("A", [0, 1, 2, 3], ["wait", "convert", "compute"]),
                              ("B", [4, 5, 6, 7], ["compute", "wait", "convert"])):
        rows, total = phases(probe, 8, names, waves)
        print(json.dumps({"group": grp, "probe_span_clk": total}))
        for r in rows:
            print(json.dumps(r))
    t = probe.cpu().numpy().astype(np.int64).reshape(PROBE_BLOCKS, 8, PROBE_ITERS, 4)
    print(json.dumps({"span_ticks": int(t[:, :, :8].max() - t[:, :, :8][t[:, :, :8] > 0].min())}))


if __name__ == "__main__":
    main()
