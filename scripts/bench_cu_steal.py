#!/usr/bin/env python
"""CU-stealing proxy benchmark: learner step time while K CUs are held
by a spinning kernel on a second stream (csrc/cu_steal.hip), standing in for RCCL's
collective kernels beside a data-parallel step on one GPU.

For each K the spinner starts first (K workgroups, one per CU: 96 KB of LDS each), then
``--steps`` learner updates replay their graphs on the main stream; their time comes
from events on the main stream only.  Ideal slowdown = 256 / (256 - K): a step whose
work moves freely between CUs.  A persistent kernel with a static split of its images
over 256 workgroups instead waits for its last K workgroups to find a CU.

    python scripts/bench_cu_steal.py --ks 0,8,16,32 --steps 80
"""
import argparse
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ks", default="0,8,16,32")
    ap.add_argument("--steps", type=int, default=80)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--lds", type=int, default=96 * 1024)
    a = ap.parse_args()
    import bench
    from apex_dqn_amd.ops import _lib, build
    _lib.require_kernels()
    # the spin kernel ships in the diagnostic library only (ops/build.py DEBUG_ONLY_SOURCES);
    # the learner keeps the release kernels
    lib = ctypes.CDLL(build.ensure_current("kernels_debug"))
    lib.apex_spin_hold.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    lib.apex_spin_hold.restype = ctypes.c_int
    dev = torch.device("cuda", 0)
    args = bench.parser().parse_args([])
    replay = bench.make_replay(args, dev, 0)
    cfg, L = bench.make_learner(args, a.dtype, dev, None, 0, replay)
    for _ in range(a.warmup):
        L.step()
    L.prepare_graphs()
    if hasattr(L, "rewarm"):
        L.rewarm(4)
    torch.cuda.synchronize()
    started = torch.zeros(1, dtype=torch.int32, device=dev)
    side = torch.cuda.Stream(dev)
    main_s = torch.cuda.current_stream(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def timed(k, hold_us):
        started.zero_()
        torch.cuda.synchronize()
        if k:
            _lib.check(lib.apex_spin_hold(k, hold_us, a.lds, ctypes.c_void_p(started.data_ptr()), side.cuda_stream),
                       "spin_hold")
            time.sleep(0.002)            # the spinner's workgroups are resident first
        ev[0].record(main_s)
        L.steps(a.steps)
        ev[1].record(main_s)
        ev[1].synchronize()
        ms = ev[0].elapsed_time(ev[1]) / a.steps
        torch.cuda.synchronize()         # the spinner's end
        return ms, int(started.item())

    base = min(timed(0, 0)[0] for _ in range(a.reps))
    hold = int(base * a.steps * 1000 * 3) + 20000
    for k in [int(x) for x in a.ks.split(",")]:
        runs = [timed(k, hold) for _ in range(a.reps)]
        ms = min(r[0] for r in runs)
        ideal = 256.0 / (256 - k)
        print(json.dumps({"K": k, "ms_per_step": round(ms, 4), "slowdown": round(ms / base, 4),
                          "ideal": round(ideal, 4), "excess_pct": round(100 * (ms / base / ideal - 1), 2),
                          "spinner_wgs_started": runs[-1][1], "dtype": a.dtype, "steps": a.steps}), flush=True)


if __name__ == "__main__":
    main()
