#!/usr/bin/env python
"""Per-layer error of the split IMPALA backward (csrc/impala_split.hip) on a real step:
every backward op of the HIP learner is re-run in fp64 (torch oracle) on the HIP's own
fp32 inputs, so each line is one kernel's error on learner data, not an accumulation.
The same op in fp32 torch is printed beside it (the conditioning of that op).
    python scripts/diag_impala_split.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
    from test_impala_split import _learner
    from apex_dqn_amd.ops.impala import ConvSpec, TorchImpalaOps
    torch.backends.cudnn.enabled = False
    L = _learner("fp32", "hip")
    L._seg1()
    L._seg2()
    torch.cuda.synchronize()
    tops = TorchImpalaOps()
    B = L.B

    def ref_spec(cs, dt):
        r = ConvSpec(cs.name, cs.cin, cs.cout, cs.cin_real, cs.H, cs.W, w=cs.w, b=cs.b, wb=cs.w.to(dt))
        return r

    def rel(a, b):
        a, b = a.double(), b.double()
        return float((a - b).norm() / (b.norm() + 1e-30))

    dO = L.dfeat32[:, :3872].view(B, 2, 11, 11, 16)
    for s in (2, 1, 0):
        f, b = L.fw[s], L.bw[s]
        c0, r0a, r0b, r1a, r1b = L.specs[s]
        steps = [("d_yb", r1b, dO, f["yb"][:B], None),
                 ("d_ra", r1a, b["d_yb"], f["ra"][:B], dO),
                 ("d_ya", r0b, b["d_ra"], f["ya"][:B], None),
                 ("d_p", r0a, b["d_ya"], f["p"][:B], b["d_ra"])]
        for name, cs, dy, mask, add in steps:
            out = {}
            for dt in (torch.float64, torch.float32):
                y = torch.zeros(b[name].shape, dtype=dt, device=dy.device)
                tops.conv(dy.to(dt), ref_spec(cs, dt), y, transpose=True, mask=mask.to(dt),
                          add=None if add is None else add.to(dt))
                out[dt] = y
            print(f"stack {s} {name}: hip vs fp64 {rel(b[name], out[torch.float64]):.2e}   "
                  f"torch fp32 vs fp64 {rel(out[torch.float32], out[torch.float64]):.2e}   "
                  f"|add|/|out| {0 if add is None else float(add.norm() / out[torch.float64].norm()):.2f}",
                  flush=True)
        if s > 0:
            dc = b["d_c0"]
            y = torch.zeros(L.bw[s - 1]["d_o"].shape, dtype=torch.float64, device=dc.device)
            tops.conv(dc.double(), ref_spec(c0, torch.float64), y, transpose=True)
            print(f"stack {s} d_o(prev): hip vs fp64 {rel(L.bw[s - 1]['d_o'], y):.2e}", flush=True)
            dO = L.bw[s - 1]["d_o"]


if __name__ == "__main__":
    main()
