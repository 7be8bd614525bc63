"""What IEEE fp32 would cost (round 3's verdict, weak #7): the learner's fc forward shape
(1,536 x 3,136 -> 1,024 with an online / target weight switch at row 1,024) as
  split      our fp32-class kernel (bf16 hi + lo operands, three MFMA products,
             ops.conv.dense_fwd128 -- the step's path)
  bf16       our kernel on bf16 operands (one product)
  torch_fp32 torch.matmul in fp32 (hipBLASLt; TF32 off: v_mfma_f32_*_f32 at 1/16 the
             bf16 rate), two GEMMs for the two weight sets
  torch_bf16 torch.matmul in bf16
each timed inside a HIP graph of repeated launches (scripts/bench_tree.py:timed).  A
3-plane split (hi + mid + lo, six products for fp32-exact operands) would cost ~2x the
split time."""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from bench_tree import timed  # noqa: E402
from apex_dqn_amd.ops import _lib, conv as C  # noqa: E402


def main():
    torch.backends.cuda.matmul.allow_tf32 = False
    dev = torch.device("cuda", 0)
    lib = _lib.require_kernels()
    M, K, N, r = 1536, 3136, 1024, 1024
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.relu(torch.randn(M, K, generator=g)).to(dev)
    w = (torch.randn(N, K, generator=g) * 0.02).to(dev)
    w2 = (torch.randn(N, K, generator=g) * 0.02).to(dev)
    b = torch.zeros(N, device=dev)

    def sp(t):
        hi = t.to(torch.bfloat16)
        return hi, (t - hi.float()).to(torch.bfloat16)

    (xh, xl), (wh, wl), (w2h, w2l) = sp(x), sp(w), sp(w2)
    out, out_lo = torch.empty(M, N, device=dev, dtype=torch.bfloat16), torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ws = C.Workspace()
    res = {}
    res["split_us"] = timed(lambda: C.dense_fwd128(lib, ws, xh, wh, b, out, True, w2h, b, r, 2, True, x_lo=xl, w_lo=wl,
                                                   w2_lo=w2l, out_lo=out_lo))
    res["bf16_us"] = timed(lambda: C.dense_fwd128(lib, ws, xh, wh, b, out, True, w2h, b, r, 2, True))
    o32 = torch.empty(M, N, device=dev)
    res["torch_fp32_us"] = timed(lambda: (torch.matmul(x[:r], w.T, out=o32[:r]), torch.matmul(x[r:], w2.T, out=o32[r:])))
    o16 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    res["torch_bf16_us"] = timed(lambda: (torch.matmul(xh[:r], wh.T, out=o16[:r]), torch.matmul(xh[r:], w2h.T, out=o16[r:])))
    ref = torch.cat([x[:r].double() @ w.double().T, x[r:].double() @ w2.double().T]).clamp_min(0)
    C.dense_fwd128(lib, ws, xh, wh, b, out, True, w2h, b, r, 2, True, x_lo=xl, w_lo=wl, w2_lo=w2l, out_lo=out_lo)
    torch.matmul(x[:r], w.T, out=o32[:r])
    torch.matmul(x[r:], w2.T, out=o32[r:])
    torch.cuda.synchronize()
    rel = lambda a: float(((a - ref).abs() / (ref.abs() + 1e-1)).max())   # noqa: E731
    res["split_rel_err_vs_fp64"] = rel(out.double() + out_lo.double())
    res["torch_fp32_rel_err_vs_fp64"] = rel(o32.double().clamp_min(0))
    res["gflop"] = 2 * M * N * K / 1e9
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) and v > 1e-3 else v) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
