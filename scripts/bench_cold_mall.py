"""Is the in-step slowdown of the fc GEMMs an Infinity-Cache (MALL) miss effect?
fc forward (split) timed warm (operands re-read every launch) and cold (a 640 MB
buffer written between launches evicts the 256 MB MALL), each as (kernel + filler)
minus filler alone, inside HIP graphs."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_tree import timed  # noqa: E402
from apex_dqn_amd.ops import _lib, conv as C  # noqa: E402


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
    o = [torch.zeros(N, 1024, device=dev, dtype=torch.bfloat16) for _ in range(2)]
    filler = torch.empty(640 << 20, dtype=torch.uint8, device=dev)
    res = {}
    for split in (False, True):
        fc = lambda: C.dense_fwd(lib, xh, wh, b, o[0], True, None, w2h, b2, 1024,
                                 **(dict(x_lo=xl, w_lo=wl, w2_lo=w2l, out_lo=o[1]) if split else {}))
        t_fc = timed(fc)
        r = {"warm_us": round(t_fc, 2)}
        for nt in (0, 1):
            fill = lambda: _lib.check(lib.apex_fill16(filler.data_ptr(), filler.numel() // 16, nt,
                                                      _lib.stream_ptr()), "fill16")
            t_fill = timed(fill)
            t_both = timed(lambda: (fill(), fc()))
            r[f"cold_nt{nt}_us"] = round(t_both - t_fill, 2)
            r[f"fill_nt{nt}_us"] = round(t_fill, 2)
        res["split" if split else "bf16"] = r
        print(json.dumps({"split": split, **r}), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(res, open("gpurun_out/cold_mall.json", "w"), indent=1)


if __name__ == "__main__":
    main()
