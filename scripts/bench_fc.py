"""Library-GEMM reference points for the dueling fc layer (1536 x 3136 -> 1024 bf16):
what hipBLASLt (torch.matmul / addmm with ReLU epilogue) reaches on the same shapes as
the fused igemm fc forward / data-gradient kernels."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters=200):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


dev = "cuda"
bf = torch.bfloat16
x = torch.randn(1536, 3136, device=dev, dtype=bf)
w = torch.randn(1024, 3136, device=dev, dtype=bf) * 0.02
w2 = torch.randn(1024, 3136, device=dev, dtype=bf) * 0.02
b = torch.zeros(1024, device=dev, dtype=bf)
dy = torch.randn(512, 1024, device=dev, dtype=bf)
out = torch.empty(1536, 1024, device=dev, dtype=bf)
for name, fn in [
    ("linear_1536", lambda: torch.nn.functional.linear(x, w, b)),
    ("addmm_relu_1536", lambda: torch._addmm_activation(b, x, w.t(), use_gelu=False)),
    ("two_linear_1024_512", lambda: (torch.nn.functional.linear(x[:1024], w, b), torch.nn.functional.linear(x[1024:], w2, b))),
    ("dgrad_512x1024x3136", lambda: dy @ w),
    ("wgrad_1024x3136_k512", lambda: dy.t() @ x[:512]),
]:
    us = timed(fn)
    print(json.dumps({"op": name, "us": round(us, 2)}), flush=True)

# tile-count sensitivity of the fused fc forward (64-row tiles x 16 column tiles):
# 256 / 384 / 512 / 768 workgroups on 256 CUs
from apex_dqn_amd.ops import _lib, conv as C  # noqa: E402
lib = _lib.require_kernels()
xb = torch.relu(torch.randn(3072, 3136, device=dev)).to(bf)
hb = torch.empty(3072, 1024, device=dev, dtype=bf)
bias32 = torch.zeros(1024, device=dev)
for M in (512, 1024, 1536, 2048, 3072):
    us = timed(lambda: C.dense_fwd(lib, xb[:M], w, bias32, hb[:M], True))
    print(json.dumps({"op": "igemm_fc_fwd", "M": M, "us": round(us, 2), "tflops": round(2 * M * 1024 * 3136 / us / 1e6, 1)}),
          flush=True)

# tile shape (1: BM=128, 2: BM=64) at the step's shape, both weight sets in one launch
for tile in (1, 2):
    C.set_launch_hints(tile, 0)
    us = timed(lambda: C.dense_fwd(lib, xb[:1536], w, bias32, hb[:1536], True, None, w2, bias32, 1024))
    print(json.dumps({"op": "igemm_fc_fwd_2sets", "tile": tile, "M": 1536, "us": round(us, 2)}), flush=True)
C.set_launch_hints()

# fp32 accuracy: the split (hi + lo bf16, 3 MFMAs) fc forward vs the library's fp32 GEMM
x32 = torch.relu(torch.randn(1536, 3136, device=dev))
w32 = torch.randn(1024, 3136, device=dev) * 0.02
xh, wh = x32.to(bf), w32.to(bf)
xl, wl = (x32 - xh.float()).to(bf), (w32 - wh.float()).to(bf)
hh, hl = torch.empty(1536, 1024, device=dev, dtype=bf), torch.empty(1536, 1024, device=dev, dtype=bf)
us = timed(lambda: C.dense_fwd(lib, xh, wh, bias32, hh, True, x_lo=xl, w_lo=wl, out_lo=hl))
ref = torch.relu(x32.double() @ w32.double().t())
err = float(((hh.float() + hl.float()).double() - ref).norm() / ref.norm())
us_lib = timed(lambda: torch.relu(torch.nn.functional.linear(x32, w32)))
err_lib = float((torch.relu(torch.nn.functional.linear(x32, w32)).double() - ref).norm() / ref.norm())
print(json.dumps({"op": "fc_fwd_fp32_split_vs_hipblaslt_fp32", "M": 1536, "split_us": round(us, 2),
                  "split_rel_err": err, "lib_fp32_us": round(us_lib, 2), "lib_rel_err": err_lib}), flush=True)
