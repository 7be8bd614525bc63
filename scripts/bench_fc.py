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

# split-K variants (fp32 partials + dense_splitk_reduce) at the step's M = 1536
ws = C.Workspace()
for ks in (1, 2, 3, 4):
    C.DENSE_KSPLIT = ks
    us = timed(lambda: C.dense_fwd(lib, xb[:1536], w, bias32, hb[:1536], True, None, w2, bias32, 1024, ws=ws))
    print(json.dumps({"op": "igemm_fc_fwd_2sets", "ksplit": ks, "us": round(us, 2)}), flush=True)
C.DENSE_KSPLIT = 0

# two K groups per block (512 threads) vs one
for kgr in (1, 2, 3, 4, 5):
    C.DENSE_KGROUPS = kgr
    for M in (1024, 1536):
        us = timed(lambda: C.dense_fwd(lib, xb[:M], w, bias32, hb[:M], True, None, w2, bias32, 1024 if M > 1024 else 512))
        print(json.dumps({"op": "igemm_fc_fwd_2sets", "kgroups": kgr, "M": M, "us": round(us, 2)}), flush=True)
C.DENSE_KGROUPS = 1

# tile shape x K groups (tile 1: BM=128, 2: BM=64) at the step's shape
for tile in (1, 2):
    for kgr in (1, 2):
        C.DENSE_KGROUPS = kgr
        C.set_launch_hints(tile, 0)
        us = timed(lambda: C.dense_fwd(lib, xb[:1536], w, bias32, hb[:1536], True, None, w2, bias32, 1024))
        print(json.dumps({"op": "igemm_fc_fwd_2sets", "tile": tile, "kgroups": kgr, "M": 1536, "us": round(us, 2)}),
              flush=True)
C.set_launch_hints()
C.DENSE_KGROUPS = 1
