"""Library-GEMM reference points for the dueling fc layer (1536 x 3136 -> 1024 bf16):
what hipBLASLt (torch.matmul / addmm with ReLU epilogue) reaches on the same shapes as
the fused igemm fc forward / data-gradient kernels."""
import json

import torch


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
