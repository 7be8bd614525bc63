#!/usr/bin/env python
"""conv1 s2d forward experiments: locality of the frame ring and grid size."""
import json, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from apex_dqn_amd.ops import _lib, conv as C

lib = _lib.require_kernels()
dev = torch.device("cuda", 0)
N3 = 1536
g = torch.Generator(device=dev).manual_seed(0)
ring = torch.randint(0, 256, (20000, 84, 84), device=dev, dtype=torch.uint8, generator=g)
w1 = (torch.randn(64, 4, 8, 8, device=dev) * 0.05).to(torch.bfloat16)
b = torch.zeros(64, device=dev)
y1 = torch.empty(N3, 20, 20, 64, device=dev, dtype=torch.bfloat16)
ws = C.Workspace()
def run(slots, grid, iters=20):
    fn = lambda: C.conv1_s2d_fwd(lib, ws, ring, slots, w1, b, 1/255., y1, w1, b, 1024, grid=grid)
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters): fn()
    e1.record(); torch.cuda.synchronize()
    return 1e3 * e0.elapsed_time(e1) / iters
rand = torch.randint(0, 20000, (N3, 4), device=dev, dtype=torch.int32, generator=g)
small = torch.randint(0, 8, (N3, 4), device=dev, dtype=torch.int32, generator=g)
for name, sl in (("random20k", rand), ("l2resident8", small)):
    for grid in (128, 256, 512, 0):
        print(json.dumps({"slots": name, "grid": grid, "us": round(run(sl, grid), 2)}), flush=True)
