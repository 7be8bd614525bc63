import torch, sys, os
sys.path.insert(0, os.getcwd())
from apex_dqn_amd.ops import _lib, conv as C
lib = _lib.require_kernels()
dev = torch.device("cuda", 0)
g = torch.Generator(device="cpu").manual_seed(1)
for N in (3, 64, 3):
    dy = torch.randn(N, 9, 9, 64, generator=g).to(dev, torch.bfloat16)
    dyl = (torch.randn(N, 9, 9, 64, generator=g) * 1e-3).to(dev, torch.bfloat16)
    w = (torch.randn(64, 4, 4, 64, generator=g) * 0.03).to(dev, torch.bfloat16)
    wl = (torch.randn(64, 4, 4, 64, generator=g) * 1e-4).to(dev, torch.bfloat16)
    y1 = torch.randn(N, 20, 20, 64, generator=g).to(dev, torch.bfloat16)
    h = torch.full((N, 20, 20, 64), float("nan"), device=dev, dtype=torch.bfloat16)
    l = torch.full_like(h, float("nan"))
    ws = C._DEFAULT_WS
    wq = ws.get_zeroed(("c2d_wq",), 2, dev)
    print("N", N, "wq before", wq.tolist())
    C.conv2_dgrad_img(lib, dy, w, y1, h, dy_lo=dyl, w_lo=wl, out_lo=l)
    torch.cuda.synchronize()
    print("wq after", wq.tolist(), "nan per image", [int(torch.isnan(h[i].float()).sum()) for i in range(min(N, 6))],
          [int(torch.isnan(l[i].float()).sum()) for i in range(min(N, 6))], flush=True)
    nz = torch.nonzero(torch.isnan(l[0].float()))
    print("nan idx img0 (pix_h, pix_w, ch):", nz[:12].tolist(), flush=True)
    # same run with outputs pre-zeroed: any inf in hi?
    h.zero_(); l.zero_()
    C.conv2_dgrad_img(lib, dy, w, y1, h, dy_lo=dyl, w_lo=wl, out_lo=l)
    torch.cuda.synchronize()
    print("inf in hi:", int(torch.isinf(h.float()).sum()), "nan in lo after zero-fill:", int(torch.isnan(l.float()).sum()), flush=True)
