"""PyTorch implementations of every fused-learner op, in the engine's layouts.

Layouts (chosen for the MFMA implicit-GEMM kernels, see csrc/conv_mfma.hip):
* frames: uint8 NCHW (B, C, 84, 84), channel = stacked frame (gathered from the
  replay frame ring by slot index);
* activations: NHWC (B, H, W, 64), post-ReLU;
* conv1 weight: OIHW (reference layout; K ordered (c, kh, kw) = 8-byte rows of a frame);
* conv2/conv3 weights: OHWI (K ordered (kh, kw, ci), 64 contiguous channels);
* fc weight: (1024, 3136) -- rows [0,512) value stream, [512,1024) advantage
  stream; columns in (h, w, c) order to match NHWC flattening.

These functions are the CPU implementation and the numerics oracle the HIP
kernels are tested against (fp32 references of the same ops).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _nchw(x):
    return x.permute(0, 3, 1, 2)


def _nhwc(x):
    return x.permute(0, 2, 3, 1)


def conv1_fwd(frames_u8: torch.Tensor, w1: torch.Tensor, b1: torch.Tensor, scale: float,
              dtype=torch.float32) -> torch.Tensor:
    x = frames_u8.to(dtype) * scale
    y = F.conv2d(x, w1.to(dtype), b1.to(dtype), stride=4)
    return _nhwc(F.relu(y)).contiguous()


def conv_fwd(x_nhwc: torch.Tensor, w_ohwi: torch.Tensor, b: torch.Tensor, stride: int,
             dtype=torch.float32) -> torch.Tensor:
    w = w_ohwi.permute(0, 3, 1, 2).to(dtype)
    y = F.conv2d(_nchw(x_nhwc).to(dtype), w, b.to(dtype), stride=stride)
    return _nhwc(F.relu(y)).contiguous()


def fc_fwd(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, dtype=torch.float32) -> torch.Tensor:
    return F.relu(x.to(dtype) @ w.to(dtype).t() + b.to(dtype))


def fc_bwd(dh: torch.Tensor, x: torch.Tensor, w: torch.Tensor, x_mask_src: torch.Tensor,
           dtype=torch.float32):
    """dh (B,N) grad at pre-ReLU fc output; x (B,K) input; returns dx (masked by x>0), dw, db."""
    dhf = dh.to(dtype)
    dx = (dhf @ w.to(dtype)) * (x_mask_src > 0).to(dtype)
    dw = dhf.t().float() @ x.float()
    db = dhf.float().sum(0)
    return dx, dw, db


def conv_dgrad(dy_nhwc: torch.Tensor, w_ohwi: torch.Tensor, in_shape_nhwc, stride: int,
               x_mask_src: torch.Tensor, dtype=torch.float32) -> torch.Tensor:
    """Grad wrt the conv input (NHWC), masked by the producer's ReLU (x > 0)."""
    B, H, W, C = in_shape_nhwc
    w = w_ohwi.permute(0, 3, 1, 2).to(dtype)
    dx = torch.nn.grad.conv2d_input((B, C, H, W), w, _nchw(dy_nhwc).to(dtype), stride=stride)
    return (_nhwc(dx) * (x_mask_src > 0).to(dtype)).contiguous()


def conv_wgrad(dy_nhwc: torch.Tensor, x_nhwc: torch.Tensor, k: int, stride: int):
    """dW in OHWI (fp32) and db (fp32)."""
    Cout = dy_nhwc.shape[-1]
    Cin = x_nhwc.shape[-1]
    dw = torch.nn.grad.conv2d_weight(_nchw(x_nhwc).float(), (Cout, Cin, k, k), _nchw(dy_nhwc).float(),
                                     stride=stride)
    return dw.permute(0, 2, 3, 1).contiguous(), dy_nhwc.float().sum((0, 1, 2))


def conv1_wgrad(dy_nhwc: torch.Tensor, frames_u8: torch.Tensor, scale: float):
    """dW1 in OIHW (fp32) and db1."""
    Cout = dy_nhwc.shape[-1]
    C = frames_u8.shape[1]
    x = frames_u8.float() * scale
    dw = torch.nn.grad.conv2d_weight(x, (Cout, C, 8, 8), _nchw(dy_nhwc).float(), stride=4)
    return dw, dy_nhwc.float().sum((0, 1, 2))
