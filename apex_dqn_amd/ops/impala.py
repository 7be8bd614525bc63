"""IMPALA-deep ResNet ops: HIP launchers (csrc/impala.hip) and the torch oracle.

Activations are "planar-16" bf16 tensors: per image C/16 planes of [H][W][16]
(shape ``(N, C/16, H, W, 16)``; the image stride may exceed the dense size, e.g.
the FC input rows of 3904 = 2*11*11*16 + 32 zero pad elements).  Conv weights
are OIHW ``(cout, cin_real, 3, 3)`` -- the torch ``nn.Conv2d`` layout -- and the
HIP kernels read them as packed MFMA fragments (``pack``), re-packed from the
bf16 master copy every step (online) or at target sync (target).

``HipImpalaOps`` and ``TorchImpalaOps`` have the same methods; the torch one is
the CPU path and the numerics oracle of every kernel (tests/test_impala.py).
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F

from . import _lib
from .switches import SW

c_p, c_i, c_i64, c_f = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float


class SconvDesc(ctypes.Structure):
    _fields_ = [("x", c_p), ("slots", c_p), ("wf", c_p), ("wf2", c_p), ("bias", c_p), ("bias2", c_p),
                ("add", c_p), ("mask", c_p), ("y", c_p), ("mask_out", c_p), ("x_img", c_i64), ("y_img", c_i64),
                ("add_img", c_i64), ("mask_img", c_i64), ("N", c_i), ("n_switch", c_i),
                ("relu_in", c_i), ("relu_out", c_i), ("scale", c_f), ("pad0", c_i)]


class SconvWgDesc(ctypes.Structure):
    _fields_ = [("dy", c_p), ("x", c_p), ("slots", c_p), ("slab", c_p), ("bslab", c_p),
                ("dy_img", c_i64), ("x_img", c_i64), ("N", c_i), ("relu_in", c_i),
                ("imgs_per_group", c_i), ("cin_real", c_i), ("amax", c_p)]


class ResDesc(ctypes.Structure):
    _fields_ = [("x", c_p), ("wf0", c_p), ("wf0b", c_p), ("b0", c_p), ("b0b", c_p), ("wf1", c_p), ("wf1b", c_p),
                ("b1", c_p), ("b1b", c_p), ("ysave", c_p), ("out", c_p), ("x_img", c_i64), ("ysave_img", c_i64),
                ("out_img", c_i64), ("N", c_i), ("n_switch", c_i), ("n_save", c_i), ("relu_out", c_i)]


class WgRedJob(ctypes.Structure):
    _fields_ = [("slab", c_p), ("out", c_p), ("bout", c_p), ("nsplit", c_i), ("NT", c_i), ("P", c_i),
                ("cin_real", c_i), ("scale", c_f), ("blk0", c_i)]


class WgRedDesc(ctypes.Structure):
    _fields_ = [("job", WgRedJob * 16), ("njobs", c_i), ("nblocks", c_i)]


class PackJob(ctypes.Structure):
    _fields_ = [("w", c_p), ("out", c_p), ("cin", c_i), ("cout", c_i), ("cin_real", c_i), ("transpose", c_i)]


class PackDesc(ctypes.Structure):
    _fields_ = [("job", PackJob * 32), ("njobs", c_i)]


# split (fp32-class) kernels: csrc/impala_split.hip
class SconvSDesc(ctypes.Structure):
    _fields_ = [("x", c_p), ("slots", c_p), ("wf", c_p), ("wf_lo", c_p), ("wf2", c_p), ("wf2_lo", c_p),
                ("bias", c_p), ("bias2", c_p), ("add", c_p), ("mask", c_p), ("y", c_p), ("mask_out", c_p),
                ("x_img", c_i64), ("y_img", c_i64), ("add_img", c_i64), ("mask_img", c_i64), ("N", c_i),
                ("n_switch", c_i), ("relu_in", c_i), ("relu_out", c_i), ("scale", c_f), ("pad0", c_i)]


class ResSDesc(ctypes.Structure):
    _fields_ = [("x", c_p), ("wf0", c_p), ("wf0_lo", c_p), ("wf0b", c_p), ("wf0b_lo", c_p), ("b0", c_p),
                ("b0b", c_p), ("wf1", c_p), ("wf1_lo", c_p), ("wf1b", c_p), ("wf1b_lo", c_p), ("b1", c_p),
                ("b1b", c_p), ("ysave", c_p), ("out", c_p), ("out_lo", c_p), ("x_img", c_i64),
                ("ysave_img", c_i64), ("out_img", c_i64), ("N", c_i), ("n_switch", c_i), ("n_save", c_i),
                ("relu_out", c_i)]


class SconvWgSDesc(ctypes.Structure):
    _fields_ = [("dy", c_p), ("x", c_p), ("slots", c_p), ("slab", c_p), ("dy_img", c_i64), ("x_img", c_i64),
                ("N", c_i), ("relu_in", c_i), ("imgs_per_group", c_i), ("cin_real", c_i), ("amax", c_p)]


_SIGS = {
    "apex_sconv_fwd": ([SconvDesc, c_i, c_i, c_i, c_i, c_i, c_i, c_p], c_i),
    "apex_sconv_wgrad": ([SconvWgDesc, c_i, c_i, c_i, c_i, c_i, c_i, c_p], c_i),
    "apex_sconv_wgrad_bands": ([c_i, c_i, c_i, c_i, c_i], c_i),
    "apex_maxpool_fwd": ([c_p, c_i64, c_i, c_i, c_i, c_p, c_i64, c_p, c_i, c_p], c_i),
    "apex_maxpool_bwd": ([c_p, c_i64, c_p, c_i, c_i, c_i, c_p, c_i64, c_i, c_p], c_i),
    "apex_sconv_pack": ([PackDesc, c_p], c_i),
    "apex_resblock_fwd": ([ResDesc, c_i, c_i, c_i, c_p], c_i),
    "apex_sconv_wgrad_reduce": ([WgRedDesc, c_p], c_i),
    "apex_sconv_frag_elems": ([c_i, c_i], c_i64),
    "apex_sconv_fwd_split": ([SconvSDesc, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_p], c_i),
    "apex_resblock_fwd_split": ([ResSDesc, c_i, c_i, c_i, c_p], c_i),
    "apex_sconv_wgrad_split": ([SconvWgSDesc, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_i, c_p], c_i),
    "apex_sconv_wgrad_split_rows": ([c_i, c_i, c_i, c_i, c_i, c_i, c_i], c_i),
    "apex_maxpool_bwd_split": ([c_p, c_i64, c_p, c_i, c_i, c_i, c_p, c_i64, c_i, c_p], c_i),
    "apex_merge_split": ([c_p, c_p, c_p, c_i64, c_p], c_i),
}


def declare(lib: ctypes.CDLL) -> None:
    for name, (args, res) in _SIGS.items():
        fn = getattr(lib, name, None)
        if fn is not None:
            fn.argtypes, fn.restype = args, res


# ----------------------------------------------------------------- layouts
def to_planar(x: torch.Tensor) -> torch.Tensor:
    """(N, C, H, W) -> (N, C/16, H, W, 16)."""
    N, C, H, W = x.shape
    return x.reshape(N, C // 16, 16, H, W).permute(0, 1, 3, 4, 2).contiguous()


def from_planar(x: torch.Tensor) -> torch.Tensor:
    """(N, P, H, W, 16) -> (N, 16 P, H, W)."""
    N, P, H, W, _ = x.shape
    return x.permute(0, 1, 4, 2, 3).reshape(N, P * 16, H, W)


def frag_elems(cin: int, cout: int) -> int:
    P, NT = cin // 16, cout // 16
    return ((9 * P + 1) // 2) * NT * 512


def img_stride(t: torch.Tensor) -> int:
    return int(t.stride(0))


@dataclass
class ConvSpec:
    """One 3x3 / pad 1 conv of the trunk: logical channels (multiples of 16;
    ``cin_real`` < ``cin`` for the 4-frame input), master views and fragments."""
    name: str
    cin: int
    cout: int
    cin_real: int
    H: int
    W: int
    w: torch.Tensor = None          # fp32 master (view of the flat params)
    b: torch.Tensor = None
    wb: torch.Tensor = None         # bf16 compute copy (view)
    frag: torch.Tensor = None       # forward fragments (online)
    fragT: torch.Tensor = None      # data-gradient fragments (online)
    frag_tgt: torch.Tensor = None   # forward fragments (target)
    # split mode (fp32-class): fragments of the lo plane of the bf16 weight copy
    # (v = hi + lo); the lo weight views are extra["wl"] / extra["w_tgt_lo"]
    frag_lo: torch.Tensor = None
    fragT_lo: torch.Tensor = None
    frag_tgt_lo: torch.Tensor = None
    extra: Dict = field(default_factory=dict)


# weight-gradient launch shape: workgroups per conv (images are split into groups, one
# fp32 partial per workgroup and band) and the cap on the partial slab (floats)
WGRAD_TUNING = {"target_wgs": SW.impala_wg_target, "slab_cap": SW.impala_slab_cap}


# fused residual block: rows per workgroup band per (channels, size); 0 = kernel default
RESBLOCK_BANDS = {(16, 42): SW.resblock_r16}   # swept: 21 777, 14 786, 11 778


def _split_bands() -> Dict[tuple, int]:
    """Row bands of the split kernels (csrc/impala_split.hip: 0 = the kernel default):
    resblock (C, HW) and sconv (cin, cout, HW, pool); SW.isplit_bands = "key=R;..." with
    keys like rb16x42 / sc16x16x42p0 overrides (APEX_SWITCHES sweeps)."""
    # defaults from the band sweep (profiles/r3_impala_split_band_sweep.txt: each +0.6 to
    # +2.4 % on the fp32 IMPALA step; 2 workgroups per CU where the 16-channel shapes fit)
    # round 5: the stack-1 pooled conv at 6 rows (3 workgroups per CU; 472.6-473.2 vs
    # 470.0-470.2 updates/s at 10, 469.4-470.5 at 4)
    # the 32 x 32 x 21² weight gradients at 256 workgroups (128 per band: half the partial
    # slab for the reduce; 504.3-505.1 vs 497.9-498.3 at 512, 491.1-492.2 at 128)
    out: Dict[tuple, int] = {("rb", 16, 42): 7, ("sc", 16, 16, 42, 0): 21, ("sc", 32, 16, 42, 0): 11,
                             ("sc", 16, 32, 42, 1): 6, ("sc", 16, 16, 84, 1): 6, ("wt", 32, 32, 21): 256}
    for item in SW.isplit_bands.split(";"):
        if "=" not in item:
            continue
        k, v = item.split("=")
        if k.startswith("rb"):
            c, hw = k[2:].split("x")
            out[("rb", int(c), int(hw))] = int(v)
        elif k.startswith("sc"):
            a, p = k[2:].split("p")
            ci, co, hw = a.split("x")
            out[("sc", int(ci), int(co), int(hw), int(p))] = int(v)
        elif k.startswith("wt"):                 # weight-gradient workgroup target: "wt32x32x11=128"
            ci, co, hw = k[2:].split("x")
            out[("wt", int(ci), int(co), int(hw))] = int(v)
        elif k.startswith("wg"):                 # weight gradient: "wg16x16x42=11/512" (rows / threads)
            ci, co, hw = k[2:].split("x")
            r, _, t = v.partition("/")
            out[("wg", int(ci), int(co), int(hw))] = (int(r), int(t or 0))
    return out


SPLIT_BANDS = _split_bands()


# ------------------------------------------------------------------ HIP backend
class HipImpalaOps:
    name = "hip"

    def __init__(self):
        self.lib = _lib.require_kernels()
        declare(self.lib)
        self.ws: Dict = {}

    def _buf(self, key, n, device, dtype=torch.float32):
        t = self.ws.get(key)
        if t is None or t.numel() < n:
            t = torch.empty(n, dtype=dtype, device=device)
            self.ws[key] = t
        return t

    # -- weights
    def pack(self, jobs: List[tuple]) -> None:
        """jobs: (w_bf16_oihw, out, cin, cout, cin_real, kind): kind 0 = forward
        fragments, 1 = data-gradient (transposed + flipped), 2 = the 4-frame ring
        conv's tap-pair layout."""
        for s in range(0, len(jobs), 32):
            d = PackDesc()
            chunk = jobs[s:s + 32]
            for i, (w, out, cin, cout, cin_real, tr) in enumerate(chunk):
                J = d.job[i]
                J.w, J.out, J.cin, J.cout, J.cin_real, J.transpose = w.data_ptr(), out.data_ptr(), cin, cout, \
                    cin_real, int(tr)
            d.njobs = len(chunk)
            _lib.check(self.lib.apex_sconv_pack(d, _lib.stream_ptr()), "sconv_pack")

    # -- convs
    def conv_pool(self, x, spec: ConvSpec, y, amax, *, second=None, n_switch=0, scale=1.0, ring=None,
                  slots=None, amax_rows: int = 0) -> None:
        """y = maxpool3x3s2(conv3x3(x) * scale + b) (+ argmax codes for images <
        ``amax_rows``, all if 0): the fused stack-entry kernel; the full-resolution
        conv output stays in LDS."""
        self._amax_rows = int(amax_rows)
        try:
            self.conv(x, spec, y, second=second, n_switch=n_switch, scale=scale, ring=ring, slots=slots,
                      _pool_amax=amax)
        finally:
            self._amax_rows = 0

    def conv(self, x, spec: ConvSpec, y, *, transpose=False, relu_in=False, relu_out=False, add=None, mask=None,
             bias=True, second=None, n_switch=0, scale=1.0, ring=None, slots=None,
             _pool_amax=False) -> None:
        """y = epi(corr3x3(x', W')): W' = W (forward) or transposed + flipped (data
        gradient); x' = relu(x) if relu_in; epi = *scale + bias, * (mask > 0), + add, relu.
        fp32 ``y``: the split (fp32-class) kernel, fp32 x / add / mask, hi + lo fragments."""
        if y.dtype == torch.float32:
            return self._conv_split(x, spec, y, transpose, relu_in, relu_out, add, mask, bias, second, n_switch,
                                    scale, ring, slots, _pool_amax)
        d = SconvDesc()
        pool = _pool_amax is not False
        if pool:
            d.mask_out = _lib.ptr(_pool_amax)
            d.pad0 = getattr(self, "_amax_rows", 0)
        N = y.shape[0]
        if ring is not None:   # 4 frames from the s2d ring, tap-pair K (fragments packed with mode 2)
            d.x, d.slots, d.x_img = ring.data_ptr(), slots.data_ptr(), 0
            mode = 3
            assert slots.shape == (N, 4) and slots.dtype == torch.int32 and spec.cin == 16 and not transpose
        else:
            assert x.shape[0] == N
            d.x, d.x_img = x.data_ptr(), img_stride(x)
            mode = 0
        d.wf = (spec.fragT if transpose else spec.frag).data_ptr()
        if second is not None:
            d.wf2 = spec.frag_tgt.data_ptr()
            d.bias2 = second.data_ptr() if bias else None
            d.n_switch = int(n_switch)
        d.bias = spec.b.data_ptr() if (bias and not transpose) else None
        if transpose:
            d.bias2 = None
        d.add, d.add_img = _lib.ptr(add), (img_stride(add) if add is not None else 0)
        d.mask, d.mask_img = _lib.ptr(mask), (img_stride(mask) if mask is not None else 0)
        d.y, d.y_img = y.data_ptr(), img_stride(y)
        d.N, d.relu_in, d.relu_out, d.scale = N, int(relu_in), int(relu_out), float(scale)
        cin, cout = (spec.cout, spec.cin) if transpose else (spec.cin, spec.cout)
        _lib.check(self.lib.apex_sconv_fwd(d, cin, cout, spec.H, spec.W, mode, int(pool), _lib.stream_ptr()),
                   f"sconv_fwd[{spec.name}{'^T' if transpose else ''}{'+pool' if pool else ''}]")

    def _conv_split(self, x, spec, y, transpose, relu_in, relu_out, add, mask, bias, second, n_switch, scale, ring,
                    slots, _pool_amax) -> None:
        d = SconvSDesc()
        pool = _pool_amax is not False
        if pool:
            d.mask_out = _lib.ptr(_pool_amax)
            d.pad0 = getattr(self, "_amax_rows", 0)
        N = y.shape[0]
        if ring is not None:
            d.x, d.slots, d.x_img = ring.data_ptr(), slots.data_ptr(), 0
            mode = 3
            assert slots.shape == (N, 4) and slots.dtype == torch.int32 and spec.cin == 16 and not transpose
        else:
            assert x.shape[0] == N and x.dtype == torch.float32
            d.x, d.x_img = x.data_ptr(), img_stride(x)
            mode = 0
        f, fl = (spec.fragT, spec.fragT_lo) if transpose else (spec.frag, spec.frag_lo)
        assert fl is not None, f"{spec.name}: no lo fragments (split mode packs them)"
        d.wf, d.wf_lo = f.data_ptr(), fl.data_ptr()
        if second is not None:
            d.wf2, d.wf2_lo = spec.frag_tgt.data_ptr(), spec.frag_tgt_lo.data_ptr()
            d.bias2 = second.data_ptr() if bias else None
            d.n_switch = int(n_switch)
        d.bias = spec.b.data_ptr() if (bias and not transpose) else None
        if transpose:
            d.bias2 = None
        for t in (add, mask):
            assert t is None or t.dtype == torch.float32
        d.add, d.add_img = _lib.ptr(add), (img_stride(add) if add is not None else 0)
        d.mask, d.mask_img = _lib.ptr(mask), (img_stride(mask) if mask is not None else 0)
        d.y, d.y_img = y.data_ptr(), img_stride(y)
        d.N, d.relu_in, d.relu_out, d.scale = N, int(relu_in), int(relu_out), float(scale)
        cin, cout = (spec.cout, spec.cin) if transpose else (spec.cin, spec.cout)
        R = SPLIT_BANDS.get(("sc", cin, cout, spec.H, int(pool)), 0)
        _lib.check(self.lib.apex_sconv_fwd_split(d, cin, cout, spec.H, spec.W, mode, int(pool), R, _lib.stream_ptr()),
                   f"sconv_fwd_split[{spec.name}{'^T' if transpose else ''}{'+pool' if pool else ''}]")

    def resblock(self, x, c0: ConvSpec, c1: ConvSpec, out, *, ysave=None, n_save=0, target=False, n_switch=0,
                 relu_out=False, out_lo=None) -> None:
        """out = x + conv1(relu(conv0(relu(x)))) (+ ReLU) in one kernel; conv0's output
        goes to ``ysave`` for images < ``n_save`` only; images >= ``n_switch`` use the
        target weights when ``target``.  fp32 ``x``: the split kernel; with ``out_lo`` the
        output is written as bf16 hi (``out``) + lo planes (the fc GEMM's split operand)."""
        if x.dtype == torch.float32:
            return self._resblock_split(x, c0, c1, out, ysave, n_save, target, n_switch, relu_out, out_lo)
        d = ResDesc()
        d.x, d.x_img = x.data_ptr(), img_stride(x)
        d.wf0, d.b0, d.wf1, d.b1 = c0.frag.data_ptr(), c0.b.data_ptr(), c1.frag.data_ptr(), c1.b.data_ptr()
        if target:
            d.wf0b, d.b0b = c0.frag_tgt.data_ptr(), c0.extra["b_tgt"].data_ptr()
            d.wf1b, d.b1b = c1.frag_tgt.data_ptr(), c1.extra["b_tgt"].data_ptr()
            d.n_switch = int(n_switch)
        if ysave is not None:
            d.ysave, d.ysave_img, d.n_save = ysave.data_ptr(), img_stride(ysave), int(n_save)
        d.out, d.out_img = out.data_ptr(), img_stride(out)
        d.N, d.relu_out = x.shape[0], int(relu_out)
        R = RESBLOCK_BANDS.get((c0.cin, c0.H), 0)
        _lib.check(self.lib.apex_resblock_fwd(d, c0.cin, c0.H, R, _lib.stream_ptr()), f"resblock_fwd[{c0.name}]")

    def _resblock_split(self, x, c0, c1, out, ysave, n_save, target, n_switch, relu_out, out_lo) -> None:
        d = ResSDesc()
        d.x, d.x_img = x.data_ptr(), img_stride(x)
        assert c0.frag_lo is not None and c1.frag_lo is not None
        d.wf0, d.wf0_lo, d.b0 = c0.frag.data_ptr(), c0.frag_lo.data_ptr(), c0.b.data_ptr()
        d.wf1, d.wf1_lo, d.b1 = c1.frag.data_ptr(), c1.frag_lo.data_ptr(), c1.b.data_ptr()
        if target:
            d.wf0b, d.wf0b_lo, d.b0b = c0.frag_tgt.data_ptr(), c0.frag_tgt_lo.data_ptr(), c0.extra["b_tgt"].data_ptr()
            d.wf1b, d.wf1b_lo, d.b1b = c1.frag_tgt.data_ptr(), c1.frag_tgt_lo.data_ptr(), c1.extra["b_tgt"].data_ptr()
            d.n_switch = int(n_switch)
        if ysave is not None:
            assert ysave.dtype == torch.float32
            d.ysave, d.ysave_img, d.n_save = ysave.data_ptr(), img_stride(ysave), int(n_save)
        if out_lo is not None:
            assert out.dtype == torch.bfloat16 and out_lo.dtype == torch.bfloat16 and out.stride() == out_lo.stride()
        else:
            assert out.dtype == torch.float32
        d.out, d.out_lo, d.out_img = out.data_ptr(), _lib.ptr(out_lo), img_stride(out)
        d.N, d.relu_out = x.shape[0], int(relu_out)
        R = SPLIT_BANDS.get(("rb", c0.cin, c0.H), 0)
        _lib.check(self.lib.apex_resblock_fwd_split(d, c0.cin, c0.H, R, _lib.stream_ptr()),
                   f"resblock_fwd_split[{c0.name}]")

    def merge(self, hi, lo, out) -> None:
        """out (fp32) = hi + lo (bf16 planes of the same shape)."""
        assert hi.is_contiguous() and lo.is_contiguous() and out.is_contiguous() and hi.numel() == out.numel()
        _lib.check(self.lib.apex_merge_split(hi.data_ptr(), lo.data_ptr(), out.data_ptr(), out.numel(),
                                             _lib.stream_ptr()), "merge_split")

    def wgrad(self, dy, x, spec: ConvSpec, gw, gb, jobs: list, *, relu_in=False, ring=None, slots=None,
              groups: int = 0, scale: float = 1.0, pool_amax=None) -> None:
        """gw = scale * sum dy (x) im2col(x') (x' = relu(x) if relu_in), gb = sum dy:
        partials now, reduced by ``finalize(jobs)``.  pool_amax: dy is the gradient of
        the 3x3/s2 max pool after this conv (its argmax codes); the ring conv (both
        precisions) forms the conv output gradient inside its staging, the others get it
        from maxpool_bwd."""
        N = dy.shape[0]
        mode = 2 if ring is not None else 0
        split = dy.dtype == torch.float32
        fuse_pool = pool_amax is not None and mode == 2
        if pool_amax is not None and not fuse_pool:
            shape = (N, spec.cout // 16, spec.H, spec.W, 16)
            full = self._buf(("pool_dx", spec.name), math.prod(shape), dy.device, dy.dtype)[:math.prod(shape)]
            full = full.view(shape)
            self.maxpool_bwd(dy, pool_amax, full)
            dy = full
        if split:
            R, nthr = SPLIT_BANDS.get(("wg", spec.cin, spec.cout, spec.H), (0, 0))
            rows = self.lib.apex_sconv_wgrad_split_rows(spec.cin, spec.cout, spec.H, spec.W, mode, R, nthr)
            bands = (spec.H + rows - 1) // rows if rows > 0 else 0
        else:
            bands = self.lib.apex_sconv_wgrad_bands(spec.cin, spec.cout, spec.H, spec.W, mode)
        if bands <= 0:
            raise ValueError(f"no wgrad kernel for {spec}")
        NT, P = spec.cout // 16, spec.cin // 16
        n = (NT * 9 * P + NT) * 256          # partial floats per split (accumulator order)
        target = SPLIT_BANDS.get(("wt", spec.cin, spec.cout, spec.H), WGRAD_TUNING["target_wgs"])
        G = groups or max(1, min(N, target // bands))
        while not groups and G > 32 and bands * G * n > WGRAD_TUNING["slab_cap"]:   # slab floats
            G //= 2
        ipg = (N + G - 1) // G
        G = (N + ipg - 1) // ipg
        nsplit = bands * G
        slab = self._buf(("slab", spec.name), nsplit * n, dy.device)
        d = SconvWgSDesc() if split else SconvWgDesc()
        d.dy, d.dy_img = dy.data_ptr(), img_stride(dy)
        if ring is not None:
            d.x, d.slots, d.x_img = ring.data_ptr(), slots.data_ptr(), 0
        else:
            d.x, d.x_img = x.data_ptr(), img_stride(x)
        d.slab = slab.data_ptr()
        d.N, d.relu_in, d.imgs_per_group, d.cin_real = N, int(relu_in), ipg, spec.cin_real
        d.amax = pool_amax.data_ptr() if fuse_pool else None
        if split:
            assert x is None or x.dtype == torch.float32
            _lib.check(self.lib.apex_sconv_wgrad_split(d, spec.cin, spec.cout, spec.H, spec.W, mode, R, nthr, G,
                                                       _lib.stream_ptr()), f"sconv_wgrad_split[{spec.name}]")
        else:
            _lib.check(self.lib.apex_sconv_wgrad(d, spec.cin, spec.cout, spec.H, spec.W, mode, G, _lib.stream_ptr()),
                       f"sconv_wgrad[{spec.name}]")
        jobs.append(dict(slab=slab, out=gw, bout=gb, nsplit=nsplit, NT=NT, P=P, cin_real=spec.cin_real,
                         scale=float(scale), cols=(NT * 9 * P + NT) * 64))

    def finalize(self, jobs: list) -> None:
        """One launch: sum every conv's split partials -> OIHW gradient + bias."""
        for s0 in range(0, len(jobs), 16):
            d = WgRedDesc()
            blk = 0
            for i, j in enumerate(jobs[s0:s0 + 16]):
                J = d.job[i]
                J.slab, J.out, J.bout = j["slab"].data_ptr(), j["out"].data_ptr(), j["bout"].data_ptr()
                J.nsplit, J.NT, J.P, J.cin_real, J.scale, J.blk0 = j["nsplit"], j["NT"], j["P"], j["cin_real"], \
                    j["scale"], blk
                blk += (j["cols"] + 15) // 16
            d.njobs, d.nblocks = min(16, len(jobs) - s0), blk
            _lib.check(self.lib.apex_sconv_wgrad_reduce(d, _lib.stream_ptr()), "sconv_wgrad_reduce")

    # -- pooling
    def maxpool(self, x, y, amax) -> None:
        N, P, H, W, _ = x.shape
        _lib.check(self.lib.apex_maxpool_fwd(x.data_ptr(), img_stride(x), P, H, W, y.data_ptr(), img_stride(y),
                                             _lib.ptr(amax), N, _lib.stream_ptr()), "maxpool_fwd")

    def maxpool_bwd(self, dy, amax, dx) -> None:
        N, P, H, W, _ = dx.shape
        if dx.dtype == torch.float32:
            assert dy.dtype == torch.float32
            _lib.check(self.lib.apex_maxpool_bwd_split(dy.data_ptr(), img_stride(dy), amax.data_ptr(), P, H, W,
                                                       dx.data_ptr(), img_stride(dx), N, _lib.stream_ptr()),
                       "maxpool_bwd_split")
            return
        _lib.check(self.lib.apex_maxpool_bwd(dy.data_ptr(), img_stride(dy), amax.data_ptr(), P, H, W, dx.data_ptr(),
                                             img_stride(dx), N, _lib.stream_ptr()), "maxpool_bwd")


# ---------------------------------------------------------------- torch oracle
def ring_frames(ring: torch.Tensor, slots: torch.Tensor) -> torch.Tensor:
    """(N, 4) slots into the space-to-depth ring -> (N, 4, 84, 84) uint8 frames."""
    from ..replay.gpu_replay import from_s2d
    raw = ring[slots.long().reshape(-1)]
    return from_s2d(raw.reshape(-1, 84, 84)).reshape(slots.shape[0], slots.shape[1], 84, 84)


class TorchImpalaOps:
    """Same contract, plain torch (fp32 math, results cast to the output dtype)."""
    name = "torch"

    def pack(self, jobs) -> None:
        pass

    @staticmethod
    def _w(spec: ConvSpec, transpose: bool, second: bool) -> torch.Tensor:
        w = (spec.extra["w_tgt"] if second else spec.wb).float()
        if spec.cin_real < spec.cin:
            w = F.pad(w, (0, 0, 0, 0, 0, spec.cin - spec.cin_real))
        if transpose:
            w = w.transpose(0, 1).flip(2, 3)
        return w

    def conv_pool(self, x, spec: ConvSpec, y, amax, *, second=None, n_switch=0, scale=1.0, ring=None,
                  slots=None, amax_rows: int = 0) -> None:
        N = y.shape[0]
        c0 = torch.zeros(N, spec.cout // 16, spec.H, spec.W, 16, dtype=y.dtype, device=y.device)
        self.conv(x, spec, c0, second=second, n_switch=n_switch, scale=scale, ring=ring, slots=slots)
        self.maxpool(c0, y, amax)

    def resblock(self, x, c0: ConvSpec, c1: ConvSpec, out, *, ysave=None, n_save=0, target=False, n_switch=0,
                 relu_out=False, out_lo=None) -> None:
        dt = x.dtype if out_lo is not None else out.dtype
        y = torch.zeros(x.shape[0], c0.cout // 16, c0.H, c0.W, 16, dtype=dt, device=out.device)
        t0 = dict(second=c0.extra["b_tgt"], n_switch=n_switch) if target else {}
        t1 = dict(second=c1.extra["b_tgt"], n_switch=n_switch) if target else {}
        self.conv(x, c0, y, relu_in=True, **t0)
        if out_lo is None:
            self.conv(y, c1, out, relu_in=True, add=x, relu_out=relu_out, **t1)
        else:    # bf16 hi / lo planes of the block output
            o = torch.zeros_like(y)
            self.conv(y, c1, o, relu_in=True, add=x, relu_out=relu_out, **t1)
            out.copy_(o.to(out.dtype))
            out_lo.copy_((o - out.to(o.dtype)).to(out_lo.dtype))
        if ysave is not None:
            ysave[:n_save].copy_(y[:n_save])

    def merge(self, hi, lo, out) -> None:
        out.copy_(hi.to(out.dtype) + lo.to(out.dtype))

    def conv(self, x, spec: ConvSpec, y, *, transpose=False, relu_in=False, relu_out=False, add=None, mask=None,
             bias=True, second=None, n_switch=0, scale=1.0, ring=None, slots=None) -> None:
        N = y.shape[0]
        cdt = torch.float64 if y.dtype == torch.float64 else torch.float32
        if ring is not None:
            xin = F.pad(ring_frames(ring, slots).to(cdt), (0, 0, 0, 0, 0, 12))
        else:
            xin = from_planar(x.to(cdt))
        if relu_in:
            xin = xin.clamp_min(0)
        outs = []
        for lo, hi, sec in ((0, n_switch if second is not None else N, False), (n_switch, N, True)):
            if hi <= lo or (sec and second is None):
                continue
            w = self._w(spec, transpose, sec).to(cdt)
            b = None
            if bias and not transpose:
                b = (second if sec else spec.b).to(cdt)
            o = F.conv2d(xin[lo:hi], w, None, padding=1) * scale
            if b is not None:
                o = o + b[None, :, None, None]
            outs.append(o)
        o = to_planar(torch.cat(outs))
        if mask is not None:
            o = o * (mask.to(cdt) > 0)
        if add is not None:
            o = o + add.to(cdt)
        if relu_out:
            o = o.clamp_min(0)
        y.copy_(o.to(y.dtype))

    def wgrad(self, dy, x, spec: ConvSpec, gw, gb, jobs: list, *, relu_in=False, ring=None, slots=None,
              groups: int = 0, scale: float = 1.0, pool_amax=None) -> None:
        if pool_amax is not None:
            full = torch.zeros(dy.shape[0], spec.cout // 16, spec.H, spec.W, 16, dtype=dy.dtype, device=dy.device)
            self.maxpool_bwd(dy, pool_amax, full)
            dy = full
        cdt = torch.float64 if gw.dtype == torch.float64 else torch.float32
        if ring is not None:
            xin = ring_frames(ring, slots).to(cdt)
        else:
            xin = from_planar(x.to(cdt))[:, :spec.cin_real]
        if relu_in:
            xin = xin.clamp_min(0)
        g = from_planar(dy.to(cdt))
        gw.copy_(torch.nn.grad.conv2d_weight(xin, gw.shape, g, padding=1) * scale)
        gb.copy_(g.sum((0, 2, 3)))

    def finalize(self, jobs) -> None:
        pass

    def maxpool(self, x, y, amax) -> None:
        xn = from_planar(x if x.dtype == torch.float64 else x.float())
        o, idx = F.max_pool2d(xn, 3, 2, 1, return_indices=True)
        y.copy_(to_planar(o).to(y.dtype))
        if amax is not None:
            H, W = xn.shape[2:]
            Ho, Wo = o.shape[2:]
            ih, iw = idx // W, idx % W
            oh = torch.arange(Ho, device=x.device)[:, None]
            ow = torch.arange(Wo, device=x.device)[None, :]
            code = (ih - (2 * oh - 1)) * 3 + (iw - (2 * ow - 1))
            amax.copy_(to_planar(code).to(torch.uint8))

    def maxpool_bwd(self, dy, amax, dx) -> None:
        N, P, H, W, _ = dx.shape
        cdt = torch.float64 if dx.dtype == torch.float64 else torch.float32
        g = from_planar(dy.to(cdt))
        code = from_planar(amax.long())
        Ho, Wo = g.shape[2:]
        oh = torch.arange(Ho, device=dy.device)[:, None]
        ow = torch.arange(Wo, device=dy.device)[None, :]
        ih = 2 * oh - 1 + code // 3
        iw = 2 * ow - 1 + code % 3
        flat = (ih * W + iw).reshape(N, P * 16, -1)
        out = torch.zeros(N, P * 16, H * W, dtype=cdt, device=dy.device)
        out.scatter_add_(2, flat, g.reshape(N, P * 16, -1))
        dx.copy_(to_planar(out.reshape(N, P * 16, H, W)).to(dx.dtype))
