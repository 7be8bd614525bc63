"""Python launchers for the MFMA implicit-GEMM family (csrc/conv_mfma.hip).

Every function writes into caller-provided buffers and launches on the
current stream, so the whole learner step is graph-capturable.  Workspaces
(wgrad split-K slabs) are cached per shape in ``Workspace``.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple


import torch

from . import _lib
from .switches import SW


class Workspace:
    def __init__(self):
        self.bufs: Dict[Tuple, torch.Tensor] = {}

    def get(self, key, numel: int, device, dtype=torch.float32) -> torch.Tensor:
        k = (key, numel, str(device), dtype)
        t = self.bufs.get(k)
        if t is None:
            t = torch.empty(numel, dtype=dtype, device=device)
            self.bufs[k] = t
        return t

    # device-side image work queues in the persistent kernels (csrc/mfma_common.h wq_next):
    # off by default (static order: each queue item costs a contended device-scope
    # atomic); the data-parallel learner turns them on, where RCCL's kernels hold CUs
    # during the conv backward.  SW.work_queue = "on" / "off" forces them on / off.
    work_queue = False

    def wq(self, key, device, overlapped: bool = True) -> int:
        """Counter pair of a work queue, or 0 (null: static order) when queues are off.
        ``overlapped``: the launch can run beside the step's collectives (the conv
        backward); the forward never does (it follows the optimizer's join), so it keeps
        the static order unless SW.work_queue = "on"."""
        mode = SW.work_queue
        on = mode == "on" or (mode != "off" and self.work_queue and overlapped)
        # one never-reset 64-bit counter per (call site, items, grid): a launch consumes
        # exactly items + grid values (csrc/mfma_common.h wq_fetch)
        return self.get_zeroed(key, 1, device, dtype=torch.int64).data_ptr() if on else 0

    def get_zeroed(self, key, numel: int, device, dtype=torch.int32) -> torch.Tensor:
        """A buffer zeroed once, when first made, and never reset: a work-queue counter
        (csrc/mfma_common.h wq_fetch) is a 64-bit count that every launch advances by
        exactly items + grid and reads modulo that, so it must serve ONE (call site,
        items, grid) on one stream -- resetting it would break the modular item map."""
        k = (key, numel, str(device), dtype)
        t = self.bufs.get(k)
        if t is None:
            t = torch.zeros(numel, dtype=dtype, device=device)
            self.bufs[k] = t
        return t


# scratch for launchers called without a workspace (tests, microbenchmarks)
_DEFAULT_WS = Workspace()

# launch-shape overrides for tuning sweeps (scripts/bench_kernels.py); 0 = kernel's choice
_HINTS: Dict[str, int] = {}


def set_launch_hints(tile: int = 0, order: int = 0) -> None:
    _HINTS["tile"], _HINTS["order"] = int(tile), int(order)


def _conv_desc(**kw) -> "_lib.ConvDesc":
    d = _lib.ConvDesc()
    d.x = kw.get("x")
    d.frame_slots = kw.get("frame_slots")
    d.w = kw["w"]
    d.bias = kw.get("bias")
    d.y = kw["y"]
    d.mask = kw.get("mask")
    d.N, d.H, d.W, d.Cin = kw["N"], kw.get("H", 1), kw.get("W", 1), kw["Cin"]
    d.OH, d.OW, d.Cout = kw.get("OH", 1), kw.get("OW", 1), kw["Cout"]
    d.KH, d.KW = kw.get("KH", 1), kw.get("KW", 1)
    d.stride, d.pad_h, d.pad_w = kw.get("stride", 1), kw.get("pad", 0), kw.get("pad", 0)
    d.mode, d.relu = kw["mode"], int(kw.get("relu", 0))
    d.ldy, d.ncls = kw.get("ldy", kw["Cout"]), kw.get("ncls", 1)
    d.ostride_h = d.ostride_w = kw.get("ostride", 1)
    d.OHfull, d.OWfull = kw.get("OHfull", d.OH), kw.get("OWfull", d.OW)
    d.K = kw["K"]
    d.in_scale = float(kw.get("scale", 1.0))
    d.w_cls_stride = kw.get("w_cls_stride", 0)
    d.w2 = kw.get("w2")
    d.bias2 = kw.get("bias2")
    d.m_switch = kw.get("m_switch", 0)
    d.bt, d.ldb = kw.get("bt", 0), kw.get("ldb", 0)
    d.tile_hint, d.order_hint = _HINTS.get("tile", 0), _HINTS.get("order", 0)
    for i, v in enumerate(kw.get("koff", ())):
        d.koff[i] = v
    # fp32-accurate ("split") mode: lo planes of A, B (both weight sets) and the output
    d.x_lo, d.w_lo, d.w2_lo, d.y_lo = kw.get("x_lo"), kw.get("w_lo"), kw.get("w2_lo"), kw.get("y_lo")
    return d


def _lo(x_lo=None, w_lo=None, w2_lo=None, out_lo=None) -> dict:
    """Descriptor fields of split mode (every tensor given, or none)."""
    if x_lo is None:
        return {}
    assert w_lo is not None and out_lo is not None
    return dict(x_lo=x_lo.data_ptr(), w_lo=w_lo.data_ptr(), w2_lo=_lib.ptr(w2_lo), y_lo=out_lo.data_ptr())


def _second(w2, b2, rows_first, per_row):
    """Descriptor fields for a second weight set on rows >= rows_first (images); the
    kernels tile the two row ranges separately (csrc/conv_mfma.hip row_tile), so the
    switch may fall on any row."""
    if w2 is None:
        return {}
    return dict(w2=w2.data_ptr(), bias2=_lib.ptr(b2), m_switch=rows_first * per_row)


def row_tiles_host(M: int, m_switch: Optional[int], bm: int) -> int:
    """Row tiles of a launch (csrc/conv_mfma.hip row_tiles): the rows before and after a
    weight switch are tiled separately."""
    if m_switch is None:
        return -(-M // bm)
    return -(-m_switch // bm) + -(-(M - m_switch) // bm)


def _launch_fwd(lib, d) -> None:
    _lib.check(lib.apex_conv_fwd(d, _lib.stream_ptr()), "conv_fwd")


def pack_w1_s2d(lib, ws: "Workspace", w1: torch.Tensor, tag: str) -> torch.Tensor:
    """OIHW conv1 weights -> s2d K order (cached buffer per tag, repacked every call)."""
    C = w1.shape[1]
    buf = ws.get(("w1s", tag), 64 * 64 * C, w1.device, torch.bfloat16)
    _lib.check(lib.apex_s2d_pack_w1(w1.data_ptr(), buf.data_ptr(), C, _lib.stream_ptr()), "s2d_pack_w1")
    return buf


def conv1_s2d_fwd(lib, ws: "Workspace", ring: torch.Tensor, slots: torch.Tensor, w1: torch.Tensor,
                  b1: torch.Tensor, scale: float, out: torch.Tensor, w2=None, b2=None, rows_first: int = 0,
                  grid: int = 0, probe: Optional[torch.Tensor] = None, w32: Optional[torch.Tensor] = None,
                  w2_32: Optional[torch.Tensor] = None, out_lo: Optional[torch.Tensor] = None,
                  c2f: Optional[Tuple] = None) -> None:
    """conv1 on the space-to-depth replay ring (persistent LDS-DMA kernel, csrc/conv1_s2d.hip).
    Split mode (``out_lo`` given): the fp32 master weights ``w32`` / ``w2_32`` (OIHW) are
    read and the output leaves as hi (``out``) / lo (``out_lo``) bf16 planes.
    ``c2f = (w2 hi, lo, target hi, lo)``: the launch also packs the split conv2 forward's
    weights for ``conv2_img_fwd(..., packed=True)`` on the same stream."""
    N, C = slots.shape
    assert out.shape == (N, 20, 20, 64) and w1.shape[1] == C and slots.dtype == torch.int32
    d = _lib.Conv1S2DDesc()
    d.ring, d.slots, d.y = ring.data_ptr(), slots.data_ptr(), out.data_ptr()
    d.w = w1.data_ptr()  # OIHW: the kernel gathers the s2d K order into LDS
    d.bias = b1.data_ptr()
    if w2 is not None:
        d.w2 = w2.data_ptr()
        d.bias2 = b2.data_ptr()
        d.m_switch = rows_first * 400
    zero = ws.get(("zero16",), 64, ring.device, torch.uint8)
    if not getattr(ws, "_zeroed", False):
        zero.zero_()
        ws._zeroed = True
    d.zero16 = zero.data_ptr()
    d.scratch = ws.get(("scratch1k",), 2048, ring.device, torch.uint8).data_ptr()
    d.N, d.C, d.in_scale = N, C, float(scale)
    if probe is not None:
        d.probe = probe.data_ptr()
    if out_lo is not None:
        assert w32 is not None and w32.dtype == torch.float32 and (w2 is None or w2_32 is not None)
        d.w32, d.w2_32, d.y_lo = w32.data_ptr(), _lib.ptr(w2_32), out_lo.data_ptr()
    if c2f is not None:
        for i, t in enumerate(c2f):
            d.c2f_src[i] = _lib.ptr(t)
        d.c2f_out = c2f_wfrag_fwd_buffer(ring.device).data_ptr()
        d.c2f_bf16 = int(out_lo is None)     # bf16 forward layout: (w2, None, target w2, None)
    _lib.check(lib.apex_conv1_s2d_fwd(d, int(grid), _lib.stream_ptr()), "conv1_s2d_fwd")


def c2f_wfrag_fwd_buffer(device) -> torch.Tensor:
    """Split conv2 forward weights of both sets in fragment order (512 KB, per stream)."""
    return _DEFAULT_WS.get(("c2f_wfrag", _lib.stream_ptr()), 4 * 8192 * 8, device, torch.bfloat16)


# conv2 (20x20x64 -> 9x9x64, 4x4/s2) on the image-resident kernel (csrc/conv2_img.hip);
# (SW.conv2_img = False selects the generic implicit GEMM)


# split conv2 forward: the launcher packs both weight sets into per-lane fragment order
# first (SW.c2f_pack; False = in-kernel gathers, the A/B of scripts/bench_split_conv2.py)


def conv2_img_fwd(lib, x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, out: torch.Tensor,
                  w2=None, b2=None, rows_first: int = 0, grid: int = 0, x_lo=None, w_lo=None, w2_lo=None,
                  out_lo=None, packed: bool = False) -> None:
    """conv2 + bias + ReLU, one persistent workgroup per CU walking whole images
    (image staged once in LDS, weights in VGPRs); online/target switch per image.
    Split mode (``x_lo`` .. ``out_lo``): the hi / lo plane kernel."""
    from .conv_sigs import Conv2ImgDesc
    N = x.shape[0]
    assert tuple(x.shape[1:]) == (20, 20, 64) and tuple(w.shape) == (64, 4, 4, 64) and tuple(out.shape) == (N, 9, 9, 64)
    assert x.is_contiguous() and out.is_contiguous() and w.is_contiguous()
    d = Conv2ImgDesc()
    d.x, d.w, d.bias, d.y = x.data_ptr(), w.data_ptr(), b.data_ptr(), out.data_ptr()
    if w2 is not None:
        assert w2.is_contiguous() and tuple(w2.shape) == (64, 4, 4, 64)
        d.w2, d.bias2 = w2.data_ptr(), b2.data_ptr()
    d.N, d.img_switch = N, int(rows_first) if w2 is not None else N
    if x_lo is not None:
        for t in (x_lo, w_lo, out_lo) + ((w2_lo,) if w2 is not None else ()):
            assert t is not None and t.is_contiguous() and t.dtype == torch.bfloat16
        d.x_lo, d.w_lo, d.w2_lo, d.y_lo = x_lo.data_ptr(), w_lo.data_ptr(), _lib.ptr(w2_lo), out_lo.data_ptr()
        if SW.c2f_pack or packed:
            d.wfrag = c2f_wfrag_fwd_buffer(x.device).data_ptr()
            d.wfrag_ready = int(packed)
    elif packed:   # bf16: fragments packed by this step's conv1 launch
        d.wfrag = c2f_wfrag_fwd_buffer(x.device).data_ptr()
        d.wfrag_ready = 1
    _lib.check(lib.apex_conv2_img_fwd(d, int(grid), _lib.stream_ptr()), "conv2_img_fwd")


# fp32 learner: conv1 -> conv2 fused with y1 kept in LDS (csrc/conv12_fused.hip);
# (SW.conv12_fused = False runs the two image-resident kernels)
CF_W1FRAG_BYTES = 2 * 2 * 2 * 2 * 4 * 2 * 64 * 16


C3F_BYTES = 4 * 4608 * 16      # csrc/conv2_wfrag.h C3F_FRAGS x 4 planes


def _conv12_desc(ws: "Workspace", ring: torch.Tensor, slots: torch.Tensor, w1, b1, w2, w2_lo, b2, scale, w1b, b1b,
                 w2b, w2b_lo, b2b, c3=None):
    from .conv_sigs import Conv12Desc
    C = int(w1.shape[1])
    assert tuple(w1.shape) == (64, C, 8, 8) and w1.dtype == torch.float32 and w1.is_contiguous()
    assert tuple(w2.shape) == (64, 4, 4, 64) and w2.dtype == torch.bfloat16
    assert w2_lo is None or w2_lo.dtype == torch.bfloat16
    d = Conv12Desc()
    d.bf16 = int(w2_lo is None)          # one bf16 plane (the bf16 learner)
    d.ring, d.slots = _lib.ptr(ring), _lib.ptr(slots)
    d.w1, d.b1, d.w2, d.w2_lo, d.b2 = w1.data_ptr(), b1.data_ptr(), w2.data_ptr(), _lib.ptr(w2_lo), b2.data_ptr()
    if w1b is not None:
        assert tuple(w1b.shape) == tuple(w1.shape) and tuple(w2b.shape) == tuple(w2.shape)
        assert (w2b_lo is None) == (w2_lo is None)
        d.w1b, d.b1b, d.w2b, d.w2b_lo, d.b2b = (w1b.data_ptr(), b1b.data_ptr(), w2b.data_ptr(), _lib.ptr(w2b_lo),
                                                 b2b.data_ptr())
    dev = w1.device
    # conv1 fragments + folded biases of both sets (csrc/conv12_fused.hip CF_W1FRAG_U4 uint4)
    # and the conv2 C2F fragments: written by the pack launch, read by every fused launch
    d.w1frag = ws.get(("cf_w1frag",), CF_W1FRAG_BYTES, dev, torch.uint8).data_ptr()
    d.scratch = ws.get(("scratch1k",), 2048, dev, torch.uint8).data_ptr()
    # (in ``ws``, not per stream: the target set packed at a sync, outside the step's
    # captured graph, must be the buffer the graph's launches read)
    d.wfrag = ws.get(("cf_c2f_wfrag",), 4 * 8192 * 16, dev, torch.uint8).data_ptr()
    d.C, d.in_scale = C, float(scale)
    if c3 is not None:
        # fused conv3: both sets' weights (packed into C3F fragments with the others)
        w3, w3l, b3, w3b, w3bl, b3t = c3
        sp = w2_lo is not None
        two = w1b is not None
        assert tuple(w3.shape) == (64, 3, 3, 64) and w3.dtype == torch.bfloat16 and w3.is_contiguous()
        assert not sp or w3l is not None
        assert not two or (w3b is not None and b3t is not None and (not sp or w3bl is not None))
        d.w3, d.w3_lo, d.b3 = w3.data_ptr(), (w3l.data_ptr() if sp else 0), b3.data_ptr()
        d.w3b, d.w3b_lo, d.b3b = (w3b.data_ptr() if two else 0), (w3bl.data_ptr() if two and sp else 0), \
            (b3t.data_ptr() if two else 0)
        d.w3frag = ws.get(("cf_c3f",), C3F_BYTES, dev, torch.uint8).data_ptr()
    return d


def conv12_pack(lib, ws: "Workspace", w1, b1, w2, w2_lo, b2, scale: float, w1b=None, b1b=None, w2b=None,
                w2b_lo=None, b2b=None, sets: int = 2, c3=None) -> None:
    """(Re)pack the fused kernel's weight fragments of ``sets`` (bit 0 online, bit 1 target)
    alone -- the learner's target sync; the step's fused launch then packs the online set
    only (``conv12_fused_fwd(pack_sets=1)``).  The input scale is folded into the conv1
    fragments: pack with the scale the forward uses."""
    d = _conv12_desc(ws, None, None, w1, b1, w2, w2_lo, b2, scale, w1b, b1b, w2b, w2b_lo, b2b, c3)
    d.pack_sets = int(sets)
    _lib.check(lib.apex_conv12_pack(d, _lib.stream_ptr()), "conv12_pack")


def conv12_frag_out(ws: "Workspace", w1: torch.Tensor, w1_off: int, w2_off: int, scale: float,
                    w3_off: Optional[int] = None):
    """``CfFragOut`` for the optimizer launch: the fused forward's online conv1 / conv2
    operand buffers of ``ws`` and the flat offsets of w1 / w2 in the parameter vector the
    optimizer updates (csrc/cf_pack.h cf_frag_store)."""
    C = int(w1.shape[1])
    dev = w1.device
    fo = _lib.CfFragOut()
    fo.w1frag = ws.get(("cf_w1frag",), CF_W1FRAG_BYTES, dev, torch.uint8).data_ptr()
    fo.c2f = ws.get(("cf_c2f_wfrag",), 4 * 8192 * 16, dev, torch.uint8).data_ptr()
    fo.w1_off, fo.w2_off, fo.C, fo.in_scale = int(w1_off), int(w2_off), C, float(scale)
    if w3_off is not None:      # the fused conv3's C3F fragments (csrc/cf_pack.h)
        fo.c3f = ws.get(("cf_c3f",), C3F_BYTES, dev, torch.uint8).data_ptr()
        fo.w3_off = int(w3_off)
    return fo


def conv12_fused_fwd(lib, ws: "Workspace", ring: torch.Tensor, slots: torch.Tensor, w1: torch.Tensor,
                     b1: torch.Tensor, w2: torch.Tensor, w2_lo: torch.Tensor, b2: torch.Tensor, scale: float,
                     y2: torch.Tensor, y2_lo: torch.Tensor, y1: Optional[torch.Tensor] = None,
                     y1_lo: Optional[torch.Tensor] = None, copy_n: int = 0, w1b=None, b1b=None, w2b=None,
                     w2b_lo=None, b2b=None, rows_first: int = 0, grid: int = 0,
                     probe: Optional[torch.Tensor] = None, pack_sets: int = 3, probe_split: int = 0,
                     c3=None, y3: Optional[torch.Tensor] = None, y3_lo: Optional[torch.Tensor] = None) -> None:
    """conv1 (fp32 OIHW weights ``w1``, exact uint8 frames from the s2d ring) + ReLU ->
    conv2 (hi / lo bf16 OHWI ``w2``, ``w2_lo``) + ReLU in one persistent launch, y1 kept
    in LDS; rows < ``copy_n`` also store y1 (hi / lo) for the backward.  Rows >=
    ``rows_first`` use the second weight set (``w1b`` ..) when given.  ``pack_sets``: the
    weight sets whose fragments the launch repacks first (the others' must be current,
    see ``conv12_pack``).  ``w2_lo`` None: the bf16 kernel (one plane; ``y1_lo``,
    ``y2_lo`` unused).  ``c3 = (w3, w3_lo, b3, w3 target, w3_lo target, b3 target)``:
    conv3 (3x3 / s1, OHWI bf16 planes) + ReLU fused too, from y2 in LDS, into ``y3``
    (``y3_lo``) [N, 7, 7, 64]; y2 is still written for every row."""
    N, C = slots.shape
    sp = w2_lo is not None
    assert slots.dtype == torch.int32 and slots.is_contiguous() and int(w1.shape[1]) == C
    assert tuple(y2.shape[:4]) == (N, 9, 9, 64) and y2.is_contiguous() and y2.dtype == torch.bfloat16
    assert not sp or (y2_lo is not None and tuple(y2_lo.shape) == (N, 9, 9, 64))
    d = _conv12_desc(ws, ring, slots, w1, b1, w2, w2_lo, b2, scale, w1b, b1b, w2b, w2b_lo, b2b, c3)
    d.img_switch = int(rows_first) if w1b is not None else N
    if copy_n > 0:
        assert y1 is not None and (y1_lo is not None or not sp) and y1.shape[0] >= copy_n and \
            tuple(y1.shape[1:]) == (20, 20, 64) and y1.is_contiguous()
        d.y1, d.y1_lo = y1.data_ptr(), (y1_lo.data_ptr() if sp else 0)
    d.copy_n = int(copy_n)
    d.y2, d.y2_lo = y2.data_ptr(), (y2_lo.data_ptr() if sp else 0)
    d.pack_sets = int(pack_sets)
    d.N = N
    d.probe = _lib.ptr(probe)
    d.probe_split = int(probe_split)
    d.wq = ws.wq(("cf_wq", N, int(grid)), ring.device, overlapped=False)
    if c3 is not None:
        assert y3 is not None and tuple(y3.shape[:4]) == (N, 7, 7, 64) and y3.is_contiguous()
        assert not sp or (y3_lo is not None and tuple(y3_lo.shape[:4]) == (N, 7, 7, 64))
        d.y3, d.y3_lo = y3.data_ptr(), (y3_lo.data_ptr() if sp else 0)
    _lib.check(lib.apex_conv12_fused_fwd(d, int(grid), _lib.stream_ptr()), "conv12_fused_fwd")


def conv_fwd(lib, x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, stride: int, out: torch.Tensor,
             w2=None, b2=None, rows_first: int = 0, x_lo=None, w_lo=None, w2_lo=None, out_lo=None,
             packed: bool = False) -> None:
    """NHWC conv + bias + ReLU with OHWI weights (conv2 / conv3).  Split mode
    (``x_lo`` ... ``out_lo``): fp32-accurate operands as hi + lo bf16 planes."""
    N, H, W, Cin = x.shape
    Cout, KH, KW, _ = w.shape
    OH, OW = out.shape[1], out.shape[2]
    if SW.conv2_img and (H, W, Cin, Cout, KH, KW, stride) == (20, 20, 64, 64, 4, 4, 2) and \
            hasattr(lib, "apex_conv2_img_fwd"):
        conv2_img_fwd(lib, x, w, b, out, w2, b2, rows_first, x_lo=x_lo, w_lo=w_lo, w2_lo=w2_lo, out_lo=out_lo,
                      packed=packed)
        return
    d = _conv_desc(x=x.data_ptr(), w=w.data_ptr(), bias=b.data_ptr(), y=out.data_ptr(), N=N, H=H, W=W,
                   Cin=Cin, OH=OH, OW=OW, Cout=Cout, KH=KH, KW=KW, stride=stride, mode=1, relu=1,
                   K=KH * KW * Cin, **_second(w2, b2, rows_first, OH * OW), **_lo(x_lo, w_lo, w2_lo, out_lo))
    _launch_fwd(lib, d)


def dense_fwd(lib, x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], out: torch.Tensor,
              relu: bool = True, mask: Optional[torch.Tensor] = None, w2=None, b2=None,
              rows_first: int = 0, ws: Optional["Workspace"] = None, x_lo=None, w_lo=None, w2_lo=None,
              out_lo=None) -> None:
    """out[M,N] = act(x[M,K] @ w[N,K]^T + b)  (or * (mask > 0)); split mode with the lo planes."""
    M, K = x.shape
    Nc = w.shape[0]
    assert w.shape[1] == K and out.shape == (M, Nc)
    d = _conv_desc(x=x.data_ptr(), w=w.data_ptr(), bias=_lib.ptr(b), y=out.data_ptr(), mask=_lib.ptr(mask),
                   N=M, Cin=K, Cout=Nc, mode=0, relu=relu and mask is None, K=K,
                   **_second(w2, b2, rows_first, 1), **_lo(x_lo, w_lo, w2_lo, out_lo))
    _launch_fwd(lib, d)


def dense_fwd128(lib, ws: "Workspace", x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor],
                 out: torch.Tensor, relu: bool = True, w2=None, b2=None, rows_first: int = 0, ksplit: int = 2,
                 loader_waves: bool = False, x_lo=None, w_lo=None, w2_lo=None, out_lo=None,
                 c2d_pack: Optional[Tuple[torch.Tensor, Optional[torch.Tensor]]] = None,
                 no_epilogue: bool = False):
    """``dense_fwd`` on 128x128 tiles with the K range split ``ksplit`` ways
    (csrc/conv_mfma.hip ``fc_gemm128_kernel``): fp32 partials in a cached workspace,
    summed in fixed order by the epilogue kernel (bias, ReLU, hi / lo planes).
    ``c2d_pack = (w2, w2_lo)``: the epilogue launch also packs conv2's weights for this
    step's conv2 data gradient (``conv2_dgrad_img(..., packed=True)``).
    ``no_epilogue``: only the GEMM runs; returns ``(partials, nz)`` for a
    consumer that finishes the epilogue itself (the DDQN head, csrc/head_common.h
    load_row_part)."""
    M, K = x.shape
    Nc = w.shape[0]
    assert w.shape[1] == K and out.shape == (M, Nc) and Nc % 128 == 0 and K % 64 == 0
    assert x.is_contiguous() and w.is_contiguous() and out.is_contiguous()
    kt = K // 64
    assert ksplit >= 1
    per = -(-kt // ksplit)
    nz = -(-kt // per)
    buf = ws.get(("fc128", _lib.stream_ptr()), nz * M * Nc, x.device)   # per stream: actors share the backend
    d = _conv_desc(x=x.data_ptr(), w=w.data_ptr(), bias=_lib.ptr(b), y=out.data_ptr(), N=M, Cin=K, Cout=Nc,
                   mode=0, relu=relu, K=K, **_second(w2, b2, rows_first, 1), **_lo(x_lo, w_lo, w2_lo, out_lo))
    from .conv_sigs import C2dPackJob
    pk = C2dPackJob()
    if c2d_pack is not None:
        pk.w, pk.w_lo = c2d_pack[0].data_ptr(), _lib.ptr(c2d_pack[1])
        pk.out = c2d_wfrag_buffer(ws, x.device).data_ptr()
    _lib.check(lib.apex_fc_gemm128(d, buf.data_ptr(), buf.numel(), int(ksplit), int(loader_waves),
                                      int(no_epilogue), pk, _lib.stream_ptr()), "fc_gemm128")
    return (buf, nz) if no_epilogue else None


def c2d_wfrag_buffer(ws: "Workspace", device) -> torch.Tensor:
    """conv2 weights in the data-gradient kernels' fragment order (hi + lo planes, 256 KB)."""
    return ws.get(("c2d_wfrag",), 2 * 8192 * 8, device, torch.bfloat16)


# K-major B-operand offsets for the dgrad GEMMs reading the natural OHWI weights.
# conv3: k-tile = output tap t of the 3x3 correlation -> weight tap 8 - t (flipped).
_KOFF3 = tuple((8 - t) * 64 for t in range(9))
# conv2 parity class (p, q), k-tile (a, b) -> weight tap (p + 2(1-a), q + 2(1-b)).
_KOFF2 = tuple(((p + 2 * (1 - a)) * 4 + (q + 2 * (1 - b))) * 64
               for p in range(2) for q in range(2) for a in range(2) for b in range(2))


def dense_dgrad(lib, dh: torch.Tensor, w: torch.Tensor, out: torch.Tensor, mask: torch.Tensor, dh_lo=None,
                w_lo=None, out_lo=None) -> None:
    """out[M,K] = (dh[M,N] @ w[N,K]) * (mask > 0): the B operand is read K-major
    straight from the natural [N][K] weight (no transposed copy)."""
    M, Nn = dh.shape
    K = w.shape[1]
    assert w.shape[0] == Nn and out.shape == (M, K)
    d = _conv_desc(x=dh.data_ptr(), w=w.data_ptr(), y=out.data_ptr(), mask=_lib.ptr(mask), N=M, Cin=Nn,
                   Cout=K, mode=0, K=Nn, bt=2, ldb=K, **_lo(dh_lo, w_lo, None, out_lo))
    _launch_fwd(lib, d)


def conv3_dgrad_img(lib, dy: torch.Tensor, w3: torch.Tensor, mask: torch.Tensor, out: torch.Tensor,
                    grid: int = 0) -> None:
    """conv3 data gradient on the image-resident kernel (csrc/conv2_img.hip): six waves
    own 32-pixel x 32-channel output tiles over the full K, dY3 in LDS."""
    from .conv_sigs import Conv3DgradImgDesc
    N = dy.shape[0]
    assert tuple(dy.shape) == (N, 7, 7, 64) and tuple(out.shape) == (N, 9, 9, 64)
    assert tuple(mask.shape) == (N, 9, 9, 64) and tuple(w3.shape) == (64, 3, 3, 64)
    assert dy.is_contiguous() and out.is_contiguous() and mask.is_contiguous() and w3.is_contiguous()
    d = Conv3DgradImgDesc()
    d.dy, d.w, d.mask, d.dx, d.N = dy.data_ptr(), w3.data_ptr(), mask.data_ptr(), out.data_ptr(), N
    _lib.check(lib.apex_conv3_dgrad_img(d, int(grid), _lib.stream_ptr()), "conv3_dgrad_img")


def conv3_dgrad(lib, dy: torch.Tensor, w3: torch.Tensor, mask: torch.Tensor, out: torch.Tensor, dy_lo=None,
                w_lo=None, out_lo=None) -> None:
    """dX2 (9x9) from dY3 (7x7): full correlation with the flipped 3x3 weights, read
    K-major from the OHWI weight (co rows, ci columns)."""
    N = dy.shape[0]
    assert w3.shape == (64, 3, 3, 64)
    if SW.conv3_dgrad_img and dy_lo is None and hasattr(lib, "apex_conv3_dgrad_img"):
        conv3_dgrad_img(lib, dy, w3, mask, out)
        return
    d = _conv_desc(x=dy.data_ptr(), w=w3.data_ptr(), y=out.data_ptr(), mask=mask.data_ptr(), N=N, H=7, W=7,
                   Cin=64, OH=9, OW=9, Cout=64, KH=3, KW=3, stride=1, pad=2, mode=1, K=576,
                   bt=1, ldb=576, koff=_KOFF3, **_lo(dy_lo, w_lo, None, out_lo))
    _launch_fwd(lib, d)


def conv2_dgrad_img(lib, dy: torch.Tensor, w2: torch.Tensor, mask: torch.Tensor, out: torch.Tensor,
                    grid: int = 0, dy_lo=None, w_lo=None, out_lo=None, ws: Optional["Workspace"] = None,
                    packed: bool = False) -> None:
    """conv2 data gradient on the image-resident kernel (csrc/conv2_img.hip): one wave
    per (stride-parity class, channel half), dY staged in LDS inside a zero ring; the
    weights are packed into per-lane fragment order first (``ws``: cached 256 KB buffer;
    ``packed``: already done earlier in the step by ``dense_fwd128(c2d_pack=...)``).
    Split mode (``dy_lo``, ``w_lo``, ``out_lo``): the hi / lo plane kernel."""
    from .conv_sigs import Conv2DgradImgDesc
    N = dy.shape[0]
    assert tuple(dy.shape) == (N, 9, 9, 64) and tuple(out.shape) == (N, 20, 20, 64)
    assert tuple(mask.shape) == (N, 20, 20, 64) and tuple(w2.shape) == (64, 4, 4, 64)
    assert dy.is_contiguous() and out.is_contiguous() and mask.is_contiguous() and w2.is_contiguous()
    d = Conv2DgradImgDesc()
    d.dy, d.w, d.mask, d.dx, d.N = dy.data_ptr(), w2.data_ptr(), mask.data_ptr(), out.data_ptr(), N
    if dy_lo is not None:
        for t in (dy_lo, w_lo, out_lo):
            assert t is not None and t.is_contiguous() and t.dtype == torch.bfloat16
        d.dy_lo, d.w_lo, d.dx_lo = dy_lo.data_ptr(), w_lo.data_ptr(), out_lo.data_ptr()
    ws = ws if ws is not None else _DEFAULT_WS
    d.wfrag = c2d_wfrag_buffer(ws, dy.device).data_ptr()
    d.wfrag_ready = int(packed)
    d.wq = ws.wq(("c2d_wq", N, int(grid)), dy.device)
    # small batches (a global-batch DP rank's rows): one workgroup per (image, class)
    d.cls_split = int(dy_lo is not None and N <= SW.conv2_dgrad_cls_max)
    _lib.check(lib.apex_conv2_dgrad_img(d, int(grid), _lib.stream_ptr()), "conv2_dgrad_img")


def conv2_dgrad(lib, dy: torch.Tensor, w2: torch.Tensor, mask: torch.Tensor, out: torch.Tensor, dy_lo=None,
                w_lo=None, out_lo=None, ws: Optional["Workspace"] = None, packed: bool = False) -> None:
    """dX1 (20x20) from dY2 (9x9), 4x4 stride 2: four stride-parity classes, each a
    2x2 stride-1 correlation (pad 1) writing every other output pixel; weights read
    K-major from the OHWI tensor per class."""
    N = dy.shape[0]
    assert w2.shape == (64, 4, 4, 64)
    if SW.conv2_dgrad_img and hasattr(lib, "apex_conv2_dgrad_img"):
        conv2_dgrad_img(lib, dy, w2, mask, out, dy_lo=dy_lo, w_lo=w_lo, out_lo=out_lo, ws=ws, packed=packed)
        return
    d = _conv_desc(x=dy.data_ptr(), w=w2.data_ptr(), y=out.data_ptr(), mask=mask.data_ptr(), N=N, H=9, W=9,
                   Cin=64, OH=10, OW=10, Cout=64, KH=2, KW=2, stride=1, pad=1, mode=1, K=256, ncls=4,
                   ostride=2, OHfull=20, OWfull=20, bt=1, ldb=1024, koff=_KOFF2, **_lo(dy_lo, w_lo, None, out_lo))
    _launch_fwd(lib, d)


def _wg_desc(**kw) -> "_lib.WgradDesc":
    d = _lib.WgradDesc()
    d.dy, d.x, d.frame_slots = kw["dy"], kw["x"], kw.get("frame_slots")
    d.slab, d.bias_slab = kw["slab"], kw.get("bias_slab")
    d.N, d.H, d.W, d.Cin = kw.get("N", 1), kw.get("H", 1), kw.get("W", 1), kw.get("Cin", 64)
    d.OH, d.OW, d.KH, d.KW = kw.get("OH", 1), kw.get("OW", 1), kw.get("KH", 1), kw.get("KW", 1)
    d.stride, d.pad_h, d.pad_w, d.mode = kw.get("stride", 1), 0, 0, kw["mode"]
    d.Co, d.Kc, d.ldd, d.ldx = kw["Co"], kw["Kc"], kw["ldd"], kw.get("ldx", 0)
    d.rows_per_split, d.Mred = kw["rows_per_split"], kw["Mred"]
    d.norm_part, d.norm_slot0 = kw.get("norm_part"), kw.get("norm_slot0", 0)
    d.dy_lo, d.x_lo = kw.get("dy_lo"), kw.get("x_lo")    # split mode (x_lo null for the exact frames)
    return d


_WG_ROWS = 64       # reduction rows per kernel step (csrc/conv_mfma.hip WG_ROWS)
_WG_TBL = 1024      # per-block row-offset table entries (WG_TBL)


def _splits(Mred: int, target_rows: int, max_rows: int) -> Tuple[int, int]:
    """Split-K partition of the reduction rows: whole 64-row steps per block
    (rows may straddle images -- the kernel's row table handles that)."""
    rows = max(_WG_ROWS, min(max_rows, (target_rows // _WG_ROWS) * _WG_ROWS))
    return (Mred + rows - 1) // rows, rows


def conv_wgrad(lib, ws: Workspace, dy: torch.Tensor, x: torch.Tensor, KH: int, stride: int,
               dw_out: torch.Tensor, db_out: torch.Tensor, target_rows: int = 0, jobs: Optional[list] = None,
               dy_lo=None, x_lo=None) -> None:
    """dW (OHWI, fp32) and db for an NHWC conv with 64 output channels.  With
    ``jobs``, the split-K reduction is appended there for ``finalize_grads``.
    ``target_rows``: reduction rows per split-K block (0 = tuned default: fewer
    rows for the small 3x3 layer, whose 9 output tiles need more splits (384: two
    68 KB blocks per CU); 704 for conv2 keeps its 4 x 59 blocks (84 KB LDS each,
    one per CU) in a single wave on 256 CUs: 3507-3572 -> 3562-3611 steps/s).  Below 256
    images (the per-rank rows of a global batch over 4+ ranks) half those rows, so the few
    images still make enough blocks: emulated W = 8 rank step 167.8 / 168.4 / 168.3 ->
    159.9 / 161.5 / 159.6 us, W = 4 ~1 %; at 290 images (W = 2) halving loses 2.5 %
    (profiles/r6_ab_wgrad_rows_small_batch.txt).
    SW.wg_rows3 / SW.wg_rows2 override for sweeps."""
    N, OH, OW, Co = dy.shape
    if target_rows <= 0:
        small = N < 256
        target_rows = {3: SW.wg_rows3, 4: SW.wg_rows2}.get(KH) or \
            ((192 if small else 384) if KH == 3 else (352 if small else 704))
    _, H, W, Cin = x.shape
    Kc = KH * KH * Cin
    Mred = N * OH * OW
    nsplit, rows = _splits(Mred, target_rows, _WG_TBL)
    slab = ws.get(("wg", Co, Kc), nsplit * Co * Kc, dy.device)
    bslab = ws.get(("wgb", Co, Kc), nsplit * Co, dy.device)
    d = _wg_desc(dy=dy.data_ptr(), x=x.data_ptr(), slab=slab.data_ptr(), bias_slab=bslab.data_ptr(), N=N,
                 H=H, W=W, Cin=Cin, OH=OH, OW=OW, KH=KH, KW=KH, stride=stride, mode=1, Co=Co, Kc=Kc, ldd=Co,
                 rows_per_split=rows, Mred=Mred, dy_lo=_lib.ptr(dy_lo), x_lo=_lib.ptr(x_lo))
    if jobs is not None:   # reduction deferred to one grad_finalize launch
        _lib.check(lib.apex_conv_wgrad(d, None, None, nsplit, 1.0, _lib.stream_ptr()), "conv_wgrad")
        jobs.append(dict(slab=slab, bslab=bslab, out=dw_out, bout=db_out, n=Co * Kc, nsplit=nsplit, nb=Co,
                         s2dC=0, Kc=Kc, scale=1.0))
        return
    _lib.check(lib.apex_conv_wgrad(d, dw_out.data_ptr(), db_out.data_ptr(), nsplit, 1.0, _lib.stream_ptr()),
               "conv_wgrad")


def conv1_wgrad_ring(lib, ws: Workspace, dy: torch.Tensor, ring: torch.Tensor, slots: torch.Tensor,
                     scale: float, dw_out: torch.Tensor, db_out: torch.Tensor, grid: int = 0,
                     jobs: Optional[list] = None, dy_lo: Optional[torch.Tensor] = None) -> None:
    """dW1 (OIHW fp32, x ``scale``) and db1 from dY1 (N, 20, 20, 64) and the uint8 frame
    stacks addressed by ring slots: image-resident kernel (csrc/conv1_wgrad.hip), one
    fp32 partial per workgroup, then the split-K reduce (s2d -> OIHW permuted store).
    Split mode (``dy_lo``): dY hi + lo against the exact frames (two MFMAs per fragment)."""
    N, OH, OW, Co = dy.shape
    C = slots.shape[1]
    assert (OH, OW, Co) == (20, 20, 64) and slots.dtype == torch.int32 and dy.is_contiguous()
    G = grid if grid > 0 else min(N, 256)
    K = 64 * C
    slab = ws.get(("wg1img", C, G), G * 64 * K, dy.device)
    bslab = ws.get(("wg1imgb", G), G * 64, dy.device)
    zero = ws.get(("zero16",), 64, ring.device, torch.uint8)
    if not getattr(ws, "_zeroed", False):
        zero.zero_()
        ws._zeroed = True
    d = _lib.Conv1WgDesc()
    d.ring, d.slots, d.dy = ring.data_ptr(), slots.data_ptr(), dy.data_ptr()
    d.slab, d.bias_slab, d.zero16 = slab.data_ptr(), bslab.data_ptr(), zero.data_ptr()
    d.N, d.C = N, C
    d.dy_lo = _lib.ptr(dy_lo)
    # item work queue where the launch runs beside the DP step's collectives (per-item
    # partial slots: the reduction does not depend on which workgroup took an item)
    d.wq = ws.wq(("c1w_wq", N, int(G)), dy.device)
    st = _lib.stream_ptr()
    _lib.check(lib.apex_conv1_wgrad_img(d, G, st), "conv1_wgrad_img")
    if jobs is not None:
        jobs.append(dict(slab=slab, bslab=bslab, out=dw_out, bout=db_out, n=64 * K, nsplit=G, nb=64, s2dC=C, Kc=K,
                         scale=float(scale)))
        return
    _lib.check(lib.apex_slab_reduce(slab.data_ptr(), G, 64 * K, float(scale), dw_out.data_ptr(), bslab.data_ptr(),
                                    64, db_out.data_ptr(), C, K, st), "slab_reduce")


def conv1_wgrad_ring_tiled(lib, ws: Workspace, dy: torch.Tensor, ring: torch.Tensor, slots: torch.Tensor,
                           scale: float, dw_out: torch.Tensor, db_out: torch.Tensor, target_rows: int = 0,
                           jobs: Optional[list] = None, dy_lo: Optional[torch.Tensor] = None) -> None:
    """The generic tiled wgrad kernel in its s2d-ring mode: the split-mode conv1 weight
    gradient (``dy_lo``) and a cross-check of the image-resident bf16 kernel."""
    if target_rows <= 0:
        target_rows = 800 if dy_lo is not None else 1024
    N, OH, OW, Co = dy.shape
    C = slots.shape[1]
    Kc = C * 64
    Mred = N * OH * OW
    nsplit, rows = _splits(Mred, target_rows, _WG_TBL // C)
    slab = ws.get(("wg1", Co, Kc), nsplit * Co * Kc, dy.device)
    bslab = ws.get(("wg1b", Co), nsplit * Co, dy.device)
    d = _wg_desc(dy=dy.data_ptr(), x=ring.data_ptr(), frame_slots=slots.data_ptr(), slab=slab.data_ptr(),
                 bias_slab=bslab.data_ptr(), N=N, H=ring.shape[1], W=ring.shape[2], Cin=C, OH=OH, OW=OW,
                 KH=8, KW=8, stride=4, mode=2, Co=Co, Kc=Kc, ldd=Co, rows_per_split=rows, Mred=Mred,
                 dy_lo=_lib.ptr(dy_lo))
    if jobs is not None:   # reduction (s2d -> OIHW permuted store) deferred to grad_finalize
        _lib.check(lib.apex_conv_wgrad(d, None, None, nsplit, 1.0, _lib.stream_ptr()), "conv1_wgrad")
        jobs.append(dict(slab=slab, bslab=bslab, out=dw_out, bout=db_out, n=Co * Kc, nsplit=nsplit, nb=Co, s2dC=C,
                         Kc=Kc, scale=float(scale)))
        return
    # the slab reduce permutes the s2d K order back to OIHW while storing
    _lib.check(lib.apex_conv_wgrad(d, dw_out.data_ptr(), db_out.data_ptr(), nsplit, float(scale),
                                   _lib.stream_ptr()), "conv1_wgrad")


_WG_SHAPES = ((1, 4), (2, 2), (4, 1), (1, 3), (1, 1), (1, 2), (2, 1))


def wgrad_blocks(Co: int, Kc: int, sp: int = 0) -> int:
    """Workgroups of one split of igemm_wgrad (mirrors csrc/igemm_wgrad.h wgrad_shape:
    ``sp`` 1 = split mode with both operands split, 2 = dY split / exact X)."""
    kt, ct = Kc // 64, Co // 64
    best, bc = (1, 1), None
    for i, (c, n) in enumerate(_WG_SHAPES):
        if kt % n or ct % c:
            continue
        if (sp == 1 and c + n > 4) or (sp == 2 and 2 * c + n > 6) or (sp == 0 and i >= 5):
            continue
        cost = (ct // c) * Kc + (kt // n) * Co
        if bc is None or cost < bc:
            best, bc = (c, n), cost
    return (kt // best[1]) * (ct // best[0])


def _dense_wgrad_desc(dy: torch.Tensor, x: torch.Tensor, dw_out: torch.Tensor, db_out: torch.Tensor,
                      norm: Optional[Tuple[torch.Tensor, int]] = None, dy_lo=None, x_lo=None):
    M, Nc = dy.shape
    K = x.shape[1]
    # row-strided operands (the gathered factor rows of the DP exchange: columns of one
    # [rows][ld] buffer); a lo plane shares its hi plane's row stride
    assert dy.stride(1) == 1 and x.stride(1) == 1
    assert dy_lo is None or dy_lo.stride() == dy.stride()
    assert x_lo is None or x_lo.stride() == x.stride()
    extra = {} if norm is None else dict(norm_part=norm[0].data_ptr(), norm_slot0=int(norm[1]))
    return _wg_desc(dy=dy.data_ptr(), x=x.data_ptr(), slab=dw_out.data_ptr(), bias_slab=db_out.data_ptr(),
                    mode=0, Co=Nc, Kc=K, ldd=dy.stride(0), ldx=x.stride(0), rows_per_split=M, Mred=M,
                    dy_lo=_lib.ptr(dy_lo), x_lo=_lib.ptr(x_lo), **extra)


def dense_wgrad(lib, dy: torch.Tensor, x: torch.Tensor, dw_out: torch.Tensor, db_out: torch.Tensor,
                norm: Optional[Tuple[torch.Tensor, int]] = None, dy_lo=None, x_lo=None) -> int:
    """dW[N,K] = dy[M,N]^T @ x[M,K] (fp32, written directly), db = sum_m dy.  With
    ``norm = (partials, slot0)`` the kernel also writes 4 squared-norm partials per
    workgroup; returns the number of slots used.  Split mode: ``dy_lo`` and ``x_lo``."""
    d = _dense_wgrad_desc(dy, x, dw_out, db_out, norm, dy_lo, x_lo)
    _lib.check(lib.apex_conv_wgrad(d, None, None, 1, 1.0, _lib.stream_ptr()), "dense_wgrad")
    return 4 * wgrad_blocks(dy.shape[1], x.shape[1], 1 if dy_lo is not None else 0)


def dense_wgrad_head_prio(lib, dy, x, dw_out, db_out, norm, Hon, dhead, g, replay, idx, gen, td, dy_lo=None,
                          x_lo=None, Hon_lo=None) -> Optional[int]:
    """The fc weight gradient (as ``dense_wgrad``), the head weight gradient and the
    priority write-back in one launch (csrc/sumtree.hip fc_wgrad_head_prio_kernel).
    Returns the norm slots used, or None when the shape is not the fused kernel's
    (nothing launched: the caller runs the three ops separately)."""
    d = _dense_wgrad_desc(dy, x, dw_out, db_out, norm, dy_lo, x_lo)
    B, A1 = dhead.shape
    rc = lib.apex_fc_wgrad_head_prio(d, Hon.data_ptr(), dhead.data_ptr(), B, A1 - 1, g["wv"].data_ptr(),
                                     g["bv"].data_ptr(), g["wa"].data_ptr(), g["ba"].data_ptr(), g["wv"].numel(),
                                     replay.tree_desc(), idx.data_ptr(), td.data_ptr(), _lib.ptr(gen),
                                     replay.gen.data_ptr(), replay.alpha, replay.eps, replay.ctr.data_ptr(),
                                     _lib.ptr(Hon_lo), _lib.ptr(replay.local_stats), _lib.stream_ptr())
    if rc == 1:          # hipErrorInvalidValue: not the compiled shape
        return None
    _lib.check(rc, "fc_wgrad_head_prio")
    return 4 * wgrad_blocks(dy.shape[1], x.shape[1], 1 if dy_lo is not None else 0)


def finalize_blocks(jobs: list, norm_range: Optional[torch.Tensor]) -> int:
    n = sum((j["n"] // 4 + 15) // 16 + (j["nb"] // 4 + 15) // 16 for j in jobs)
    return n + (1 if norm_range is not None else 0)


def finalize_job_blocks(j: dict) -> int:
    """grad_finalize blocks of one job: 16 float4 columns per block, ``cpb`` times that
    for a wide job (csrc/conv_mfma.hip RedJob)."""
    c = int(j.get("cpb", 1))
    w = 256 * -c if c < 0 else 16 * max(1, c)       # (cpb < 0: direct mode, 256 columns per pass)
    return (j["n"] // 4 + w - 1) // w + (j["nb"] // 4 + w - 1) // w


def dense_wgrad_split(lib, ws: Workspace, dy: torch.Tensor, x: torch.Tensor, nsplit: int, dw_out: torch.Tensor,
                      db_out: torch.Tensor, jobs: list, dy_lo=None, x_lo=None, cpb: int = -1,
                      jnorm: Optional[torch.Tensor] = None) -> int:
    """dW[N,K] = dy[M,N]^T @ x[M,K] as ``nsplit`` split-K partial slabs (the small-batch DP
    step's fc rows: a few row tiles over a long reduction fill the chip only when the
    reduction rows are split), reduced by the step's ``grad_finalize`` launch: the job is
    appended to ``jobs`` (``cpb``: finalize blocks of -cpb x 256 columns, one thread per
    column, the splits summed in order; with ``jnorm`` the job's squared-norm partials, one
    per finalize block).  Returns that block count."""
    M, Nc = dy.shape
    K = x.shape[1]
    rows = -(-M // nsplit)
    rows = -(-rows // 64) * 64
    nsplit = -(-M // rows)
    slab = ws.get(("wgd", Nc, K, nsplit), nsplit * Nc * K, dy.device)
    bslab = ws.get(("wgdb", Nc, nsplit), nsplit * Nc, dy.device)
    d = _dense_wgrad_desc(dy, x, slab, bslab, None, dy_lo, x_lo)
    d.rows_per_split = rows
    _lib.check(lib.apex_conv_wgrad(d, None, None, nsplit, 1.0, _lib.stream_ptr()), "dense_wgrad_split")
    j = dict(slab=slab, bslab=bslab, out=dw_out, bout=db_out, n=Nc * K, nsplit=nsplit, nb=Nc, s2dC=0, Kc=K,
             scale=1.0, cpb=int(cpb), jnorm=jnorm)
    jobs.append(j)
    return finalize_job_blocks(j)


def finalize_grads(lib, jobs: list, norm_range: Optional[torch.Tensor] = None, norm_part=None, slot0: int = 0,
                   total=None) -> int:
    """One launch for every deferred split-K reduction; with ``norm_part`` also the
    squared-norm partials of everything it writes (+ ``norm_range``) into slots from
    ``slot0``, then the grand total of ``norm_part[:slot0 + blocks]`` into ``total``
    (one small kernel).  Returns the blocks used."""
    d = _lib.FinalizeDesc()
    assert len(jobs) <= 4
    blk = 0
    for i, j in enumerate(jobs):
        J = d.job[i]
        J.slab, J.bslab, J.out, J.bout = j["slab"].data_ptr(), j["bslab"].data_ptr(), j["out"].data_ptr(), \
            j["bout"].data_ptr()
        J.n, J.nsplit, J.nb, J.s2dC, J.Kc, J.scale, J.blk0 = j["n"], j["nsplit"], j["nb"], j["s2dC"], j["Kc"], \
            j["scale"], blk
        J.cpb = int(j.get("cpb", 1))
        J.jnorm = _lib.ptr(j.get("jnorm"))
        blk += finalize_job_blocks(j)
    d.njobs = len(jobs)
    if norm_range is not None and norm_part is not None:
        d.nrm_ptr, d.nrm_n = norm_range.data_ptr(), norm_range.numel()
        blk += 1
    d.nblocks = blk
    if norm_part is not None:
        d.norm_part, d.norm_slot0 = norm_part.data_ptr(), int(slot0)
    _lib.check(lib.apex_grad_finalize(d, _lib.stream_ptr()), "grad_finalize")
    if norm_part is not None and total is not None:   # else the optimizer sums the partials itself
        _lib.check(lib.apex_norm_total(norm_part.data_ptr(), int(slot0) + blk, total.data_ptr(), _lib.stream_ptr()),
                   "norm_total")
    return blk


def pack_dgrad_weights(lib, wfc, w3, w2, wfcT, w3tf, w2t) -> None:
    _lib.check(lib.apex_pack_dgrad_weights(wfc.data_ptr(), w3.data_ptr(), w2.data_ptr(), wfcT.data_ptr(),
                                           w3tf.data_ptr(), w2t.data_ptr(), _lib.stream_ptr()), "pack")
