"""ctypes signatures of the conv / GEMM kernel family (csrc/conv_mfma.hip, csrc/conv2_img.hip)."""
from __future__ import annotations

import ctypes

c_p = ctypes.c_void_p
c_i = ctypes.c_int
c_i64 = ctypes.c_int64
c_f = ctypes.c_float


class Conv2ImgDesc(ctypes.Structure):
    """Image-resident conv2 forward (mirrors ``Conv2ImgDesc`` in csrc/conv2_img.hip)."""
    _fields_ = [("x", c_p), ("w", c_p), ("w2", c_p), ("bias", c_p), ("bias2", c_p), ("y", c_p),
                ("N", c_i), ("img_switch", c_i), ("x_lo", c_p), ("w_lo", c_p), ("w2_lo", c_p), ("y_lo", c_p),
                ("wfrag", c_p), ("wfrag_ready", c_i)]


class Conv12Desc(ctypes.Structure):
    """Fused conv1 -> conv2 forward, split or bf16 (mirrors ``Conv12Desc`` in csrc/conv12_fused.hip)."""
    _fields_ = [("ring", c_p), ("slots", c_p), ("w1", c_p), ("w1b", c_p), ("b1", c_p), ("b1b", c_p),
                ("w2", c_p), ("w2_lo", c_p), ("w2b", c_p), ("w2b_lo", c_p), ("wfrag", c_p), ("pack_sets", c_i),
                ("b2", c_p), ("b2b", c_p), ("y1", c_p), ("y1_lo", c_p), ("y2", c_p), ("y2_lo", c_p),
                ("w1frag", c_p), ("scratch", c_p), ("N", c_i), ("C", c_i), ("img_switch", c_i), ("copy_n", c_i),
                ("in_scale", ctypes.c_float), ("probe", c_p), ("wq", c_p), ("bf16", c_i), ("probe_split", c_i),
                ("w3", c_p), ("w3_lo", c_p), ("w3b", c_p), ("w3b_lo", c_p), ("b3", c_p), ("b3b", c_p),
                ("y3", c_p), ("y3_lo", c_p), ("w3frag", c_p)]


class Conv2DgradImgDesc(ctypes.Structure):
    """Image-resident conv2 data gradient (mirrors ``Conv2DgradImgDesc`` in csrc/conv2_img.hip)."""
    _fields_ = [("dy", c_p), ("w", c_p), ("mask", c_p), ("dx", c_p), ("N", c_i), ("dy_lo", c_p), ("w_lo", c_p),
                ("dx_lo", c_p), ("wfrag", c_p), ("wfrag_ready", c_i), ("wq", c_p), ("cls_split", c_i)]


class C2dPackJob(ctypes.Structure):
    """conv2 weight-fragment pack riding on the fc epilogue launch (``C2dPackJob``)."""
    _fields_ = [("w", c_p), ("w_lo", c_p), ("out", c_p)]


class Conv3DgradImgDesc(ctypes.Structure):
    """Image-resident conv3 data gradient (mirrors ``Conv3DgradImgDesc`` in csrc/conv2_img.hip)."""
    _fields_ = [("dy", c_p), ("w", c_p), ("mask", c_p), ("dx", c_p), ("N", c_i)]


def declare(lib: ctypes.CDLL) -> None:
    from ._lib import ConvDesc, WgradDesc
    sigs = {
        "apex_conv2_img_fwd": ([Conv2ImgDesc, c_i, c_p], c_i),
        "apex_conv12_fused_fwd": ([Conv12Desc, c_i, c_p], c_i),
        "apex_conv12_pack": ([Conv12Desc, c_p], c_i),
        "apex_conv2_dgrad_img": ([Conv2DgradImgDesc, c_i, c_p], c_i),
        "apex_conv3_dgrad_img": ([Conv3DgradImgDesc, c_i, c_p], c_i),
        "apex_conv_fwd": ([ConvDesc, c_p], c_i),
        "apex_fc_gemm128": ([ConvDesc, c_p, c_i64, c_i, c_i, c_i, C2dPackJob, c_p], c_i),
        "apex_conv_wgrad": ([WgradDesc, c_p, c_p, c_i, c_f, c_p], c_i),
        "apex_pack_dgrad_weights": ([c_p, c_p, c_p, c_p, c_p, c_p, c_p], c_i),
    }
    for name, (args, res) in sigs.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.argtypes = args
        fn.restype = res
