"""ctypes signatures of the conv / GEMM kernel family (csrc/conv_mfma.hip, csrc/gemm_mfma.hip)."""
from __future__ import annotations

import ctypes

c_p = ctypes.c_void_p
c_i = ctypes.c_int
c_i64 = ctypes.c_int64
c_f = ctypes.c_float


def declare(lib: ctypes.CDLL) -> None:
    from ._lib import ConvDesc, WgradDesc
    sigs = {
        "apex_conv_fwd": ([ConvDesc, c_p], c_i),
        "apex_conv_wgrad": ([WgradDesc, c_p, c_p, c_i, c_f, c_p], c_i),
        "apex_pack_dgrad_weights": ([c_p, c_p, c_p, c_p, c_p, c_p, c_p], c_i),
    }
    for name, (args, res) in sigs.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.argtypes = args
        fn.restype = res
