"""ctypes binding of ``libapex_kernels.so`` (C ABI, built in-tree by ``ops/build.py``).

The library is loaded *after* torch so that its ``libamdhip64.so.7`` NEEDED
entry resolves (by SONAME) to the HIP runtime torch already loaded: kernels
then share torch's device context and run on torch's current stream
(``torch.cuda.current_stream().cuda_stream``), so they are captured by
``torch.cuda.graph`` like any torch op.

On a GPU host a missing or stale library is an error (``require_kernels``),
never a silent fallback: the torch implementations in ``ops/reference.py``
exist only for CPU runs and as test oracles.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch

from . import build as _build

c_p = ctypes.c_void_p
c_i = ctypes.c_int
c_i64 = ctypes.c_int64
c_u64 = ctypes.c_uint64
c_f = ctypes.c_float


class TreeDesc(ctypes.Structure):
    _fields_ = [("leaf", c_p), ("nodes", c_p), ("off", c_i64 * 8), ("n", c_i64 * 8), ("L", c_i),
                ("min_bits", c_p)]


class RecordDesc(ctypes.Structure):
    _fields_ = [("obs", c_p), ("nxt", c_p), ("act", c_p), ("rew", c_p), ("gam", c_p), ("gen", c_p),
                ("C", c_i), ("cap", c_i64), ("nframes", c_i64)]


class HeadParams(ctypes.Structure):
    _fields_ = [("wv", c_p), ("bv", c_p), ("wa", c_p), ("ba", c_p)]


class HeadLo(ctypes.Structure):
    """Split-mode lo planes of the head's activations / gradient (``HeadLo``, csrc/head_common.h)."""
    _fields_ = [("Hon", c_p), ("Htg", c_p), ("dH", c_p)]


class HeadPart(ctypes.Structure):
    """fc split-K partials consumed by the DDQN head (mirrors ``HeadPart``, csrc/head_common.h)."""
    _fields_ = [("part", c_p), ("zstride", c_i64), ("nz", c_i), ("bias_on", c_p), ("bias_tg", c_p),
                ("two_b", c_i), ("hon", c_p), ("hon_lo", c_p)]


class IsNorm(ctypes.Structure):
    """Batch-max IS normalisation output of the head kernel (``IsNorm``, csrc/ddqn_head.hip)."""
    _fields_ = [("wscale", c_p), ("out", c_p), ("valid_count", c_p)]


class CfFragOut(ctypes.Structure):
    """The optimizer's stores of the fused forward's online operands (``CfFragOut``,
    csrc/cf_pack.h); all-zero = off."""
    _fields_ = [("w1frag", c_p), ("c2f", c_p), ("w1_off", c_i64), ("w2_off", c_i64), ("C", c_i),
                ("in_scale", c_f), ("c3f", c_p), ("w3_off", c_i64)]


class RmsSegs(ctypes.Structure):
    """Ranges of the flat parameters one optimizer launch updates (``RmsSegs``,
    csrc/sumtree.hip; the sharded data-parallel update)."""
    _fields_ = [("nseg", c_i), ("blk0", c_i * 4), ("off", c_i64 * 3), ("len", c_i64 * 3)]


class C2dPack(ctypes.Structure):
    """conv2 weight-fragment pack job riding on another launch (``C2dPackJob``, csrc/conv2_wfrag.h)."""
    _fields_ = [("w", c_p), ("w_lo", c_p), ("out", c_p)]


class ConvDesc(ctypes.Structure):
    """Implicit-GEMM forward/dgrad problem (mirrors ``ConvDesc`` in csrc/conv_mfma.hip)."""
    _fields_ = [("x", c_p), ("frame_slots", c_p), ("w", c_p), ("bias", c_p), ("y", c_p), ("mask", c_p),
                ("N", c_i), ("H", c_i), ("W", c_i), ("Cin", c_i),
                ("OH", c_i), ("OW", c_i), ("Cout", c_i), ("KH", c_i),
                ("KW", c_i), ("stride", c_i), ("pad_h", c_i), ("pad_w", c_i),
                ("mode", c_i), ("relu", c_i), ("ldy", c_i), ("ncls", c_i),
                ("ostride_h", c_i), ("ostride_w", c_i), ("OHfull", c_i), ("OWfull", c_i),
                ("K", c_i), ("in_scale", c_f), ("w_cls_stride", c_i64),
                ("w2", c_p), ("bias2", c_p), ("m_switch", c_i),
                ("bt", c_i), ("ldb", c_i), ("koff", c_i * 16), ("tile_hint", c_i), ("order_hint", c_i),
                ("x_lo", c_p), ("w_lo", c_p), ("w2_lo", c_p), ("y_lo", c_p)]


class WgradDesc(ctypes.Structure):
    """Weight-gradient problem (mirrors ``WgradDesc`` in csrc/conv_mfma.hip)."""
    _fields_ = [("dy", c_p), ("x", c_p), ("frame_slots", c_p), ("slab", c_p), ("bias_slab", c_p),
                ("N", c_i), ("H", c_i), ("W", c_i), ("Cin", c_i),
                ("OH", c_i), ("OW", c_i), ("KH", c_i), ("KW", c_i),
                ("stride", c_i), ("pad_h", c_i), ("pad_w", c_i), ("mode", c_i),
                ("Co", c_i), ("Kc", c_i), ("ldd", c_i), ("ldx", c_i),
                ("rows_per_split", c_i), ("Mred", c_i), ("norm_part", c_p), ("norm_slot0", c_i), ("pad0", c_i),
                ("dy_lo", c_p), ("x_lo", c_p)]


class RedJob(ctypes.Structure):
    """One split-K finalisation job (mirrors ``RedJob`` in csrc/conv_mfma.hip)."""
    _fields_ = [("slab", c_p), ("bslab", c_p), ("out", c_p), ("bout", c_p), ("n", c_i64),
                ("nsplit", c_i), ("nb", c_i), ("s2dC", c_i), ("Kc", c_i), ("scale", c_f), ("blk0", c_i),
                ("cpb", c_i), ("jnorm", c_p)]


class FinalizeDesc(ctypes.Structure):
    """All split-K reductions of a step + squared-norm partials (``FinalizeDesc``)."""
    _fields_ = [("job", RedJob * 4), ("njobs", c_i), ("nrm_n", c_i), ("nrm_ptr", c_p), ("norm_part", c_p),
                ("norm_slot0", c_i), ("nblocks", c_i)]


class Conv1WgDesc(ctypes.Structure):
    """Image-resident conv1 weight gradient (mirrors ``Conv1WgDesc`` in csrc/conv1_wgrad.hip)."""
    _fields_ = [("ring", c_p), ("slots", c_p), ("dy", c_p), ("slab", c_p), ("bias_slab", c_p), ("zero16", c_p),
                ("N", c_i), ("C", c_i), ("dy_lo", c_p), ("wq", c_p)]


class Conv1S2DDesc(ctypes.Structure):
    """conv1 on the space-to-depth ring (mirrors ``Conv1S2DDesc`` in csrc/conv1_s2d.hip)."""
    _fields_ = [("ring", c_p), ("slots", c_p), ("w", c_p), ("w2", c_p), ("bias", c_p), ("bias2", c_p),
                ("y", c_p), ("zero16", c_p), ("scratch", c_p), ("N", c_i), ("C", c_i), ("m_switch", c_i),
                ("in_scale", c_f), ("probe", c_p), ("w32", c_p), ("w2_32", c_p), ("y_lo", c_p),
                ("c2f_src", c_p * 4), ("c2f_out", c_p), ("c2f_bf16", c_i)]


_SIGS = {
    "apex_abi_version": ([], c_i),
    "apex_build_id": ([], ctypes.c_char_p),
    "apex_fill16": ([c_p, c_i64, c_i, c_p], c_i),
    "apex_tree_update": ([TreeDesc, c_p, c_p, c_i, c_i, c_f, c_f, c_p, c_p, c_i, c_p, c_p], c_i),
    "apex_tree_zero_range": ([TreeDesc, c_i64, c_i64, c_p], c_i),
    "apex_replay_insert": ([TreeDesc, RecordDesc, c_i64, c_i, c_p, c_p, c_p, c_p, c_p, c_p, c_f, c_f, c_p],
                           c_i),
    "apex_tree_sample": ([TreeDesc, RecordDesc, c_i, c_u64, c_p, c_f, c_p, c_p, c_p, c_p, c_p, c_p, c_p,
                          c_p, c_p, c_p, c_i, c_i, c_u64, c_p, c_i64, c_p], c_i),
    "apex_tree_rebuild": ([TreeDesc, c_p], c_i),
    "apex_gather_frames": ([c_p, c_p, c_i, c_i64, c_i64, c_p, c_p], c_i),
    "apex_debug_bounds_enabled": ([], c_i),
    "apex_debug_errors": ([c_p, c_p, c_i], c_i),
    "apex_grad_sqnorm_partials": ([c_p, c_i64, c_p, c_p], c_i),
    "apex_rmsprop_step": ([c_p, c_p, c_p, c_p, c_p, c_i64, c_p, c_f, c_f, c_f, c_f, c_i, c_p, c_p, c_p, c_i, c_i,
                           c_p], c_i),
    "apex_cast_bf16": ([c_p, c_p, c_i64, c_p, c_p], c_i),
    "apex_spin_hold": ([c_i, c_i, c_i, c_p, c_p], c_i),
    "apex_rmsprop_step_np": ([c_p, c_p, c_p, c_p, c_p, c_i64, c_p, c_i, c_f, c_f, c_f, c_f, c_i, c_p, c_p, c_p,
                              c_i, c_i, c_p], c_i),
    "apex_grad_finalize": ([FinalizeDesc, c_p], c_i),
    "apex_norm_total": ([c_p, c_i, c_p, c_p], c_i),
    "apex_ddqn_head": ([c_p, c_p, HeadParams, HeadParams, c_p, c_p, c_p, c_p, c_i, c_i, c_i, c_f, c_f, c_p,
                        c_p, c_p, c_p, c_p, c_p, c_i, c_i, HeadLo, HeadPart, C2dPack, IsNorm, c_p], c_i),
    "apex_rmsprop_sample": ([c_p, c_p, c_p, c_p, c_p, c_i64, c_p, c_i, c_f, c_f, c_f, c_f, c_i, c_p,
                             TreeDesc, RecordDesc, c_i, c_u64, c_p, c_f, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p,
                             c_p, c_p, c_i, c_i, c_u64, c_p, c_i64, c_p, c_p, c_i, c_i, CfFragOut, c_p, c_p, c_i64,
                             c_p], c_i),
    "apex_head_wgrad_prio": ([c_p, c_p, c_i, c_i, c_p, c_p, c_p, c_p, c_i, TreeDesc, c_p, c_p, c_p, c_p, c_f, c_f,
                              c_p, c_p, c_p, c_p, c_p, c_p, c_i, c_i, c_p, c_i64, c_p], c_i),
    "apex_fc_wgrad_head_prio": ([WgradDesc, c_p, c_p, c_i, c_i, c_p, c_p, c_p, c_p, c_i, TreeDesc, c_p, c_p, c_p,
                                 c_p, c_f, c_f, c_p, c_p, c_p, c_p], c_i),
    "apex_head_wgrad": ([c_p, c_p, c_i, c_i, c_p, c_p, c_p, c_p, c_i, c_p, c_p], c_i),
    "apex_actor_head": ([c_p, HeadParams, c_i, c_i, c_p, c_u64, c_p, c_p, c_p, c_i, c_p, c_p], c_i),
    "apex_conv1_s2d_fwd": ([Conv1S2DDesc, c_i, c_p], c_i),
    "apex_conv1_wgrad_img": ([Conv1WgDesc, c_i, c_p], c_i),
    "apex_slab_reduce": ([c_p, c_i, c_i64, c_f, c_p, c_p, c_i, c_p, c_i, c_i, c_p], c_i),
    "apex_s2d_pack_w1": ([c_p, c_p, c_i, c_p], c_i),
    "apex_s2d_unpack_w1_grad": ([c_p, c_p, c_i, c_p], c_i),
    "apex_s2d_frames": ([c_p, c_p, c_i64, c_i64, c_i64, c_p], c_i),
    "apex_pack_rows": ([c_p, c_p, c_p, c_i, c_i, c_p, c_i64, c_p], c_i),
    "apex_sqnorm_ranges": ([c_p, c_i64, c_p, c_i64, c_p, c_i, c_p], c_i),
    "apex_copy_segments": ([c_i, c_p, c_p, c_p, c_p], c_i),
}

_LIB: Optional[ctypes.CDLL] = None
_LOAD_ERROR: Optional[str] = None


def _declare(lib: ctypes.CDLL) -> None:
    for name, (args, res) in _SIGS.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.argtypes = args
        fn.restype = res
    # optional families declared by their own modules (conv / gemm)
    from . import conv_sigs
    conv_sigs.declare(lib)


ABI_VERSION = 8      # csrc/sumtree.hip apex_abi_version(): the launchers' argument lists


def load(build_if_missing: bool = True) -> Optional[ctypes.CDLL]:
    """Load the kernel library, after checking the build id compiled into it against
    the tree (ops/build.py: sources, headers, flags, compiler): a stale library is
    rebuilt first (``build_if_missing``) or refused -- never run."""
    global _LIB, _LOAD_ERROR
    if _LIB is not None:
        return _LIB
    debug = debug_bounds_requested()
    try:
        path = _build.ensure_current("kernels_debug" if debug else "kernels", allow_build=build_if_missing)
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
        _declare(lib)
        if lib.apex_abi_version() != ABI_VERSION:
            raise RuntimeError(f"{path}: ABI {lib.apex_abi_version()} != {ABI_VERSION}")
        _LIB = lib
    except Exception as e:  # pragma: no cover - depends on toolchain
        _LOAD_ERROR = repr(e)
        _LIB = None
    return _LIB


def debug_bounds_requested() -> bool:
    """``APEX_DEBUG_BOUNDS=1`` selects the bounds-checking kernel library
    (``libapex_kernels_debug.so``, built with ``-DAPEX_DEBUG_BOUNDS``)."""
    return os.environ.get("APEX_DEBUG_BOUNDS", "0") not in ("", "0")


DEBUG_SITES = ("tree_update.leaf", "replay_insert.slot", "tree_sample.slot", "gather_frames.frame",
               "replay_insert.frame_value", "tree_zero_range.slot", "unused6", "unused7")


def debug_errors(reset: bool = True) -> dict:
    """Per-site bounds-violation counts of the debug library (synchronises the
    device).  ``{site: (count, first_bad_index)}`` for sites with violations;
    always empty for the release library."""
    lib = require_kernels()
    counts = (ctypes.c_int * 8)()
    first = (ctypes.c_longlong * 8)()
    check(lib.apex_debug_errors(ctypes.addressof(counts), ctypes.addressof(first), int(reset)), "debug_errors")
    return {DEBUG_SITES[i]: (int(counts[i]), int(first[i])) for i in range(8) if counts[i]}


def available() -> bool:
    return load() is not None


def require_kernels() -> ctypes.CDLL:
    lib = load()
    if lib is None:
        raise RuntimeError(f"apex HIP kernel library unavailable: {_LOAD_ERROR}. "
                           f"Run `python -m apex_dqn_amd.ops.build`.")
    return lib


def stream_ptr(device: Optional[torch.device] = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def head_lo(Hon_lo=None, Htg_lo=None, dH_lo=None) -> HeadLo:
    """Split-mode lo planes for the head kernels (all None in bf16 mode)."""
    lo = HeadLo()
    lo.Hon, lo.Htg, lo.dH = ptr(Hon_lo), ptr(Htg_lo), ptr(dH_lo)
    return lo


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with hipError {rc}")
