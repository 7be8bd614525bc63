"""Bounds-checking debug build of the replay kernels.

``libapex_kernels_debug.so`` (``-DAPEX_DEBUG_BOUNDS``, selected at load time by
``APEX_DEBUG_BOUNDS=1``) checks every leaf / ring-slot / frame index the replay
kernels dereference.  A violation is counted per site, the first bad index is
kept, and the access is clamped or dropped -- the kernel never faults.  The GPU
test feeds deliberately corrupt indices and reads the report back."""
import ctypes
import os
import subprocess

import numpy as np
import pytest
import torch

from apex_dqn_amd.ops import build as _build


def test_debug_library_builds_with_checks():
    path = _build.build_kernels(debug=True)
    assert path.endswith("libapex_kernels_debug.so") and os.path.exists(path)
    syms = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True).stdout
    assert "apex_debug_errors" in syms and "apex_debug_bounds_enabled" in syms


def test_debug_env_selects_library(monkeypatch):
    from apex_dqn_amd.ops import _lib as L
    monkeypatch.setenv("APEX_DEBUG_BOUNDS", "1")
    assert L.debug_bounds_requested()
    monkeypatch.setenv("APEX_DEBUG_BOUNDS", "0")
    assert not L.debug_bounds_requested()


@pytest.mark.gpu
def test_debug_bounds_report_instead_of_fault(monkeypatch):
    from apex_dqn_amd.ops import _lib as L
    from apex_dqn_amd.replay.gpu_replay import GpuReplayShard
    dev = torch.device("cuda", 0)
    saved = L._LIB
    try:
        L._LIB = None
        monkeypatch.setenv("APEX_DEBUG_BOUNDS", "1")
        lib = L.require_kernels()
        assert lib.apex_debug_bounds_enabled() == 1
        L.debug_errors(reset=True)
        rp = GpuReplayShard(256, 256, 512, 4, device=dev)
        assert rp.lib is lib
        rng = np.random.default_rng(0)
        seqs = rp.append_frames(rng.integers(0, 255, (72, 84, 84), dtype=np.uint8))
        K = 64
        st = np.stack([seqs[i:i + 4] for i in range(K)])
        rp.insert(dict(S_t=st, S_tpn=st + 3, A_t=np.zeros(K, np.int64), R=np.zeros(K, np.float32),
                       Gamma=np.full(K, 0.9, np.float32), priority=np.ones(K, np.float32)))
        assert L.debug_errors() == {}, "valid inserts must not trip the checks"

        # frame gather with a slot past the frame ring: clamped, reported
        slots = torch.zeros(2, 4, dtype=torch.int32, device=dev)
        slots[1, 2] = rp.F + 7
        rp.gather_frames(slots)
        # priority write-back to a leaf past the tree: dropped, reported
        rp.update_priorities(torch.tensor([3, rp.cap + 5], device=dev), torch.ones(2, device=dev), None)
        # raw insert of a record whose frame-slot value is outside the ring
        bad = torch.full((1, 4), -3, dtype=torch.int32, device=dev)
        one_i = torch.zeros(1, dtype=torch.int32, device=dev)
        one_f = torch.ones(1, dtype=torch.float32, device=dev)
        L.check(lib.apex_replay_insert(rp.tree_desc(), rp.record_desc(), 100, 1, bad.data_ptr(), bad.data_ptr(),
                                       one_i.data_ptr(), one_f.data_ptr(), one_f.data_ptr(), one_f.data_ptr(),
                                       rp.alpha, rp.eps, torch.cuda.current_stream(dev).cuda_stream), "insert")
        err = L.debug_errors(reset=True)
        assert err["gather_frames.frame"] == (1, rp.F + 7)
        assert err["tree_update.leaf"] == (1, rp.cap + 5)
        assert err["replay_insert.frame_value"][1] == -3
        assert L.debug_errors() == {}
        torch.cuda.synchronize()
    finally:
        L._LIB = saved
