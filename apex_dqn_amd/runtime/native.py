"""ctypes bindings for the native host runtime (csrc/runtime/host_runtime.cpp).

The library is built in-tree by ``apex_dqn_amd.ops.build`` (g++, no GPU
needed).  Every class here keeps the exact interface and storage of its numpy
counterpart, so the numpy versions stay as the test oracles and as a fallback
when the library cannot be built (``available()`` is False).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

from ..envs.vector_envs import CartPoleVec
from ..replay.sumtree import SumTree

_LIB: Optional[ctypes.CDLL] = None
_TRIED = False

c_i, c_i64, c_p, c_d = ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_double

_SIGS = {
    "apex_rt_version": ([], c_i),
    "apex_rt_st_update": ([c_p, c_p, c_i64, c_i64, c_p, c_p, c_i64], c_i),
    "apex_rt_st_find": ([c_p, c_i64, c_i64, c_p, c_i64, c_p], c_i),
    "apex_rt_st_sample_stratified": ([c_p, c_i64, c_i64, c_i64, c_p, c_p], c_i),
    "apex_rt_cp_reset": ([c_p, c_p, c_p, c_p, c_i, c_p, c_p], None),
    "apex_rt_cp_step": ([c_p, c_p, c_p, c_p, c_i, c_p, c_p, c_p, c_p, c_p, c_p, c_p], None),
    "apex_rt_seqlock_write": ([c_p, c_p, c_p, c_i64], c_i64),
    "apex_rt_seqlock_read": ([c_p, c_p, c_p, c_i64, c_i64, c_i], c_i64),
    "apex_rt_ns_create": ([c_i, c_i, c_d, c_i, c_i64], c_p),
    "apex_rt_ns_destroy": ([c_p], None),
    "apex_rt_ns_step": ([c_p, c_p, c_p, c_i, c_p, c_p, c_p, c_p], c_i),
    "apex_rt_ns_size": ([c_p], c_i64),
    "apex_rt_ns_take": ([c_p, c_i64, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p], c_i64),
}


def lib() -> Optional[ctypes.CDLL]:
    """Load (building if needed) libapex_runtime.so; None if unavailable."""
    global _LIB, _TRIED
    if _LIB is not None or _TRIED:
        return _LIB
    _TRIED = True
    if os.environ.get("APEX_DISABLE_NATIVE_RUNTIME") == "1":
        return None
    try:
        from ..ops import build
        # content-addressed: a library whose build id does not match the sources is rebuilt
        path = build.ensure_current("runtime")
        L = ctypes.CDLL(path)
        for name, (args, res) in _SIGS.items():
            f = getattr(L, name)
            f.argtypes, f.restype = args, res
        _LIB = L
    except Exception:  # pragma: no cover - toolchain missing
        _LIB = None
    return _LIB


def available() -> bool:
    return lib() is not None


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


class NativeSumTree(SumTree):
    """``SumTree`` whose update / prefix search run in C++ on the same arrays."""

    def update(self, idx, values) -> None:
        idx = np.ascontiguousarray(np.asarray(idx, np.int64).ravel())
        values = np.ascontiguousarray(np.asarray(values, np.float64).ravel())
        if idx.size == 0:
            return
        if lib().apex_rt_st_update(_ptr(self.sum), _ptr(self.min), self.size2, self.capacity, _ptr(idx),
                                   _ptr(values), idx.size) != 0:
            raise IndexError("sum-tree index out of range")

    def find_prefix(self, u) -> np.ndarray:
        u = np.ascontiguousarray(np.asarray(u, np.float64).ravel())
        out = np.empty(u.size, np.int64)
        lib().apex_rt_st_find(_ptr(self.sum), self.size2, self.capacity, _ptr(u), u.size, _ptr(out))
        return out

    def sample_stratified(self, batch: int, rng: np.random.Generator) -> np.ndarray:
        r = rng.random(batch)
        out = np.empty(batch, np.int64)
        if lib().apex_rt_st_sample_stratified(_ptr(self.sum), self.size2, self.capacity, batch, _ptr(r),
                                              _ptr(out)) != 0:
            raise RuntimeError("cannot sample from an empty sum-tree")
        return out


def make_sum_tree(capacity: int) -> SumTree:
    return NativeSumTree(capacity) if available() else SumTree(capacity)


class NativeCartPoleVec(CartPoleVec):
    """``CartPoleVec`` stepped in C++ (same dynamics; resets draw from a
    per-env splitmix stream seeded from ``seed``)."""

    def __init__(self, num_envs: int, seed: int = 0):
        super().__init__(num_envs, seed)
        self.rng_state = np.array([(seed * 1_000_003 + i) * 0x9E3779B97F4A7C15 % (1 << 64)
                                   for i in range(self.E)], np.uint64)
        self._obs = np.zeros((self.E, 4), np.float32)
        self._rew = np.zeros(self.E, np.float32)
        self._done = np.zeros(self.E, np.uint8)
        self._trunc = np.zeros(self.E, np.uint8)
        self._iret = np.zeros(self.E, np.float64)
        self._ilen = np.zeros(self.E, np.int64)

    def reset(self) -> np.ndarray:
        self.state = np.ascontiguousarray(self.state)
        lib().apex_rt_cp_reset(_ptr(self.state), _ptr(self.t), _ptr(self.ep_ret), _ptr(self.rng_state), self.E,
                               None, _ptr(self._obs))
        return self._obs.copy()

    def step(self, actions: np.ndarray):
        a = np.ascontiguousarray(np.asarray(actions, np.int64).ravel())
        lib().apex_rt_cp_step(_ptr(self.state), _ptr(self.t), _ptr(self.ep_ret), _ptr(self.rng_state), self.E,
                              _ptr(a), _ptr(self._obs), _ptr(self._rew), _ptr(self._done), _ptr(self._trunc),
                              _ptr(self._iret), _ptr(self._ilen))
        done = self._done.astype(bool)
        info = {"episode_return": self._iret.copy(), "episode_length": self._ilen.copy(),
                "truncated": self._trunc.astype(bool)}
        return self._obs.copy(), self._rew.copy(), done, info


class NativeNStepBuilder:
    """``actors.nstep.NStepBuilder`` in C++ (csrc/runtime/nstep.cpp): same
    semantics, emission order and ``get`` batches; observations are opaque
    fixed-shape payloads of ``obs_dtype``."""

    def __init__(self, num_envs: int, n: int, gamma: float, obs_shape, obs_dtype, env_id_offset: int = 0):
        self.E, self.n, self.gamma = int(num_envs), int(n), float(gamma)
        self.obs_shape = tuple(obs_shape)
        self.obs_dtype = np.dtype(obs_dtype)
        self._ob = int(np.prod(self.obs_shape)) * self.obs_dtype.itemsize
        self.env_ids = np.arange(self.E, dtype=np.int64) + int(env_id_offset)
        self._lib = lib()
        self._h = self._lib.apex_rt_ns_create(self.E, self.n, self.gamma, self._ob, int(env_id_offset))
        if not self._h:
            raise ValueError("invalid n-step builder shape")

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h and self._lib is not None:
            self._lib.apex_rt_ns_destroy(h)

    def step(self, obs, q, actions, rewards, dones, next_obs) -> None:
        obs = np.ascontiguousarray(obs, self.obs_dtype)
        nxt = np.ascontiguousarray(next_obs, self.obs_dtype)
        q = np.ascontiguousarray(q, np.float32)
        a = np.ascontiguousarray(actions, np.int64)
        r = np.ascontiguousarray(rewards, np.float32)
        d = np.ascontiguousarray(dones, np.uint8)
        if self._lib.apex_rt_ns_step(self._h, _ptr(obs), _ptr(q), q.shape[1], _ptr(a), _ptr(r), _ptr(d),
                                     _ptr(nxt)) != 0:
            raise IndexError("action out of range")

    @property
    def size(self) -> int:
        return int(self._lib.apex_rt_ns_size(self._h))

    def get(self, max_items: Optional[int] = None):
        k = self.size if max_items is None else min(self.size, int(max_items))
        if self.size == 0:
            return None
        out = dict(S_t=np.empty((k,) + self.obs_shape, self.obs_dtype),
                   S_tpn=np.empty((k,) + self.obs_shape, self.obs_dtype),
                   A_t=np.empty(k, np.int64), R=np.empty(k, np.float32), Gamma=np.empty(k, np.float32),
                   priority=np.empty(k, np.float32), key=np.empty(k, np.int64), env=np.empty(k, np.int64))
        got = self._lib.apex_rt_ns_take(self._h, k, _ptr(out["S_t"]), _ptr(out["S_tpn"]), _ptr(out["A_t"]),
                                        _ptr(out["R"]), _ptr(out["Gamma"]), _ptr(out["priority"]),
                                        _ptr(out["key"]), _ptr(out["env"]))
        assert got == k
        return out


class SeqLock:
    """Seqlock over two shared-memory torch tensors (sequence word + payload)."""

    def __init__(self, seq_tensor, payload_tensor):
        self.seq, self.payload = seq_tensor, payload_tensor

    def write(self, src) -> int:
        src = src.contiguous()
        return int(lib().apex_rt_seqlock_write(self.seq.data_ptr(), self.payload.data_ptr(), src.data_ptr(),
                                               src.numel() * src.element_size()))

    def read_into(self, dst, last: int, tries: int = 1000) -> int:
        """Copy a consistent snapshot into ``dst``: returns its (even) version,
        -2 when the version still equals ``last``, -1 when no stable read
        happened within ``tries``."""
        return int(lib().apex_rt_seqlock_read(self.seq.data_ptr(), dst.data_ptr(), self.payload.data_ptr(),
                                              dst.numel() * dst.element_size(), int(last), int(tries)))
