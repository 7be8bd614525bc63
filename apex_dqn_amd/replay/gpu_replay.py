"""HBM-resident prioritized replay shard (one per GPU rank).

Storage per shard (sized for 288 GB HBM3E):
* frame ring  uint8 [F, 84, 84]      -- each env frame stored once, in space-to-depth(4)
                                       byte order (21x21 blocks of 4x4 pixels, 16 B each) so
                                       conv1 reads whole 16-B blocks by LDS-DMA;
* records     int32 [cap, C] x2      -- frame-ring slots of S_t / S_{t+n} stacks,
              int32 act, fp32 R, fp32 Gamma, int32 generation;
* sum-tree    64-ary (leaf fp32 = p^alpha, internal fp64) -- ``csrc/sumtree.hip``.

Reference parity (``replay.py``): ``add`` -> :meth:`insert`, ``sample`` ->
:meth:`sample`, ``set_priorities`` -> :meth:`update_priorities`,
``remove_to_fit`` -> :meth:`remove_to_fit`, ``size`` -> :meth:`size`.

All mutating kernels run on the caller's current stream (single writer per
shard; SURVEY §5.2 race A24 is designed out).  Slot generations make a
priority write-back for a slot that was overwritten after it was sampled a
no-op; writes to evicted slots never resurrect them.

Data parallelism (:meth:`enable_sharding`): the W shards are ONE prioritized
replay.  Each step the shards all-gather their (sum p^alpha, min p^alpha) and run
one global stratified draw -- identical on every rank -- over the concatenated
mass intervals; rank r keeps the draws that land in its interval.  An item's
sampling probability is p_i / sum over ALL shards, exactly as in the reference's
single ``ReplayMemory.sample`` (``replay.py:44-57``), the per-rank batch varies
with the shard's share of the mass (fixed B-row buffers, unused rows carry IS
weight 0), and IS weights are normalised by the global minimum priority.  Each
shard holds ``ceil(soft_capacity / W)`` transitions, so the global FIFO bound is
the reference's ``soft_capacity`` (``replay.py:71-80``).

On CPU (tests) the same class runs a torch implementation with identical
semantics (exact recompute instead of fp64 deltas; the same counter-based
uniforms as the kernel, so the global draw is bit-identical).
"""
from __future__ import annotations

import math
import threading
from typing import Dict, Optional

import numpy as np
import torch

from ..ops import _lib


def to_s2d(x: torch.Tensor) -> torch.Tensor:
    """(n, 84, 84) frames -> space-to-depth(4) byte layout [21][21][4][4], viewed as (n, 84, 84)."""
    n = x.shape[0]
    return x.reshape(n, 21, 4, 21, 4).permute(0, 1, 3, 2, 4).contiguous().reshape(n, 84, 84)


def from_s2d(y: torch.Tensor) -> torch.Tensor:
    """Inverse of :func:`to_s2d` (the axis permutation is an involution)."""
    n = y.shape[0]
    return y.reshape(n, 21, 21, 4, 4).permute(0, 1, 3, 2, 4).contiguous().reshape(n, 84, 84)


_MASK64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix64(z: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser (csrc/apex_common.h ``apex_mix64``), wrapping uint64 math."""
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def apex_uniform(seed: int, ctr: int, idx) -> np.ndarray:
    """The kernels' counter-based uniform in [0, 1) (``apex_uniform``), float32."""
    i = np.asarray(idx, dtype=np.uint64)
    with np.errstate(over="ignore"):
        inner = _mix64(np.uint64(ctr & 0xFFFFFFFFFFFFFFFF) * np.uint64(0x100000001B3) + i)
    r = _mix64(np.uint64(seed & 0xFFFFFFFFFFFFFFFF) ^ inner)
    return (r >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)


# per-shard statistics all-gathered every DP step (csrc/sumtree.hip SHARD_STATS):
# (sum p^alpha, min p^alpha, max IS weight of the shard's rows in the current batch)
SHARD_STATS = 3


def global_draw(stats: np.ndarray, rank: int, B: int, seed: int, ctr: int, mcap: Optional[int] = None):
    """The sharded sampler's global stratified draw as seen by ``rank`` (mirror of
    csrc/sumtree.hip ``tree_sample_body``): returns (u_local (B,) float64, valid (B,)
    bool, wscale, pmin_global) for the all-gathered ``stats`` [W, >=2] = (total, min p, ...).
    ``mcap`` caps the global batch M (default W B)."""
    W = stats.shape[0]
    mcap = W * B if not mcap or mcap <= 0 else int(mcap)
    sm = c0 = tmax = 0.0
    pm = math.inf
    for q in range(W):
        tq = float(stats[q, 0])
        if q < rank:
            c0 += tq
        sm += tq
        tmax = max(tmax, tq)
        mq = float(np.float32(stats[q, 1]))
        if tq > 0.0 and mq > 0.0:
            pm = min(pm, mq)
    tr = float(stats[rank, 0])
    c1 = c0 + tr
    if tmax > 0.0:
        mb = B if W == 1 else math.floor((B - 2) * sm / tmax)
        M = int(min(mcap, max(mb, 0)))
    else:
        M = 0
    u = np.zeros(B, np.float64)
    valid = np.zeros(B, bool)
    wscale = 1.0
    if M > 0 and tr > 0.0:
        delta = sm / M
        j0 = int(math.floor(c0 / delta))
        if (j0 + float(apex_uniform(seed, ctr, j0))) * delta < c0:
            j0 += 1
        j = j0 + np.arange(B, dtype=np.int64)
        uj = (j.astype(np.float64) + apex_uniform(seed, ctr, j).astype(np.float64)) * delta
        valid = (j < M) & ((uj < c1) | (rank == W - 1))
        u = np.where(valid, uj - c0, 0.0)
        wscale = float(np.float32(W * B / M))
    return u, valid, wscale, pm


def _tree_levels(cap: int):
    sizes = [cap]
    while sizes[-1] > 1:
        sizes.append((sizes[-1] + 63) // 64)
    return sizes  # sizes[0] = leaves, sizes[-1] = 1 (root)


class GpuReplayShard:
    def __init__(self, capacity: int, soft_capacity: int, frame_capacity: int, stack: int,
                 frame_shape=(84, 84), alpha: float = 0.6, beta: float = 0.4, eps: float = 1e-6,
                 device: torch.device = torch.device("cuda"), seed: int = 0, use_hip: Optional[bool] = None):
        self.device = torch.device(device)
        self.cap = int(capacity)
        self.soft_capacity = int(min(soft_capacity, capacity))
        self.F = int(frame_capacity)
        self.C = int(stack)
        self.frame_shape = tuple(frame_shape)
        self.frame_bytes = int(np.prod(frame_shape))
        self.alpha, self.beta, self.eps = float(alpha), float(beta), float(eps)
        self.seed = int(seed)
        on_gpu = self.device.type == "cuda"
        self.use_hip = on_gpu if use_hip is None else bool(use_hip)
        if self.use_hip:
            self.lib = _lib.require_kernels()
        d = self.device
        self.sizes = _tree_levels(self.cap)
        self.L = len(self.sizes) - 1
        if self.L > 7:
            raise ValueError("capacity too large for an 8-level 64-ary tree")
        self.leaf = torch.zeros(self.cap, dtype=torch.float32, device=d)
        n_int = sum(self.sizes[1:])
        self.nodes = torch.zeros(max(n_int, 1), dtype=torch.float64, device=d)
        self.offs = [0] * 8
        o = 0
        for k in range(1, self.L + 1):
            self.offs[k] = o
            o += self.sizes[k]
        self.min_bits = torch.full((1,), 0x7f800000, dtype=torch.int32, device=d)
        self.frames = torch.zeros((self.F,) + self.frame_shape, dtype=torch.uint8, device=d)
        self.obs = torch.zeros(self.cap, self.C, dtype=torch.int32, device=d)
        self.nxt = torch.zeros(self.cap, self.C, dtype=torch.int32, device=d)
        self.act = torch.zeros(self.cap, dtype=torch.int32, device=d)
        self.rew = torch.zeros(self.cap, dtype=torch.float32, device=d)
        self.gam = torch.zeros(self.cap, dtype=torch.float32, device=d)
        self.gen = torch.zeros(self.cap, dtype=torch.int32, device=d)
        self.ctr = torch.zeros(1, dtype=torch.int64, device=d)  # sampling RNG counter (device-side)
        self.zero16 = torch.zeros(64, dtype=torch.uint8, device=d)  # DMA source for padding rows
        # host bookkeeping
        self.head = 0          # next record slot
        self.live = 0
        self.frame_head = 0    # next frame sequence number
        self.total_inserted = 0
        # bumped by host-side mutations that can invalidate a batch drawn ahead of time
        # (eviction, rebuild): a learner that samples its next batch inside the previous
        # step resamples when this changed in between.  Inserts and frame appends do
        # not: the early draw is then a proportional sample of the replay as of the end
        # of the previous update (Ape-X's learner consumes prefetched batches the same
        # way), its records are gathered copies, and a slot re-used before the priority
        # write-back is caught by the generation check.
        self.version = 0
        self.min_frame_seq = np.full(self.cap, -1, np.int64)  # oldest frame referenced per slot
        # host-state lock: an actor thread appends / inserts while the learner thread
        # evicts (runtime/actor_thread.py); the kernels each section enqueues land on the
        # stream in the order the sections run
        self.lock = threading.RLock()
        self._pin_ev = None                 # pinned frame staging (append_frames)
        self._tdesc = None
        self._rdesc = None
        # sharding (enable_sharding): all-gathered (total, min p) of every shard, fp64
        self.shard_rank, self.shard_world, self.shard_seed, self.shard_group = 0, 1, 0, None
        self.shard_mcap = 0     # cap on a draw's global batch M (0: W x the per-rank batch)
        self.local_stats = None
        self.shard_stats = None

    # -------------------------------------------------------------- sharding
    def enable_sharding(self, rank: int, world: int, shard_seed: int, group=None, mcap: int = 0) -> None:
        """Make this shard part of ONE global prioritized replay over ``world`` ranks
        (see the module docstring).  ``shard_seed`` must be equal on every rank;
        the sampling counter ``ctr`` advances in lock-step with the DP updates.
        ``mcap``: the global batch of a draw is M = min(mcap, floor((B - 2) sum / max_r
        T_r)) strata (B = the per-rank row buffer); 0 = W B (per-rank batches).  With
        ``Runtime.batch_scope = "global"`` mcap is ``replay_sample_size`` and B holds
        ceil(mcap / W) rows plus slack, so M = mcap unless one shard carries more than
        (B - 2) / mcap of the total mass (then M shrinks, identically on every rank)."""
        d = self.device
        self.shard_rank, self.shard_world = int(rank), int(world)
        self.shard_seed, self.shard_group = int(shard_seed), group
        self.shard_mcap = int(mcap)
        self.shard_stats = torch.zeros(SHARD_STATS * self.shard_world, dtype=torch.float64, device=d)
        # this shard's slot of the gathered statistics (the all-gather runs in place)
        r = self.shard_rank
        self.local_stats = self.shard_stats[SHARD_STATS * r:SHARD_STATS * (r + 1)]

    @property
    def sharded(self) -> bool:
        return self.shard_stats is not None

    def gather_shard_stats(self, async_op: bool = False, coll=None, fresh_local: bool = False):
        """All-gather every shard's (sum p^alpha, min p^alpha, batch IS max) into ``shard_stats``
        (a collective; device-side, HIP-graph capturable over RCCL; in place: ``local_stats``
        is this shard's slot).  Call it after the last tree mutation that the next draw
        must see (the third field is written by the learner's head kernel:
        ``local_stats[2]``).  ``fresh_local``: the first two fields are already current
        (written by the priority write-back kernel, csrc/sumtree.hip ``stats_out``).
        ``coll``: the learner's collectives (parallel/rccl.py; torch.distributed by
        default).  With ``async_op`` the returned handle's ``wait()`` orders the result."""
        from ..parallel.rccl import TorchCollectives
        if not fresh_local:
            root = self.offs[self.L]
            self.local_stats[0:1].copy_(self.nodes[root:root + 1])
            self.local_stats[1:2].copy_(self.min_bits.view(torch.float32))
        work = (coll or TorchCollectives(self.shard_group)).all_gather_into(self.shard_stats, self.local_stats)
        if async_op:
            return work
        work.wait()
        return None

    # ----------------------------------------------------------- descriptors
    def tree_desc(self) -> "_lib.TreeDesc":
        if self._tdesc is None:
            t = _lib.TreeDesc()
            t.leaf = self.leaf.data_ptr()
            t.nodes = self.nodes.data_ptr()
            for k in range(8):
                t.off[k] = self.offs[k]
                t.n[k] = self.sizes[k] if k < len(self.sizes) else 0
            t.L = self.L
            t.min_bits = self.min_bits.data_ptr()
            self._tdesc = t
        return self._tdesc

    def record_desc(self) -> "_lib.RecordDesc":
        if self._rdesc is None:
            r = _lib.RecordDesc()
            r.obs, r.nxt = self.obs.data_ptr(), self.nxt.data_ptr()
            r.act, r.rew, r.gam, r.gen = (self.act.data_ptr(), self.rew.data_ptr(), self.gam.data_ptr(),
                                          self.gen.data_ptr())
            r.C, r.cap, r.nframes = self.C, self.cap, self.F
            self._rdesc = r
        return self._rdesc

    def _stream(self):
        return _lib.stream_ptr(self.device)

    # --------------------------------------------------------------- insert
    def append_frames(self, frames) -> np.ndarray:
        """Store new frames (n, H, W) uint8; returns their sequence numbers."""
        with self.lock:
            return self._append_frames_locked(frames)

    def insert(self, batch: Dict[str, np.ndarray]) -> np.ndarray:
        """Insert n-step transitions whose S_t/S_tpn payloads are frame seqs (K, C)."""
        with self.lock:
            return self._insert_locked(batch)

    def remove_to_fit(self) -> int:
        """FIFO eviction to soft_capacity + drop slots whose frames were overwritten."""
        with self.lock:
            return self._remove_to_fit_locked()

    def _append_frames_locked(self, frames) -> np.ndarray:
        """Store new frames (n, H, W) uint8; returns their sequence numbers."""
        if isinstance(frames, np.ndarray) and self.device.type == "cuda":
            frames = self._pinned(frames)      # async H2D from a pinned staging buffer
        frames = torch.as_tensor(frames)
        n = frames.shape[0]
        seqs = self.frame_head + np.arange(n, dtype=np.int64)
        skip = max(0, n - self.F)  # only the newest F frames survive a wrap
        src = frames[skip:].to(self.device, non_blocking=True).contiguous()
        if self._pin_ev is not None and frames.is_pinned():
            self._pin_ev[self._pin_k].record()
        start = (self.frame_head + skip) % self.F
        if self.use_hip and self.frame_shape == (84, 84):
            # s2d permutation + ring scatter (with wrap) in one kernel
            _lib.check(self.lib.apex_s2d_frames(src.data_ptr(), self.frames.data_ptr(), src.shape[0], self.F,
                                                start, self._stream()), "s2d_frames")
        else:
            src = to_s2d(src) if self.frame_shape == (84, 84) else src
            pos, k = start, 0
            while k < src.shape[0]:
                m = min(src.shape[0] - k, self.F - pos)
                self.frames[pos:pos + m].copy_(src[k:k + m], non_blocking=True)
                k += m
                pos = 0
        self.frame_head += n
        return seqs

    def _acquire_pin(self, shape) -> torch.Tensor:
        """The next of two pinned staging buffers of ``shape`` (the copy of its previous
        use must have finished: its event is waited on first).  Refuses while another
        thread's staged frames (stage_frames) wait for their append: rotating the
        buffers then would hand that thread's buffer out again and overwrite its frames."""
        st = getattr(self, "_staged", None)
        if st is not None and st[2] != threading.get_ident():
            raise RuntimeError("GpuReplayShard: frames staged by another thread are not appended yet "
                               "(stage_frames / append_frames must pair up on one thread)")
        shape = tuple(shape)
        if getattr(self, "_pin_shape", None) != shape:
            self._pin_buf = [torch.empty(shape, dtype=torch.uint8).pin_memory() for _ in range(2)]
            self._pin_ev = [torch.cuda.Event(), torch.cuda.Event()]
            self._pin_used = [False, False]
            self._pin_shape, self._pin_k = shape, 1
        self._pin_k ^= 1
        k = self._pin_k
        if self._pin_used[k]:
            self._pin_ev[k].synchronize()
        self._pin_used[k] = True
        return self._pin_buf[k]

    def stage_frames(self, n: int) -> Optional[np.ndarray]:
        """A pinned host buffer for the next append of ``n`` frames (GPU shards): an env
        that writes its frames straight into it (``step(actions, out=...)``) saves the
        staging copy -- append_frames of exactly that array starts its H2D copy from it.
        None off the GPU."""
        if self.device.type != "cuda" or self.frame_shape is None:
            return None
        with self.lock:
            buf = self._acquire_pin((int(n),) + tuple(self.frame_shape))
            arr = buf.numpy()
            # one staging slot per shard: the append of this array must come from the same
            # thread before anything else takes a pinned buffer (_acquire_pin checks)
            self._staged = (buf, arr, threading.get_ident())
            return arr

    def _pinned(self, frames: np.ndarray) -> torch.Tensor:
        """Host frames in a pinned staging buffer: the buffer itself when ``frames`` is the
        array stage_frames handed out, else a copy into the next one."""
        st = getattr(self, "_staged", None)
        if st is not None and frames is st[1]:
            self._staged = None
            return st[0]
        if st is not None and st[2] == threading.get_ident():
            self._staged = None       # this thread staged and then appended other frames: drop it
        buf = self._acquire_pin(frames.shape)
        np.copyto(buf.numpy(), frames)
        return buf

    def _insert_locked(self, batch: Dict[str, np.ndarray]) -> np.ndarray:
        """Insert n-step transitions whose S_t/S_tpn payloads are frame seqs (K, C)."""
        K = len(batch["A_t"])
        if K == 0:
            return np.zeros(0, np.int64)
        if K > self.cap:
            raise ValueError("insert batch larger than replay capacity")
        obs_seq = np.asarray(batch["S_t"], np.int64).reshape(K, self.C)
        nxt_seq = np.asarray(batch["S_tpn"], np.int64).reshape(K, self.C)
        slots = (self.head + np.arange(K)) % self.cap
        self.min_frame_seq[slots] = np.minimum(obs_seq.min(1), nxt_seq.min(1))
        d = self.device
        s_obs = torch.from_numpy((obs_seq % self.F).astype(np.int32)).to(d, non_blocking=True)
        s_nxt = torch.from_numpy((nxt_seq % self.F).astype(np.int32)).to(d, non_blocking=True)
        s_act = torch.from_numpy(np.asarray(batch["A_t"], np.int32)).to(d, non_blocking=True)
        s_rew = torch.from_numpy(np.asarray(batch["R"], np.float32)).to(d, non_blocking=True)
        s_gam = torch.from_numpy(np.asarray(batch["Gamma"], np.float32)).to(d, non_blocking=True)
        pr = batch.get("priority")
        if pr is None:
            pr = np.ones(K, np.float32)
        s_pr = torch.from_numpy(np.asarray(pr, np.float32)).to(d, non_blocking=True)
        if self.use_hip:
            _lib.check(self.lib.apex_replay_insert(self.tree_desc(), self.record_desc(), self.head, K,
                                                   s_obs.data_ptr(), s_nxt.data_ptr(), s_act.data_ptr(),
                                                   s_rew.data_ptr(), s_gam.data_ptr(), s_pr.data_ptr(),
                                                   self.alpha, self.eps, self._stream()), "replay_insert")
        else:
            ts = torch.from_numpy(slots).to(d)
            self.obs[ts] = s_obs
            self.nxt[ts] = s_nxt
            self.act[ts] = s_act
            self.rew[ts] = s_rew
            self.gam[ts] = s_gam
            self.gen[ts] += 1
            self._torch_set_leaves(ts, (s_pr.abs().double() + self.eps) ** self.alpha)
        self.head = int((self.head + K) % self.cap)
        self.live = min(self.live + K, self.cap)
        self.total_inserted += K
        return slots

    def size(self) -> int:
        return int(self.live)

    # ------------------------------------------------------------- sampling
    def sample(self, B: int, out: Optional[Dict[str, torch.Tensor]] = None,
               nxt2: Optional[torch.Tensor] = None) -> Dict[str, torch.Tensor]:
        """Stratified proportional sample of B slots; IS weights max-normalised
        (globally over the shards once :meth:`enable_sharding` ran: then rows whose
        global draw fell in another shard carry weight 0 and generation -1).

        ``out`` (preallocated tensors) makes the call graph-capturable; ``nxt2``
        receives a second copy of the S_{t+n} frame slots (target-network rows).
        """
        d = self.device
        if out is None:
            out = self.alloc_sample_buffers(B)
        if self.sharded and B < 3:
            raise ValueError("sharded sampling needs B >= 3")
        if self.use_hip:
            _lib.check(self.lib.apex_tree_sample(*self.sample_launch_args(B, out, nxt2), self._stream()),
                       "tree_sample")
            return out
        leaf = self.leaf.double().cpu()
        total = leaf.sum()
        ctr = int(self.ctr.item())
        valid = np.ones(B, bool)
        wscale = 1.0
        if self.sharded:
            st = self.shard_stats.double().cpu().numpy().reshape(self.shard_world, SHARD_STATS)
            u, valid, wscale, pmin = global_draw(st, self.shard_rank, B, self.shard_seed, ctr, self.shard_mcap)
            u = torch.from_numpy(u).clamp_(0.0, float(total))
        else:
            uu = torch.from_numpy(apex_uniform(self.seed, ctr, np.arange(B))).double()
            u = (torch.arange(B, dtype=torch.float64) + uu) * (total / B)
            pos = leaf[leaf > 0]
            pmin = float(np.float32(pos.min())) if pos.numel() else 0.0
        c = torch.cumsum(leaf, 0)
        idx = torch.searchsorted(c, u, right=True).clamp_(max=self.cap - 1)
        # never return an empty leaf (round-off at the top of the range)
        empty = leaf[idx] <= 0
        if empty.any():
            nz = torch.nonzero(leaf > 0).flatten()
            idx[empty] = nz[-1] if nz.numel() else 0
        p = leaf[idx].float()
        vt = torch.from_numpy(valid)
        w = torch.where(vt & (p > 0) & (pmin > 0), (p / max(pmin, 1e-38)).pow(-self.beta).clamp(max=1.0),
                        torch.zeros_like(p)) * wscale
        idx = idx.to(d)
        out["idx"].copy_(idx)
        out["weights"].copy_(w.float())
        out["gen"].copy_(torch.where(vt.to(d), self.gen[idx], torch.full_like(self.gen[idx], -1)))
        out["obs"].copy_(self.obs[idx])
        out["nxt"].copy_(self.nxt[idx])
        out["act"].copy_(self.act[idx])
        out["rew"].copy_(self.rew[idx])
        out["gam"].copy_(self.gam[idx])
        if "wscale" in out:
            out["wscale"].fill_(wscale)
        if nxt2 is not None:
            nxt2.copy_(out["nxt"])
        return out

    def sample_launch_args(self, B: int, out: Dict[str, torch.Tensor], nxt2: Optional[torch.Tensor] = None) -> tuple:
        """The tree_sample arguments (TreeDesc .. shard_seed) of :meth:`sample`, for
        kernels that draw the batch inside another launch (``apex_rmsprop_sample``)."""
        return (self.tree_desc(), self.record_desc(), B, self.seed, self.ctr.data_ptr(), self.beta,
                out["idx"].data_ptr(), out["weights"].data_ptr(), out["gen"].data_ptr(), out["obs"].data_ptr(),
                out["nxt"].data_ptr(), out["act"].data_ptr(), out["rew"].data_ptr(), out["gam"].data_ptr(),
                _lib.ptr(nxt2), _lib.ptr(self.shard_stats), self.shard_rank, self.shard_world, self.shard_seed,
                _lib.ptr(out.get("wscale")), int(self.shard_mcap))

    def alloc_sample_buffers(self, B: int) -> Dict[str, torch.Tensor]:
        d = self.device
        return dict(idx=torch.zeros(B, dtype=torch.int64, device=d),
                    weights=torch.zeros(B, dtype=torch.float32, device=d),
                    gen=torch.zeros(B, dtype=torch.int32, device=d),
                    obs=torch.zeros(B, self.C, dtype=torch.int32, device=d),
                    nxt=torch.zeros(B, self.C, dtype=torch.int32, device=d),
                    act=torch.zeros(B, dtype=torch.int32, device=d),
                    rew=torch.zeros(B, dtype=torch.float32, device=d),
                    gam=torch.zeros(B, dtype=torch.float32, device=d),
                    wscale=torch.ones(1, dtype=torch.float32, device=d))

    def gather_frames(self, slots: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """slots (B, C) int32 -> stacked frames (B, C, H, W) uint8 in natural pixel order."""
        B = slots.shape[0]
        raw = torch.empty((B, self.C) + self.frame_shape, dtype=torch.uint8, device=self.device)
        if self.use_hip:
            _lib.check(self.lib.apex_gather_frames(self.frames.data_ptr(), slots.data_ptr(), B * self.C, self.F,
                                                   self.frame_bytes, raw.data_ptr(), self._stream()),
                       "gather_frames")
        else:
            raw.copy_(self.frames[slots.long()])
        nat = from_s2d(raw.reshape(B * self.C, 84, 84)).reshape(raw.shape) if self.frame_shape == (84, 84) else raw
        if out is None:
            return nat
        out.copy_(nat)
        return out

    # ------------------------------------------------------------ priorities
    def update_priorities(self, idx: torch.Tensor, td_abs: torch.Tensor, gen: Optional[torch.Tensor] = None,
                          bump_ctr: bool = True) -> None:
        n = idx.numel()
        if self.use_hip:
            _lib.check(self.lib.apex_tree_update(self.tree_desc(), idx.data_ptr(), td_abs.data_ptr(), n, 1,
                                                 self.alpha, self.eps, _lib.ptr(gen), self.gen.data_ptr(), 1,
                                                 self.ctr.data_ptr() if bump_ctr else None, self._stream()),
                       "tree_update")
        else:
            idx_c = idx.long()
            # rows of a sharded draw that fell in another shard (generation -1) write
            # nothing and take no part in the dedupe
            valid = torch.ones(n, dtype=torch.bool, device=idx.device) if gen is None else gen >= 0
            keep = valid.clone()
            # last occurrence (among the valid rows) wins
            for i in range(n):
                if keep[i] and (valid[i + 1:] & (idx_c[i + 1:] == idx_c[i])).any():
                    keep[i] = False
            keep &= self.leaf[idx_c] > 0
            if gen is not None:
                keep &= self.gen[idx_c] == gen
            sel = idx_c[keep]
            vals = (td_abs[keep].abs().double() + self.eps) ** self.alpha
            self._torch_set_leaves(sel, vals)
            if bump_ctr:
                self.ctr += 1

    def _remove_to_fit_locked(self) -> int:
        """FIFO eviction to soft_capacity + drop slots whose frames were overwritten."""
        self.version += 1
        excess = self.live - self.soft_capacity
        n_ev = 0
        if excess > 0:
            oldest = (self.head - self.live) % self.cap
            self._zero_range(oldest, excess)
            self.live -= excess
            n_ev += excess
        # frame-ring guard: a live slot must not reference overwritten frames
        frame_tail = self.frame_head - self.F
        if frame_tail > 0 and self.live > 0:
            oldest = (self.head - self.live) % self.cap
            k = 0
            while k < self.live and self.min_frame_seq[(oldest + k) % self.cap] < frame_tail:
                k += 1
            if k:
                self._zero_range(oldest, k)
                self.live -= k
                n_ev += k
        return n_ev

    def rebuild(self) -> None:
        """Exact recompute of all internal nodes and the min (drift guard)."""
        self.version += 1
        if self.use_hip:
            _lib.check(self.lib.apex_tree_rebuild(self.tree_desc(), self._stream()), "tree_rebuild")
        else:
            self._torch_rebuild()

    # ------------------------------------------------------------ internals
    def _zero_range(self, start: int, count: int) -> None:
        if self.use_hip:
            _lib.check(self.lib.apex_tree_zero_range(self.tree_desc(), int(start), int(count), self._stream()),
                       "tree_zero_range")
        else:
            sl = torch.from_numpy((start + np.arange(count)) % self.cap).to(self.device)
            self._torch_set_leaves(sl, torch.zeros(count, dtype=torch.float64, device=self.device))

    def _torch_set_leaves(self, idx: torch.Tensor, vals: torch.Tensor) -> None:
        self.leaf[idx] = vals.float()
        self._torch_rebuild()

    def _torch_rebuild(self) -> None:
        prev = self.leaf.double()
        for k in range(1, self.L + 1):
            n = self.sizes[k]
            pad = torch.zeros(n * 64, dtype=torch.float64, device=self.device)
            pad[:prev.numel()] = prev
            lvl = pad.view(n, 64).sum(1)
            self.nodes[self.offs[k]:self.offs[k] + n] = lvl
            prev = lvl
        pos = self.leaf[self.leaf > 0]
        mn = float(pos.min()) if pos.numel() else math.inf
        self.min_bits.copy_(torch.tensor([mn], dtype=torch.float32).view(torch.int32))

    # ---------------------------------------------------------------- stats
    def total(self) -> float:
        return float(self.nodes[self.offs[self.L]].item())

    def min_leaf(self) -> float:
        return float(self.min_bits.view(torch.float32).item())
