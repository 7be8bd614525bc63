"""MI355X learner for the dueling NatureCNN: one GPU-resident step.

Per step (B = local batch), entirely on device, one stream, no host sync:

  online fwd on 2B rows, target fwd on B rows    conv1_s2d (reads the uint8 replay ring
                                                 by slot) / conv2_img / conv3 / fc
  DDQN target + Huber*IS loss + |delta| + dH     csrc/ddqn_head.hip
  fc wgrad + head wgrad + priority write-back    ONE launch (csrc/sumtree.hip
  (generation-checked, last writer wins)         fc_wgrad_head_prio_kernel)
  backward: fc, conv3, conv2 dgrad+wgrad, conv1  csrc/conv_mfma.hip, conv1_wgrad.hip
  wgrad, one split-K finalisation
  (DP) flat-gradient all-reduce over RCCL        parallel/dist.py
  grad-norm clip + centered RMSprop + bf16 pack  ONE launch (csrc/sumtree.hip
  + the NEXT step's prioritized sample           rmsprop_sample_kernel)

Periodic host work between steps: target sync (D2D copy, every
``q_target_sync_freq``), FIFO eviction + exact tree rebuild (every
``remove_old_xp_freq``), checkpoint (rank 0).

Reference parity: ``Learner.learn`` / ``compute_loss_and_priorities`` /
``update_Q`` (``learner.py:29-80``) with defects A16-A21, A30 fixed.
The step can be captured once and replayed as a HIP graph (``use_graphs``).
"""
from __future__ import annotations

import contextlib
import os

from typing import Any, Dict, Optional

import torch

from ..config import ApexConfig

# priority write-back: in the head-wgrad launch (one extra single-block tree update,
# default) or in the head kernel itself (APEX_PRIO_IN_HEAD=1)
_PRIO_IN_HEAD = os.environ.get("APEX_PRIO_IN_HEAD", "0") == "1"
from ..models.dueling import DuellingDQN
from ..models.flat_params import (FlatLayout, flat_to_reference_state, nature_segments,
                                  reference_state_to_flat)
from ..ops.fused_ops import HipBackend, TorchBackend
from ..utils.checkpoint import load_checkpoint, save_checkpoint


class FusedNatureLearner:
    def __init__(self, cfg: ApexConfig, device, replay, comm=None, backend: Optional[str] = None,
                 batch_size: Optional[int] = None):
        self.cfg = cfg
        self.rt = cfg.Runtime
        self.device = torch.device(device)
        self.replay = replay
        self.comm = comm
        self.C = cfg.frame_stack
        self.A = int(cfg.env_conf.action_dim)
        self.B = int(batch_size or cfg.Learner.replay_sample_size)
        # nature32 (Nature DQN's 32-filter conv1) runs zero-padded to 64 filters on the
        # same kernels (models/flat_params.py:reference_state_to_flat): exact math
        self.c1 = 32 if cfg.network == "nature32" else 64
        if backend is None:
            backend = "hip" if (self.device.type == "cuda" and self.rt.use_hip_kernels) else "torch"
        self.ops = HipBackend() if backend == "hip" else TorchBackend(
            torch.bfloat16 if self.device.type == "cuda" else torch.float32)
        self.act_dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        d = self.device
        self.layout = FlatLayout(nature_segments(self.C, self.A, 64))
        n = self.layout.numel
        self.p32 = torch.zeros(n, dtype=torch.float32, device=d)
        self.pbf = torch.zeros(n, dtype=self.act_dtype, device=d)
        self.g32 = torch.zeros(n, dtype=torch.float32, device=d)
        self.rms_v = torch.zeros(n, dtype=torch.float32, device=d)
        self.rms_m = torch.zeros(n, dtype=torch.float32, device=d)
        self.t32 = torch.zeros(n, dtype=torch.float32, device=d)
        self.tbf = torch.zeros(n, dtype=self.act_dtype, device=d)
        self.P = self.layout.views(self.p32)
        self.Pb = self.layout.views(self.pbf)
        self.G = self.layout.views(self.g32)
        self.T = self.layout.views(self.t32)
        self.Tb = self.layout.views(self.tbf)
        # random init identical in distribution to the reference module (torch default init)
        init = DuellingDQN((self.C, 84, 84), self.A, conv1_channels=self.c1)
        reference_state_to_flat(init.state_dict(), {k: v for k, v in self.P.items()})
        if comm is not None and comm.world_size > 1:
            comm.broadcast_flat(self.p32)
        self.pbf.copy_(self.p32)
        self.sync_target()
        self.num_q_updates = 0
        self.world = comm.world_size if comm is not None else 1
        self._alloc(self.B)
        self._graphs = None
        self._multi = None      # Runtime.graph_steps-step graph (steps())
        # Optional side stream for the weight-gradient GEMMs and the head wgrad
        # (Runtime.overlap_wgrad, off by default).  In the captured HIP graph every
        # cross-stream edge becomes an inter-queue signal wait of ~6-15 us and the
        # runtime maps branches onto hardware queues its own way (the trace showed
        # the dgrad chain queued behind side work), so one stream measured faster
        # once the latency-bound tree kernels moved into the head / optimizer
        # launches: 3454 vs 3317 steps/s (profiles/r1_step_kernels_*.md).
        self._side = torch.cuda.Stream(d) if (d.type == "cuda" and self.rt.overlap_wgrad) else None
        # clip norm: the optimizer launch sums the producers' squared-norm partials
        # itself (no separate one-block total kernel); APEX_NORM_TOTAL=1 restores it
        self._norm_total_kernel = os.environ.get("APEX_NORM_TOTAL", "0") == "1"
        self._npart = 0
        # DP gradient payload: fp32 in place, or a bf16 copy (cast inside the captured
        # segments, summed by RCCL in bf16, cast back before the optimizer)
        if self.rt.allreduce_dtype not in ("fp32", "bf16"):
            raise ValueError("Runtime.allreduce_dtype must be fp32 or bf16")
        self._comm_bf16 = self.world > 1 and self.rt.allreduce_dtype == "bf16"
        self.gcomm = torch.zeros(n, dtype=torch.bfloat16, device=d) if self._comm_bf16 else self.g32
        # producer-summed clip norm: single rank only (with DP the norm is of the
        # all-reduced gradient, so the separate squared-norm pass stays)
        self._fuse_norm = self.world == 1 and self.ops.name == "hip" and getattr(self.ops, "native_conv", False)
        # cross-shard IS-weight normaliser: min over ranks of (min_i p_i / total)
        self.ratio_local = torch.zeros(1, dtype=torch.float32, device=d)
        self.ratio_buf = torch.zeros(2, 1, dtype=torch.float32, device=d)   # double-buffered (see _dp_step)
        self.ratio_min = None
        self._ratio_work = [None, None]
        self._ratio_k = 0
        if self.world > 1:
            self.ratio_min = torch.zeros(1, dtype=torch.float32, device=d)
            self._init_ratio()
        # next-batch pre-sampling: the batch of step t+1 is drawn at the end of step t,
        # after the priority write-back -- on the HIP backend inside the optimizer
        # launch (its first blocks run the sampler: csrc/sumtree.hip
        # rmsprop_sample_kernel), so no lone latency-bound sample launch heads the
        # step.  Same draws as sampling at the head of t+1: nothing device-side
        # touches the tree in between; host-side mutations (inserts, eviction,
        # rebuild) bump replay.version and force a fresh sample at the head of t+1.
        # (The earlier side-stream variant lost: 3153 vs 3360 steps/s, the extra
        # cross-stream graph edges cost more than the sample they hid.)
        self._presample = bool(self.rt.presample)
        self._sample_ver = None
        ls = cfg.Learner.load_saved_state
        if ls:
            self.load(ls)

    # ------------------------------------------------------------- buffers
    def _alloc(self, B: int) -> None:
        d, ad = self.device, self.act_dtype
        C = self.C
        # rows [0,B) = S_t, [B,2B) = S_{t+n} (online net), [2B,3B) = S_{t+n} (target net):
        # every forward layer is ONE launch over 3B images with the weight set
        # switched at row 2B (block-uniform)
        self.S = self.replay.alloc_sample_buffers(B)
        self.slots = torch.zeros(3 * B, C, dtype=torch.int32, device=d)
        self.S["obs"] = self.slots[:B]
        self.S["nxt"] = self.slots[B:2 * B]
        self.frames = torch.zeros(3 * B, C, 84, 84, dtype=torch.uint8, device=d) if self.ops.name != "hip" \
            else torch.zeros(1, C, 84, 84, dtype=torch.uint8, device=d)
        self.y1 = torch.zeros(3 * B, 20, 20, 64, dtype=ad, device=d)
        self.y2 = torch.zeros(3 * B, 9, 9, 64, dtype=ad, device=d)
        self.y3 = torch.zeros(3 * B, 7, 7, 64, dtype=ad, device=d)
        self.h = torch.zeros(3 * B, 1024, dtype=ad, device=d)
        self.dH = torch.zeros(B, 1024, dtype=ad, device=d)
        self.dY3 = torch.zeros(B, 7, 7, 64, dtype=ad, device=d)
        self.dY2 = torch.zeros(B, 9, 9, 64, dtype=ad, device=d)
        self.dY1 = torch.zeros(B, 20, 20, 64, dtype=ad, device=d)
        self.dhead = torch.zeros(B, self.A + 1, dtype=torch.float32, device=d)
        self.td_abs = torch.zeros(B, dtype=torch.float32, device=d)
        self.loss_b = torch.zeros(B, dtype=torch.float32, device=d)
        self.partials = torch.zeros(1024, dtype=torch.float64, device=d)
        # single rank, HIP: the clip norm is summed by the gradient producers (fc wgrad
        # epilogue + grad_finalize blocks) instead of a separate pass over g32
        self.norm_part = torch.zeros(8192, dtype=torch.float64, device=d)
        self.norm_total = torch.zeros(1, dtype=torch.float64, device=d)
        self._fc_slots = 0
        self.gnorm = torch.zeros(1, dtype=torch.float32, device=d)
        # head-gradient region (zeroed by the head kernel, accumulated by head_wgrad)
        o0 = self.layout.offsets["wv"]
        o1 = self.layout.offsets["ba"] + self.A
        self.g_head_region = self.g32[o0:o1]

    # ------------------------------------------------------------ forward
    def forward_all(self) -> None:
        """Online net on rows [0,2B), target net on rows [2B,3B): one launch per layer.
        bf16 weights (Pb / Tb), fp32 biases (P / T)."""
        ops, rt, B = self.ops, self.rt, self.B
        Pb, P, Tb, T = self.Pb, self.P, self.Tb, self.T
        n = 3 * B
        ops.conv1_fwd_ring(self.replay.frames, self.slots, self.frames, Pb["w1"], P["b1"], rt.obs_scale, self.y1,
                           Tb["w1"], T["b1"], 2 * B)
        ops.conv_fwd(self.y1, Pb["w2"], P["b2"], 2, self.y2, Tb["w2"], T["b2"], 2 * B)
        ops.conv_fwd(self.y2, Pb["w3"], P["b3"], 1, self.y3, Tb["w3"], T["b3"], 2 * B)
        ops.fc_fwd(self.y3.reshape(n, 3136), Pb["wfc"], P["bfc"], self.h, Tb["wfc"], T["bfc"], 2 * B)

    def _head_params(self, V):
        return {k: V[k] for k in ("wv", "bv", "wa", "ba")}

    # ---------------------------------------------------------------- step
    # The step is three segments.  With one rank they run back to back (one HIP
    # graph).  With data parallelism the flat gradient is all-reduced in two
    # buckets over RCCL: the fc+heads bucket (12.9 MB, complete once segment 1
    # has produced the head and fc WEIGHT gradients) is reduced on RCCL's stream
    # WHILE segment 2 runs the fc dgrad and the whole conv backward on the compute
    # stream; the small conv bucket follows; segment 3 (clip + RMSprop) waits for
    # both.  Gradients are pre-scaled by 1/(B*world) in the head kernel, so the SUM
    # all-reduce yields the mean.
    def _seg1(self) -> None:
        """(sample), forward (online+target), loss, head + fc weight gradients with the
        priority write-back."""
        B, rt, ops = self.B, self.rt, self.ops
        ops.prepare(self.Pb)
        if not self._presample or self._sample_ver != self.replay.version:
            self._sample()
        S = self.S
        self._mark("sample")
        # conv1 reads the uint8 frame stacks straight from the replay ring by slot
        self.forward_all()
        self._mark("forward")
        isw = S["weights"] if rt.use_is_weights else None
        # the batch's priorities go back into the sum-tree from the head-wgrad launch
        # (HIP: one extra block, csrc/sumtree.hip head_wgrad_prio_kernel)
        ops.head(self.h[:2 * B], self.h[2 * B:], self._head_params(self.P), self._head_params(self.T), S["act"],
                 S["rew"], S["gam"], isw, rt.loss == "huber", rt.huber_delta, 1.0 / (B * self.world),
                 self.td_abs, self.loss_b, self.dH, self.dhead, zero=self.g_head_region,
                 prio=(self.replay, S["idx"], S["gen"]) if _PRIO_IN_HEAD else None)
        self._mark("head")
        prio = None if _PRIO_IN_HEAD else (self.replay, S["idx"], S["gen"], self.td_abs)
        nrm = (self.norm_part, 0) if self._fuse_norm else None
        if self._side is None:
            # fc wgrad + head wgrad + priority write-back: one launch on the HIP backend
            # (csrc/sumtree.hip fc_wgrad_head_prio_kernel)
            self._fc_slots = ops.fc_head_wgrad(self.dH, self.y3[:B], self.G["wfc"], self.G["bfc"], self.h,
                                               self.dhead, self.G, prio, norm=nrm)
        else:
            with self._on_side():
                ops.head_wgrad(self.h, self.dhead, self.G, prio=prio)
            with self._on_side(self.rt.overlap_wgrad):
                self._fc_slots = ops.fc_wgrad(self.dH, self.y3[:B], self.G["wfc"], self.G["bfc"], norm=nrm) or 0
        if self.world > 1:
            self._join_side()   # the fc/heads bucket all-reduce starts right after this segment
            if self._comm_bf16:
                cut = self.layout.offsets["wfc"]
                self.gcomm[cut:].copy_(self.g32[cut:])
        self._mark("fc_wgrad")

    def _sample(self) -> None:
        """The sampler writes idx / IS weights / records and the frame-ring slots of
        S_t, S_{t+n} (twice: online and target rows) into the step's buffers."""
        self.replay.sample(self.B, out=self.S, ratio_min_global=self.ratio_min, nxt2=self.slots[2 * self.B:])
        self._sample_ver = self.replay.version

    def _seg2(self) -> None:
        """fc dgrad + conv backward (with DP, all of it overlaps the fc/heads bucket
        all-reduce): the dgrad chain, conv3/conv2 wgrad (side stream when
        ``overlap_wgrad``), conv1 wgrad last."""
        B, rt, ops, G, Pb = self.B, self.rt, self.ops, self.G, self.Pb
        jobs = []    # split-K reductions, finalised in ONE launch at the end
        ops.fc_dgrad(self.dH, self.y3[:B], Pb["wfc"], self.dY3)
        with self._on_side(rt.overlap_wgrad):
            ops.conv_wgrad(self.dY3, self.y2[:B], 3, 1, G["w3"], G["b3"], jobs=jobs)
        ops.conv_dgrad(self.dY3, Pb["w3"], 1, self.y2[:B], self.dY2)
        with self._on_side(rt.overlap_wgrad):
            ops.conv_wgrad(self.dY2, self.y1[:B], 4, 2, G["w2"], G["b2"], jobs=jobs)
        ops.conv_dgrad(self.dY2, Pb["w2"], 2, self.y1[:B], self.dY1)
        ops.conv1_wgrad_ring(self.dY1, self.replay.frames, self.slots[:B], self.frames, rt.obs_scale, G["w1"],
                             G["b1"], jobs=jobs)
        self._join_side()      # (overlap_wgrad) side-stream wgrads done before the finalisation
        norm = dict(part=self.norm_part, slot0=self._fc_slots,
                    total=self.norm_total if self._norm_total_kernel else None) if self._fuse_norm else None
        self._npart = ops.finalize_grads(jobs, self.g_head_region if self._fuse_norm else None, norm)
        if self._comm_bf16:
            cut = self.layout.offsets["wfc"]
            self.gcomm[:cut].copy_(self.g32[:cut])
        if self.world > 1:
            self._join_side()  # a graph segment must rejoin its forked streams
        self._mark("conv_backward")

    # ------------------------------------------------------- phase timing
    _marks = None

    def _mark(self, name: str) -> None:
        """Record a CUDA event at a phase boundary (eager profiling steps only)."""
        if self._marks is not None:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self._marks.append((name, ev))

    def profile_step(self) -> Dict[str, float]:
        """Run ONE eager (un-graphed) learner step with CUDA events between its
        phases; returns milliseconds per phase (sample, forward, head,
        fc_wgrad, conv_backward (fc dgrad + convs), [allreduce_wait], optimizer) and
        the total.  Counts as a normal update."""
        if self.device.type != "cuda":
            return {}
        start = torch.cuda.Event(enable_timing=True)
        start.record()
        self._marks = []
        try:
            if self.world > 1:
                self._dp_step(False)
            else:
                self._step_body()
        finally:
            marks, self._marks = self._marks, None
        torch.cuda.synchronize(self.device)
        out, prev = {}, start
        for name, ev in marks:
            out[name] = out.get(name, 0.0) + prev.elapsed_time(ev)
            prev = ev
        out["total"] = start.elapsed_time(prev)
        self.num_q_updates += 1
        return out

    def _on_side(self, enabled: bool = True):
        """Context: launches go to the side stream, after everything queued so far on
        the compute stream (fork).  No-op without a GPU or when not ``enabled``."""
        if self._side is None or not enabled:
            return contextlib.nullcontext()
        self._side.wait_stream(torch.cuda.current_stream(self.device))
        return torch.cuda.stream(self._side)

    def _join_side(self) -> None:
        if self._side is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._side)

    def _seg3(self) -> None:
        """clip + centered RMSprop (+bf16 pack) with the next batch's draw, shard stats
        (DP)."""
        rt, ops = self.rt, self.ops
        if self._comm_bf16:
            self.g32.copy_(self.gcomm)
        # with pre-sampling the optimizer launch also draws step t+1's batch (every
        # read of this step's sample buffers is behind us)
        nxt = (self.replay, self.B, self.S, self.ratio_min, self.slots[2 * self.B:]) if self._presample else None
        ops.optimizer(self.p32, self.g32, self.rms_v, self.rms_m, self.pbf, rt.lr, rt.rms_decay, rt.rms_eps,
                      rt.grad_clip, rt.centered_rmsprop, self.partials, self.gnorm,
                      norm_total=self._norm_arg(), sample=nxt)
        if self._presample:
            self._sample_ver = self.replay.version
        self._mark("optimizer")
        if self.world > 1:
            # local min_i p_i / total for the global IS-weight normaliser (all-reduced MIN after the step)
            rp = self.replay
            tot = rp.nodes[rp.offs[rp.L]:rp.offs[rp.L] + 1].float()
            self.ratio_local.copy_(rp.min_bits.view(torch.float32) / tot)

    def _norm_arg(self):
        """The optimizer's clip-norm source: None (it computes the norm of g32), the
        one-value total, or (partials, count) summed inside the optimizer launch."""
        if not self._fuse_norm:
            return None
        return self.norm_total if self._norm_total_kernel else (self.norm_part, self._npart)

    def _step_body(self) -> None:
        self._seg1()
        self._seg2()
        self._seg3()

    def _dp_step(self, graphs: bool) -> None:
        import torch.distributed as dist
        cut = self.layout.offsets["wfc"]
        run = (lambda i: self._graphs[i].replay()) if graphs else (lambda i: (self._seg1, self._seg2,
                                                                                self._seg3)[i]())
        # The IS normaliser all-reduced after step t-1 is consumed by step t+1, not
        # step t: that tiny MIN all-reduce then completes under step t's compute
        # (RCCL's stream already ran it before step t's gradient buckets) instead of
        # sitting between seg3 and the next sample as a latency bubble.  The
        # normaliser is a global per-step scale of the IS weights; one step of lag
        # changes it by the few priorities one step rewrites.
        k = self._ratio_k
        prev = self._ratio_work[k]
        if prev is not None:
            prev.wait()
            self.ratio_min.copy_(self.ratio_buf[k])
            self._ratio_work[k] = None
        run(0)
        w_fc = dist.all_reduce(self.gcomm[cut:], op=dist.ReduceOp.SUM, async_op=True)
        run(1)  # conv backward overlaps the fc/head bucket all-reduce
        w_cv = dist.all_reduce(self.gcomm[:cut], op=dist.ReduceOp.SUM, async_op=True)
        w_fc.wait()
        w_cv.wait()
        self._mark("allreduce_wait")
        run(2)
        self.ratio_buf[k].copy_(self.ratio_local)
        self._ratio_work[k] = dist.all_reduce(self.ratio_buf[k], op=dist.ReduceOp.MIN, async_op=True)
        self._ratio_k = 1 - k

    def step(self) -> None:
        """One learner update (asynchronous on the current stream)."""
        graphs = self.rt.use_graphs and self.device.type == "cuda"
        if graphs and self._graphs is None:
            self._capture()
        if graphs and self._presample and self._sample_ver != self.replay.version:
            self._sample()     # host-side replay mutation since the pre-sample: redraw
        if self.world > 1:
            self._dp_step(graphs)
        elif graphs:
            self._graphs[0].replay()
        else:
            self._step_body()
        self.num_q_updates += 1
        L = self.cfg.Learner
        if self.num_q_updates % L.q_target_sync_freq == 0:
            self.sync_target()

    def steps(self, n: int) -> None:
        """``n`` learner updates.  On one rank with HIP graphs, chunks of
        ``Runtime.graph_steps`` updates replay ONE graph holding that many steps
        (each graph launch costs ~9 us of idle GPU at its boundary); chunks never
        straddle a target-network sync.  Same updates as ``n`` calls of :meth:`step`."""
        k = int(self.rt.graph_steps)
        graphs = self.rt.use_graphs and self.device.type == "cuda"
        if k <= 1 or not graphs or self.world > 1:
            for _ in range(n):
                self.step()
            return
        f = self.cfg.Learner.q_target_sync_freq
        while n > 0:
            to_sync = f - self.num_q_updates % f
            if n < k or to_sync < k:
                self.step()
                n -= 1
                continue
            if self._graphs is None:
                self._capture()
            if self._multi is None:
                self._multi = torch.cuda.CUDAGraph()
                torch.cuda.synchronize(self.device)
                with torch.cuda.graph(self._multi):
                    for _ in range(k):
                        self._step_body()
            if self._presample and self._sample_ver != self.replay.version:
                self._sample()
            self._multi.replay()
            self.num_q_updates += k
            n -= k
            if self.num_q_updates % f == 0:
                self.sync_target()

    def _capture(self) -> None:
        """Warm up on a side stream (allocator pools, workspaces), restore state,
        then capture: one graph for a single rank, three segment graphs for DP."""
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        snap = self._snapshot()
        with torch.cuda.stream(s):
            for _ in range(2):
                self._step_body()
        torch.cuda.current_stream(self.device).wait_stream(s)
        self._restore(snap)
        if self._presample:    # the graphs start from a drawn batch (their seg1 holds no sample)
            self._sample()
        torch.cuda.synchronize(self.device)
        if self.world == 1:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._step_body()
            self._graphs = [g]
        else:
            self._graphs = []
            for seg in (self._seg1, self._seg2, self._seg3):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    seg()
                self._graphs.append(g)
        # capture recorded the step without executing it; state is as before

    def _init_ratio(self) -> None:
        import torch.distributed as dist
        rp = self.replay
        tot = rp.nodes[rp.offs[rp.L]:rp.offs[rp.L] + 1].float().clamp_min(1e-30)
        buf = self.ratio_buf[0]
        buf.copy_(rp.min_bits.view(torch.float32) / tot)
        dist.all_reduce(buf, op=dist.ReduceOp.MIN)
        self.ratio_min.copy_(buf)

    def refresh_replay_stats(self) -> None:
        """Re-derive the cross-shard IS normaliser (after inserts / eviction)."""
        if self.world > 1:
            for i, w in enumerate(self._ratio_work):
                if w is not None:
                    w.wait()
                    self._ratio_work[i] = None
            self._init_ratio()

    def _snapshot(self):
        rp = self.replay
        return [t.clone() for t in (self.p32, self.pbf, self.rms_v, self.rms_m, rp.leaf, rp.nodes,
                                    rp.min_bits, rp.ctr)]

    def _restore(self, snap) -> None:
        rp = self.replay
        for dst, src in zip((self.p32, self.pbf, self.rms_v, self.rms_m, rp.leaf, rp.nodes, rp.min_bits,
                             rp.ctr), snap):
            dst.copy_(src)

    def sync_target(self) -> None:
        self.t32.copy_(self.p32)
        self.tbf.copy_(self.pbf)

    # ------------------------------------------------------------ metrics
    def last_metrics(self) -> Dict[str, float]:
        return {"loss": float(self.loss_b.mean()), "td_abs_mean": float(self.td_abs.mean()),
                "grad_norm": float(self.gnorm[0])}

    def q_values(self, frames_u8: torch.Tensor) -> torch.Tensor:
        """Greedy-evaluation helper: q for a (N, C, 84, 84) uint8 batch."""
        sd = self.reference_state_dict()
        net = DuellingDQN((self.C, 84, 84), self.A, conv1_channels=self.c1).to(self.device)
        net.load_state_dict(sd)
        with torch.no_grad():
            return net(frames_u8.to(self.device))[2]

    # ------------------------------------------------------------- params
    def reference_state_dict(self):
        return flat_to_reference_state(self.P, self.c1)

    def load_reference_state_dict(self, sd) -> None:
        reference_state_to_flat(sd, self.P)
        self.pbf.copy_(self.p32)

    def save(self, path: str) -> None:
        tgt = flat_to_reference_state(self.T, self.c1)
        save_checkpoint(path, self.reference_state_dict(), Q_target_state=tgt,
                        optimizer_state={"rms_v": self.rms_v.cpu(), "rms_m": self.rms_m.cpu()},
                        num_q_updates=self.num_q_updates, config=self.cfg.to_dict())

    def load(self, path: str) -> bool:
        ck = load_checkpoint(path)
        if ck is None:
            return False
        self.load_reference_state_dict(ck["Q_state"])
        if "Q_target_state" in ck:
            reference_state_to_flat(ck["Q_target_state"], self.T)
            self.tbf.copy_(self.t32)
        else:
            self.sync_target()
        opt = ck.get("optimizer_state")
        if isinstance(opt, dict) and "rms_v" in opt:
            self.rms_v.copy_(opt["rms_v"])
            self.rms_m.copy_(opt["rms_m"])
        self.num_q_updates = int(ck.get("num_q_updates", 0))
        return True
