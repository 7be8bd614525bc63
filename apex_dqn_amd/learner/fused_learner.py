"""MI355X learner for the dueling NatureCNN: one GPU-resident step.

Per step (B = local batch), entirely on device, one stream, no host sync:

  online fwd on 2B rows, target fwd on B rows    conv1_s2d (reads the uint8 replay ring
                                                 by slot) / conv2 / conv3 / fc
  DDQN target + Huber*IS loss + |delta| + dH     csrc/ddqn_head.hip
  fc wgrad + head wgrad + priority write-back    ONE launch (csrc/sumtree.hip
  (generation-checked, last writer wins)         fc_wgrad_head_prio_kernel)
  backward: fc, conv3, conv2 dgrad+wgrad, conv1  csrc/conv_mfma.hip, conv2_img.hip,
  wgrad, one split-K finalisation                conv1_wgrad.hip
  (DP) gradient exchange over RCCL               learner/dp_step.py: factored fc exchange,
                                                 bucketed all-reduce, sharded optimizer,
                                                 the replay shards' statistics (one global
                                                 prioritized replay), captured in the
                                                 step's HIP graph
  grad-norm clip + centered RMSprop + bf16 pack  ONE launch (csrc/sumtree.hip
  + the NEXT step's prioritized sample           rmsprop_sample_kernel)

Precision (``Runtime.dtype``):
  * ``fp32`` (default, the reference's precision: ``learner.py:37-38`` ``.float()``,
    fp32 ``nn.Conv2d`` / ``nn.Linear``): "split" operands.  Every bf16 weight copy,
    activation and gradient carries a lo plane (value = hi + lo); the GEMM kernels
    issue three bf16 MFMAs per fragment pair (hi.hi + lo.hi + hi.lo) with fp32
    accumulation, conv1 multiplies the exact uint8 pixels by f16 hi + lo weights;
    per-product error ~2^-17 relative, vs 2^-9 for plain bf16.  fp32 master
    weights, fp32 gradients and fp32 RMSprop state as before.
  * ``bf16``: bf16 operands, fp32 accumulation and master weights (the round-1 path).

Periodic host work between steps: target sync (D2D copy, every
``q_target_sync_freq``), FIFO eviction + exact tree rebuild (every
``remove_old_xp_freq``), checkpoint (rank 0).

Reference parity: ``Learner.learn`` / ``compute_loss_and_priorities`` /
``update_Q`` (``learner.py:29-80``) with defects A16-A21, A30 fixed.
The step is captured once and replayed as a HIP graph (``use_graphs``).
"""
from __future__ import annotations

from typing import Any, Dict, Optional

import torch

from ..config import ApexConfig
from ..models.dueling import DuellingDQN
from ..models.flat_params import (FlatLayout, flat_to_reference_state, nature_segments,
                                  reference_state_to_flat)
from ..ops.fused_ops import HipBackend, TorchBackend, split_into
from ..ops.switches import SW
from ..utils.checkpoint import (adopt_obs_scale, layout_segments, load_checkpoint, pack_flat_state,
                                save_checkpoint, unpack_flat_state, checkpoint_network)
from .dp_step import DataParallelStep, Streams
from .is_norm import IsNormMixin


def _enable_sharding(replay, comm, rt, mcap: int = 0) -> None:
    """Turn the rank-local replay into one shard of the global replay (idempotent;
    ``mcap``: the cap on a draw's global batch, ``ApexConfig.dp_batch``)."""
    if not replay.sharded:
        # the global draw must use ONE seed on every rank (rank 0's Runtime.seed: the
        # ranks may seed their local RNGs differently, e.g. bench.py's 1234 + rank)
        seed0 = comm.broadcast_int(int(rt.seed)) if hasattr(comm, "broadcast_int") else int(rt.seed)
        replay.enable_sharding(comm.rank, comm.world_size, shard_seed=(seed0 << 20) ^ 0x5EED,
                               group=comm.group, mcap=mcap)
    replay.shard_mcap = int(mcap)
    if not rt.use_is_weights:
        replay.beta = 0.0


def dp_layout(cfg: ApexConfig, comm, batch_size: Optional[int] = None, allow_force: bool = True):
    """(world, dp, rows per rank, global-batch cap) of a learner on ``comm``: the DP
    step runs at world > 1 or with ``Runtime.force_dp``; ``Runtime.batch_scope`` decides
    whether ``replay_sample_size`` is the update's global batch or every rank's
    (``ApexConfig.dp_batch``).  ``batch_size`` overrides the rows per rank."""
    world = comm.world_size if comm is not None else 1
    dp = world > 1 or (allow_force and bool(cfg.Runtime.force_dp) and comm is not None)
    rows, mcap = cfg.dp_batch(world, dp)
    if batch_size:
        rows = int(batch_size)
        mcap = mcap if cfg.Runtime.batch_scope == "global" else world * rows
    return world, dp, rows, mcap


class FusedNatureLearner(IsNormMixin, DataParallelStep):
    kind = "fused"

    def __init__(self, cfg: ApexConfig, device, replay, comm=None, backend: Optional[str] = None,
                 batch_size: Optional[int] = None, split: Optional[bool] = None):
        self.cfg = cfg
        self.rt = cfg.Runtime
        self.device = torch.device(device)
        self.replay = replay
        self.comm = comm
        self.C = cfg.frame_stack
        self.A = int(cfg.env_conf.action_dim)
        # B = the rows this rank computes: replay_sample_size, or with a global-batch DP
        # step (Runtime.batch_scope) its share of the global draw plus slack (dp_layout)
        self.world, self._dp, self.B, self.mcap = dp_layout(cfg, comm, batch_size)
        if self.rt.dtype not in ("fp32", "bf16"):
            raise ValueError("Runtime.dtype must be fp32 or bf16")
        self.precision = self.rt.dtype
        cuda = self.device.type == "cuda"
        # nature32 (Nature DQN's 32-filter conv1) runs zero-padded to 64 filters on the
        # same kernels (models/flat_params.py:reference_state_to_flat): exact math
        self.c1 = 32 if cfg.network == "nature32" else 64
        if backend is None:
            backend = "hip" if (cuda and self.rt.use_hip_kernels) else "torch"
        if backend == "hip":
            self.ops = HipBackend()
        else:
            # torch backend: the fp32 oracle (or torch bf16 when asked for on a GPU)
            self.ops = TorchBackend(torch.bfloat16 if (cuda and self.precision == "bf16") else torch.float32)
        # split mode: fp32-accurate hi/lo bf16 operands (the HIP path of dtype fp32; the
        # torch backend emulates it when forced, which tests the plumbing on the CPU)
        self.split = (self.precision == "fp32" and backend == "hip") if split is None else bool(split)
        self.act_dtype = torch.bfloat16 if (self.split or (cuda and self.ops.name == "hip")
                                            or (cuda and self.precision == "bf16")) else torch.float32
        # conv1 -> conv2 forward in one launch, y1 kept in LDS (csrc/conv12_fused.hip): the
        # split kernel in fp32 mode, its one-plane variant for the bf16 learner
        # (SW.conv12_bf16 = False: the bf16 learner runs the two image-resident kernels)
        # (the torch backend emulates the split kernel's contract: ops.conv12_fwd)
        self._c12 = self.split or (backend == "hip" and self.ops._conv12_native() and SW.conv12_bf16)
        d = self.device
        self.layout = FlatLayout(nature_segments(self.C, self.A, 64))
        n = self.layout.numel
        self.p32 = torch.zeros(n, dtype=torch.float32, device=d)
        # bf16 compute copies [hi | lo] of the online / target parameters (lo: split mode)
        nb = 2 * n if self.split else n
        self._pbf_all = torch.zeros(nb, dtype=self.act_dtype, device=d)
        self._tbf_all = torch.zeros(nb, dtype=self.act_dtype, device=d)
        self.pbf, self.tbf = self._pbf_all[:n], self._tbf_all[:n]
        self.pbf_lo = self._pbf_all[n:] if self.split else None
        self.tbf_lo = self._tbf_all[n:] if self.split else None
        self.g32 = torch.zeros(n, dtype=torch.float32, device=d)
        self.rms_v = torch.zeros(n, dtype=torch.float32, device=d)
        self.rms_m = torch.zeros(n, dtype=torch.float32, device=d)
        self.t32 = torch.zeros(n, dtype=torch.float32, device=d)
        self._frag_out = None    # the optimizer stores the fused forward's online operands
        self.P = self.layout.views(self.p32)
        self.Pb = self.layout.views(self.pbf)
        self.G = self.layout.views(self.g32)
        self.T = self.layout.views(self.t32)
        self.Tb = self.layout.views(self.tbf)
        self.Pl = self.layout.views(self.pbf_lo) if self.split else None
        self.Tl = self.layout.views(self.tbf_lo) if self.split else None
        # random init identical in distribution to the reference module (torch default init)
        init = DuellingDQN((self.C, 84, 84), self.A, conv1_channels=self.c1)
        reference_state_to_flat(init.state_dict(), {k: v for k, v in self.P.items()})
        if comm is not None and comm.world_size > 1:
            comm.broadcast_flat(self.p32)
        self._refresh_bf16()
        self._tgt_packed = False
        self.sync_target()
        self.num_q_updates = 0
        # self._dp: the data-parallel step (collectives, sharded replay); Runtime.force_dp
        # runs it at world 1 too (an initialised process group of one rank: RCCL capture
        # checks and the segmented-step overhead on a single GPU)
        # image work queues in the persistent kernels (ops/conv.py Workspace.work_queue):
        # only where RCCL's kernels may hold CUs during the step -- world > 1 (a forced-DP
        # step on one rank has no peer traffic beside it: static order)
        if hasattr(self.ops, "ws"):
            self.ops.ws.work_queue = self.world > 1
        self._alloc(self.B)
        self._init_is_norm()
        self._graphs = None     # one-update graph
        self._multi = None      # Runtime.graph_steps-update graph (steps())
        self.graph_captures = 0  # HIP graphs captured so far (the bench asserts none in its timed region)
        self._graphs_warm = False
        self._npart = 0
        # DP gradient payload: fp32 in place, or a bf16 copy (cast inside the step, summed
        # by RCCL in bf16, cast back before the optimizer)
        if self.rt.allreduce_dtype not in ("fp32", "bf16"):
            raise ValueError("Runtime.allreduce_dtype must be fp32 or bf16")
        self._comm_bf16 = self._dp and self.rt.allreduce_dtype == "bf16"
        self.gcomm = torch.zeros(n, dtype=torch.bfloat16, device=d) if self._comm_bf16 else self.g32
        # DP exchange of the fc weight gradient (Runtime.dp_fc_exchange).  Its gradient is
        # dW = dH^T X over the global batch: rank r holds rows (dH_r, X_r), rank <= its row
        # count.  "factors" all-gathers those rows -- exactly the bf16 (hi / lo) operands
        # the kernels multiply -- and every rank forms dW of the WHOLE global batch with the
        # same kernel in the same order: W x rows x (1024 + 3136) values move instead of the
        # 3.2 M-float gradient (a global-batch step at W = 8: 1.2 MB sent per rank vs 12.9 MB
        # all-reduced), the result is bit-identical on every rank, and only the conv and
        # head gradients (0.48 MB) are all-reduced.  "auto": factors while W x rows <= 1024
        # and W > 1 (at world 1 -- the forced-DP rehearsal -- there is no traffic to save and
        # the all-gather, separate head wgrad and pack cost ~20 us more than the copy-like
        # all-reduce: 2,319 vs 2,441 steps/s, profiles/r4_bench_forced_dp_*).
        mode = self.rt.dp_fc_exchange
        self._fc_factors = self._dp and not self._comm_bf16 and (
            mode == "factors" or (mode == "auto" and 1 < self.world and self.world * self.B <= 1024))
        if self._fc_factors:
            planes = 2 if self.split else 1
            self._fx_cols = [1024] * planes + [3136] * planes      # [dH | dH lo | X | X lo]
            self._alloc_factors()
        # producer-summed clip norm: the fc wgrad epilogue and the grad_finalize blocks
        # write squared-norm partials of the values they store, the optimizer launch sums
        # them.  With DP the norm is of the all-reduced gradient: the optimizer's own pass.
        self._fuse_norm = not self._dp and self.ops.name == "hip" and getattr(self.ops, "native_conv", False)
        # DP: the rank-local replay shards form ONE prioritized replay (replay/gpu_replay.py
        # enable_sharding): every step all-gathers the shards' (sum p^alpha, min p^alpha)
        # right after the priority write-back and the next batch is one global draw,
        # identical on every rank, of which each rank keeps the part in its own shard.
        # Rows drawn elsewhere carry IS weight 0, so the IS weights always enter the loss
        # (with use_is_weights off: beta = 0, i.e. weights 0 / W B / M only).
        self._isw = bool(self.rt.use_is_weights) or self._dp
        # batch-max IS normalisation (Runtime.is_normalise): the head kernel leaves the
        # batch's largest (p / p_min)^-beta -- with DP in this rank's slot of the shard
        # statistics, all-gathered later in the step -- and the optimizer divides the
        # gradient by the maximum (csrc/ddqn_head.hip IsNorm, rmsprop_common.h)
        # the DP step's collectives: torch.distributed (RCCL process group / gloo) or the
        # native RCCL communicator on its own stream (Runtime.comm_backend, parallel/rccl.py)
        self.coll = None
        if self._dp:
            from ..parallel.rccl import make_collectives
            # (the native communicator joins an RCCL process group's ranks; gloo groups -- CPU
            # tests, several ranks rehearsing on one GPU -- use torch.distributed)
            backend = self.rt.comm_backend if (cuda and self._backend_name() == "nccl") else "torch"
            self.coll = make_collectives(comm, backend, self.device)
            _enable_sharding(replay, comm, self.rt, self.mcap)
            replay.gather_shard_stats(coll=self.coll)
        # DP step as ONE captured graph including the RCCL collectives (the native
        # communicator, or emulated copies); gloo (CPU tests, one-GPU rehearsals) cannot be
        # captured, and the torch.distributed RCCL process group is run eagerly: its watchdog
        # queried events recorded inside the capture (hipErrorCapturedEvent abort,
        # profiles/r5_dp_capture_probe.txt)
        self._dp_graphs = self._dp and cuda and self.coll.name in ("native", "emulated")
        self._ordered_coll = self._dp and cuda and (self.coll.name in ("native", "emulated")
                                                   or self._backend_name() == "nccl")
        # single rank: the weight gradients beside the data-gradient chain (SW.bwd_branches);
        # the DP step always runs them on the branch (learner/dp_step.py)
        self._branched = (not self._dp) and cuda and SW.bwd_branches
        # (a high-priority branch stream measured neutral: 2,677 / 2,674 vs 2,685 / 2,684,
        # profiles/r4_ab_branch_priority_neutral.txt -- the captured graph's queues do not
        # keep it)
        self._wg_stream = torch.cuda.Stream(self.device) if (self._branched or (self._dp and cuda)) else None
        self._streams = Streams(self.device, self._wg_stream if self._dp else None)
        if self._dp and cuda and hasattr(self.coll, "use_stream"):
            # the collectives run on the backward's branch stream itself: the captured step
            # then has two chains (main, branch) as the single-rank step, which the HIP graph
            # executor runs on two queues -- with a third (comm) stream it interleaved the
            # chains' kernels on shared queues and serialized the branch behind the main
            # chain (profiles/r5_step_timeline_emu8_comm_stream.txt)
            self.coll.use_stream(self._wg_stream)
        self._dp_setup()
        # the fc layer's split-K epilogue runs inside the head launch (ops.fc_fwd defer_head;
        # SW.fc_epi_in_head = False keeps the separate epilogue launch)
        self._defer_fc_epilogue = SW.fc_epi_in_head
        # next-batch pre-sampling: the batch of step t+1 is drawn at the end of step t,
        # after the priority write-back -- on the HIP backend inside the optimizer launch
        # (its first blocks run the sampler: csrc/sumtree.hip rmsprop_sample_kernel), so
        # no lone latency-bound sample launch heads the step.  Same draws as sampling at
        # the head of t+1: nothing device-side touches the tree in between; host-side
        # mutations (eviction, rebuild) bump replay.version and force a fresh sample at
        # the head of t+1.
        self._presample = bool(self.rt.presample)
        self._sample_ver = None
        self._setup_frag_out()
        self._fit_rows()          # global batch: rows for the largest shard's share (dp_step.py)
        ls = cfg.Learner.load_saved_state
        if ls:
            self.load(ls)

    def _setup_frag_out(self) -> None:
        """Split mode on the fused conv1 -> conv2 forward with pre-sampling: the optimizer +
        sample launch stores the updated w1 / w2 in the forward's fragment order
        (csrc/cf_pack.h cf_frag_store; elementwise, no hand-off between workgroups), so the
        step runs no pack launch for the online set (forward_all pack_sets).  Host-side
        weight changes repack eagerly (_online_changed).  SW.opt_frags = False: pack launch."""
        self._frag_out = None
        ops = self.ops
        if not SW.opt_frags:
            return
        if not (self._c12 and self._presample and getattr(self.replay, "use_hip", False)
                and getattr(ops, "_conv12_native", lambda: False)()):
            return
        from ..ops import conv as C
        off = self.layout.offsets
        self._frag_out = C.conv12_frag_out(ops.ws, self.P["w1"], off["w1"], off["w2"], self.rt.obs_scale,
                                           w3_off=off["w3"])
        self._online_changed()

    def _online_changed(self) -> None:
        """Online weights changed outside a step (init, load, restore, replica fix): repack
        the fused forward's online operands now (the optimizer keeps them current)."""
        if getattr(self, "_frag_out", None) is not None:
            c1, c2 = self._conv12_weights()
            self.ops.conv12_pack(c1, c2, self.rt.obs_scale, sets=1, c3=self._conv3_weights())

    def _backend_name(self) -> str:
        try:
            import torch.distributed as dist
            return dist.get_backend() if dist.is_initialized() else ""
        except Exception:  # pragma: no cover
            return ""

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

        def act(*shape):
            """hi buffer (+ its lo plane in split mode)"""
            return (torch.zeros(*shape, dtype=ad, device=d),
                    torch.zeros(*shape, dtype=ad, device=d) if self.split else None)

        self.y1, self.y1_lo = act(3 * B, 20, 20, 64)
        self.y2, self.y2_lo = act(3 * B, 9, 9, 64)
        self.y3, self.y3_lo = act(3 * B, 7, 7, 64)
        self.h, self.h_lo = act(3 * B, 1024)
        self.dH, self.dH_lo = act(B, 1024)
        self.dY3, self.dY3_lo = act(B, 7, 7, 64)
        self.dY2, self.dY2_lo = act(B, 9, 9, 64)
        self.dY1, self.dY1_lo = act(B, 20, 20, 64)
        self.dhead = torch.zeros(B, self.A + 1, dtype=torch.float32, device=d)
        self.td_abs = torch.zeros(B, dtype=torch.float32, device=d)
        self.loss_b = torch.zeros(B, dtype=torch.float32, device=d)
        self.partials = torch.zeros(1024, dtype=torch.float64, device=d)
        # single rank, HIP: the clip norm is summed by the gradient producers (fc wgrad
        # epilogue + grad_finalize blocks) instead of a separate pass over g32
        self.norm_part = torch.zeros(8192, dtype=torch.float64, device=d)
        self._fc_slots = 0
        self.gnorm = torch.zeros(1, dtype=torch.float32, device=d)
        # head-gradient region (zeroed by the head kernel, accumulated by head_wgrad)
        o0 = self.layout.offsets["wv"]
        o1 = self.layout.offsets["ba"] + self.A
        self.g_head_region = self.g32[o0:o1]

    def _lo(self, **kw) -> Dict[str, Any]:
        """Split-mode keyword arguments of an op (empty in bf16 / plain fp32 mode)."""
        return kw if self.split else {}

    # ------------------------------------------------------------ forward
    @property
    def _conv123(self) -> bool:
        """conv3 inside the fused conv1 -> conv2 launch (small launches only, SW.conv123_max_images)."""
        return bool(self._c12) and 0 < 3 * self.B <= SW.conv123_max_images

    def forward_all(self, defer_head: bool = False) -> None:
        """Online net on rows [0,2B), target net on rows [2B,3B): one launch per layer.
        bf16 weights (Pb / Tb, + Pl / Tl lo planes in split mode), fp32 biases (P / T).
        ``defer_head``: the fc layer's split-K epilogue may be left to the step's head
        launch (which then writes h rows [0, B) only)."""
        ops, rt, B = self.ops, self.rt, self.B
        Pb, P, Tb, T, Pl, Tl = self.Pb, self.P, self.Tb, self.T, self.Pl, self.Tl
        sp = self.split
        n = 3 * B
        # c2f: conv2's weights packed for its forward in the same launch (csrc/conv2_wfrag.h)
        if self._c12:
            # conv1 -> conv2 in one launch, y1 kept in LDS; only the S_t rows' y1 (the
            # backward's input) is written out (csrc/conv12_fused.hip)
            # (the target set's weight fragments are repacked at each target change:
            # _target_changed; the step packs the online set only)
            c1, c2 = self._conv12_weights()
            online = 0 if self._frag_out is not None else 1     # (stored by the last optimizer launch)
            # conv3 in the same launch from y2 in LDS (SW.conv123_fused)
            c3 = self._conv3_weights() if self._conv123 else None
            ops.conv12_fwd(self.replay.frames, self.slots, self.frames, rt.obs_scale, self.y1, self.y1_lo, self.y2,
                           self.y2_lo, c1, c2, rows_first=2 * B, copy_n=B,
                           pack_sets=online | (0 if self._tgt_packed else 2), c3=c3, y3=self.y3, y3_lo=self.y3_lo)
        else:
            c2f = (Pb["w2"], None, Tb["w2"], None)
            ops.conv1_fwd_ring(self.replay.frames, self.slots, self.frames, Pb["w1"], P["b1"], rt.obs_scale, self.y1,
                               Tb["w1"], T["b1"], 2 * B, c2f=c2f)
            ops.conv_fwd(self.y1, Pb["w2"], P["b2"], 2, self.y2, Tb["w2"], T["b2"], 2 * B)
        self._issue_params()      # sharded DP update: a deferred fc-row all-gather (learner/dp_step.py)
        if not self._conv123:
            ops.conv_fwd(self.y2, Pb["w3"], P["b3"], 1, self.y3, Tb["w3"], T["b3"], 2 * B,
                         **self._lo(x_lo=self.y2_lo, w_lo=sp and Pl["w3"], w2_lo=sp and Tl["w3"], out_lo=self.y3_lo))
        self._wait_params()       # sharded DP update: the last update's fc rows (learner/dp_step.py)
        ops.fc_fwd(self.y3.reshape(n, 3136), Pb["wfc"], P["bfc"], self.h, Tb["wfc"], T["bfc"], 2 * B,
                   c2d=(Pb["w2"], Pl["w2"] if sp else None), defer_head=defer_head,
                   **self._lo(x_lo=sp and self.y3_lo.reshape(n, 3136), w_lo=sp and Pl["wfc"],
                              w2_lo=sp and Tl["wfc"], out_lo=self.h_lo))

    def _conv12_weights(self):
        P, T, Pb, Tb, Pl, Tl = self.P, self.T, self.Pb, self.Tb, self.Pl, self.Tl
        sp = self.split
        return ((P["w1"], P["b1"], T["w1"], T["b1"]),
                (Pb["w2"], Pl["w2"] if sp else None, P["b2"], Tb["w2"], Tl["w2"] if sp else None, T["b2"]))

    def _conv3_weights(self):
        """The fused conv3's weights (both sets): packed with the conv1 / conv2 fragments
        whenever those are (the fused launch may or may not run conv3, SW.conv123_max_images)."""
        P, T, Pb, Tb, Pl, Tl = self.P, self.T, self.Pb, self.Tb, self.Pl, self.Tl
        sp = self.split
        return (Pb["w3"], Pl["w3"] if sp else None, P["b3"], Tb["w3"], Tl["w3"] if sp else None, T["b3"])

    def _target_changed(self) -> None:
        """The target weights (t32 / tbf) changed: repack the fused forward's target
        fragments (fused conv1 -> conv2 forward)."""
        if self._c12:
            c1, c2 = self._conv12_weights()
            self.ops.conv12_pack(c1, c2, self.rt.obs_scale, sets=2, c3=self._conv3_weights())
            self._tgt_packed = True

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
        self.forward_all(defer_head=self._defer_fc_epilogue)
        self._mark("forward")
        isw = S["weights"] if self._isw else None
        sp = self.split
        ops.head(self.h[:2 * B], self.h[2 * B:], self._head_params(self.P), self._head_params(self.T), S["act"],
                 S["rew"], S["gam"], isw, rt.loss == "huber", rt.huber_delta, 1.0 / (B * self.world),
                 self.td_abs, self.loss_b, self.dH, self.dhead, zero=self.g_head_region,
                 isn=self._isn(), **self._lo(lo=sp and (self.h_lo[:2 * B], self.h_lo[2 * B:], self.dH_lo)))
        self._mark("head")
        prio = (self.replay, S["idx"], S["gen"], self.td_abs)
        if self._branched or self._dp:
            return           # the weight gradients: _seg2_branched / the DP step (dp_step.py)
        # fc wgrad + head wgrad + priority write-back: one launch on the HIP backend
        # (csrc/sumtree.hip fc_wgrad_head_prio_kernel)
        nrm = (self.norm_part, 0) if self._fuse_norm else None
        self._fc_slots = ops.fc_head_wgrad(self.dH, self.y3[:B], self.G["wfc"], self.G["bfc"], self.h,
                                           self.dhead, self.G, prio, norm=nrm,
                                           **self._lo(dh_lo=self.dH_lo, x_lo=sp and self.y3_lo[:B],
                                                      Hon_lo=self.h_lo))
        if self._comm_bf16:
            cut = self.layout.offsets["wfc"]
            self.gcomm[cut:].copy_(self.g32[cut:])
        self._mark("fc_wgrad")

    def _sample(self) -> None:
        """The sampler writes idx / IS weights / records and the frame-ring slots of
        S_t, S_{t+n} (twice: online and target rows) into the step's buffers."""
        self.replay.sample(self.B, out=self.S, nxt2=self.slots[2 * self.B:])
        self._sample_ver = self.replay.version

    def _seg2(self, after_first=None) -> None:
        """fc dgrad + conv backward (with DP, all of it overlaps the fc/heads bucket
        all-reduce): the dgrad chain, conv3/conv2 wgrad, conv1 wgrad last.
        ``after_first``: called once the first kernel (fc dgrad) is enqueued.  The
        single-rank branched step (SW.bwd_branches) runs :meth:`_seg2_branched`."""
        if self._branched:
            assert after_first is None
            return self._seg2_branched()
        B, rt, ops, G, Pb, Pl = self.B, self.rt, self.ops, self.G, self.Pb, self.Pl
        sp = self.split
        jobs = []    # split-K reductions of conv3 / conv2, finalised at the end
        ops.fc_dgrad(self.dH, self.y3[:B], Pb["wfc"], self.dY3,
                     **self._lo(dh_lo=self.dH_lo, w_lo=sp and Pl["wfc"], dx_lo=self.dY3_lo))
        if after_first is not None:
            after_first()
        ops.conv_wgrad(self.dY3, self.y2[:B], 3, 1, G["w3"], G["b3"], jobs=jobs,
                       **self._lo(dy_lo=self.dY3_lo, x_lo=sp and self.y2_lo[:B]))
        ops.conv_dgrad(self.dY3, Pb["w3"], 1, self.y2[:B], self.dY2,
                       **self._lo(dy_lo=self.dY3_lo, w_lo=sp and Pl["w3"], dx_lo=self.dY2_lo))
        ops.conv_wgrad(self.dY2, self.y1[:B], 4, 2, G["w2"], G["b2"], jobs=jobs,
                       **self._lo(dy_lo=self.dY2_lo, x_lo=sp and self.y1_lo[:B]))
        ops.conv_dgrad(self.dY2, Pb["w2"], 2, self.y1[:B], self.dY1,
                       **self._lo(dy_lo=self.dY2_lo, w_lo=sp and Pl["w2"], dx_lo=self.dY1_lo))
        jobs1 = []
        ops.conv1_wgrad_ring(self.dY1, self.replay.frames, self.slots[:B], self.frames, rt.obs_scale, G["w1"],
                             G["b1"], jobs=jobs1, **self._lo(dy_lo=self.dY1_lo))
        # two finalisations, as the branched step runs them (conv3 / conv2 + the head
        # region's norm partials, then conv1): the same norm-partial slots, so the two
        # schedules give bit-identical updates
        fuse = self._fuse_norm
        n1 = ops.finalize_grads(jobs, self.g_head_region if fuse else None,
                                dict(part=self.norm_part, slot0=self._fc_slots) if fuse else None)
        n2 = ops.finalize_grads(jobs1, None, dict(part=self.norm_part, slot0=n1) if fuse else None)
        self._npart = n2 if fuse else 0
        if self._comm_bf16:
            cut = self.layout.offsets["wfc"]
            self.gcomm[:cut].copy_(self.g32[:cut])
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
            if self._dp:
                self._dp_body()
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

    def _seg3(self, norm_slots: Optional[int] = None, segs=None, norm_prefix=None) -> None:
        """clip + centered RMSprop (+ bf16 hi / lo pack) with the next batch's draw.
        ``norm_slots``: the clip norm is the sum of ``norm_part[:norm_slots]`` (written by
        the gradient producers of the DP step) plus, with ``norm_prefix``, the squares of
        that gradient range (summed inside the launch).  ``segs``: the flat ranges to
        update (the sharded DP update, learner/dp_step.py)."""
        rt, ops = self.rt, self.ops
        if self._comm_bf16:
            self.g32.copy_(self.gcomm)
        # with pre-sampling the optimizer launch also draws step t+1's batch (every
        # read of this step's sample buffers is behind us)
        nxt = (self.replay, self.B, self.S, self.slots[2 * self.B:]) if self._presample else None
        ops.optimizer(self.p32, self.g32, self.rms_v, self.rms_m, self.pbf, rt.lr, rt.rms_decay, rt.rms_eps,
                      rt.grad_clip, rt.centered_rmsprop, self.partials, self.gnorm,
                      norm_total=(self.norm_part, self._npart) if self._fuse_norm else
                      ((self.norm_part, norm_slots) if norm_slots else None), sample=nxt,
                      wnorm=self._wnorm(), **self._lo(pb_lo=self.pbf_lo),
                      **({"frag_out": self._frag_out} if (self._frag_out is not None and nxt is not None) else {}),
                      **({"segs": segs} if segs is not None else {}),
                      **({"norm_prefix": norm_prefix} if norm_prefix is not None else {}))
        if self._presample:
            self._sample_ver = self.replay.version
        self._mark("optimizer")

    def _seg2_branched(self) -> None:
        """Backward with the weight gradients on a second stream (SW.bwd_branches): the
        step's critical path is the data-gradient chain (fc dgrad -> conv3 dgrad -> conv2
        dgrad -> conv1 wgrad); fc wgrad (+ head wgrad + priority write-back), conv3 wgrad
        and conv2 wgrad need only its intermediate dY and run beside it -- in the captured
        graph, a branch forked after the head and joined before the split-K finalisation.
        Each main-stream kernel is enqueued before the branch work that waits on it, so the
        chain stays the fork's first child (on the step's hardware queue)."""
        B, rt, ops, G, Pb, Pl, S = self.B, self.rt, self.ops, self.G, self.Pb, self.Pl, self.S
        sp = self.split
        main, side = torch.cuda.current_stream(self.device), self._wg_stream
        jobs = []
        prio = (self.replay, S["idx"], S["gen"], self.td_abs)
        nrm = (self.norm_part, 0) if self._fuse_norm else None

        def fc_wgrad():
            self._fc_slots = ops.fc_head_wgrad(self.dH, self.y3[:B], G["wfc"], G["bfc"], self.h, self.dhead, G,
                                               prio, norm=nrm,
                                               **self._lo(dh_lo=self.dH_lo, x_lo=sp and self.y3_lo[:B],
                                                          Hon_lo=self.h_lo))

        # auto: fp32-class at >= 256 rows, 2,681 / 2,679 vs 2,654 / 2,665 steps/s; bf16 and
        # 74 rows lose (4,264 / 4,214 vs 4,367 / 4,403; 6,077 vs 6,415),
        # profiles/r4_ab_fc_wgrad_main.txt
        fc_main = SW.fc_wgrad_main == "on" or (SW.fc_wgrad_main == "auto" and sp and B >= 256)
        if not fc_main:
            ev = torch.cuda.Event()
            ev.record(main)
        ops.fc_dgrad(self.dH, self.y3[:B], Pb["wfc"], self.dY3,
                     **self._lo(dh_lo=self.dH_lo, w_lo=sp and Pl["wfc"], dx_lo=self.dY3_lo))
        if fc_main:
            # fc dgrad and the fc weight gradient back to back on the main stream, each on
            # the whole chip; the branch forks after them (its first wait, conv3's wgrad)
            fc_wgrad()
        else:
            side.wait_event(ev)
            with torch.cuda.stream(side):
                fc_wgrad()
        # (conv3's weight gradient after conv1's on the main stream, where the chain has
        # slack at 512 rows: 2,674 / 2,668 vs 2,677 / 2,675 fp32, 4,271 / 4,312 vs 4,388 /
        # 4,489 bf16, 6,078 / 6,056 vs 6,478 / 6,437 at 74 rows -- the co-running kernels
        # stretch instead, profiles/r4_ab_wgrad3_main_rejected.txt)
        self._conv32_branched(main, side, jobs)
        fuse = self._fuse_norm
        jobs1 = []
        ops.conv1_wgrad_ring(self.dY1, self.replay.frames, self.slots[:B], self.frames, rt.obs_scale, G["w1"],
                             G["b1"], jobs=jobs1, **self._lo(dy_lo=self.dY1_lo))
        with torch.cuda.stream(side):
            # conv3 / conv2 split-K reductions (+ the head region's norm partials) on the
            # branch, beside conv1's weight gradient
            n_side = ops.finalize_grads(jobs, self.g_head_region if fuse else None,
                                        dict(part=self.norm_part, slot0=self._fc_slots) if fuse else None)
        n_main = ops.finalize_grads(jobs1, None, dict(part=self.norm_part, slot0=n_side) if fuse else None)
        main.wait_stream(side)
        self._npart = n_main
        self._mark("conv_backward")

    def _conv2_wgrad(self, jobs) -> None:
        B, sp = self.B, self.split
        self.ops.conv_wgrad(self.dY2, self.y1[:B], 4, 2, self.G["w2"], self.G["b2"], jobs=jobs,
                            **self._lo(dy_lo=self.dY2_lo, x_lo=sp and self.y1_lo[:B]))

    def _conv3_wgrad(self, jobs) -> None:
        B, sp = self.B, self.split
        self.ops.conv_wgrad(self.dY3, self.y2[:B], 3, 1, self.G["w3"], self.G["b3"], jobs=jobs,
                            **self._lo(dy_lo=self.dY3_lo, x_lo=sp and self.y2_lo[:B]))

    def _conv32_branched(self, main, side, jobs, wgrad2: bool = True) -> None:
        """Branched backward, middle part: conv3 / conv2 data gradients on the main stream,
        conv3 and (``wgrad2``) conv2 weight gradients on the branch, each after a wait for
        the data gradient it reads.  (One wait before both weight gradients -- one graph
        edge fewer -- measured 5,937 / 6,062 vs 6,240 / 6,437 steps/s at 74 rows and
        neutral at 512, profiles/r4_ab_bwd_one_wait_rejected.txt.)"""
        B, ops, G, Pb, Pl, sp = self.B, self.ops, self.G, self.Pb, self.Pl, self.split
        ev3 = torch.cuda.Event()
        ev3.record(main)
        ops.conv_dgrad(self.dY3, Pb["w3"], 1, self.y2[:B], self.dY2,
                       **self._lo(dy_lo=self.dY3_lo, w_lo=sp and Pl["w3"], dx_lo=self.dY2_lo))
        side.wait_event(ev3)
        with torch.cuda.stream(side):
            self._conv3_wgrad(jobs)
        ev2 = torch.cuda.Event()
        ev2.record(main)
        ops.conv_dgrad(self.dY2, Pb["w2"], 2, self.y1[:B], self.dY1,
                       **self._lo(dy_lo=self.dY2_lo, w_lo=sp and Pl["w2"], dx_lo=self.dY1_lo))
        side.wait_event(ev2)
        if wgrad2:
            with torch.cuda.stream(side):
                self._conv2_wgrad(jobs)

    def _step_body(self) -> None:
        self._seg1()
        self._seg2()
        self._seg3()

    def _body(self) -> None:
        if self._dp:
            self._dp_body()
        else:
            self._step_body()
        if not self._defer_params:
            self._wait_params()

    # called after update i of the multi-step graph's capture (its work is captured into
    # the graph): tests record every update's state and next batch from inside the graph
    _step_hook = None

    # set when the DP step's graph capture (or its first replay) failed on some rank: every
    # rank then runs the eager DP step (prepare_graphs)
    graph_fallback = None
    _inject_capture_failure = False    # tests: fail the one-update capture after its body

    def _graphs_enabled(self) -> bool:
        return (bool(self.rt.use_graphs) and self.device.type == "cuda" and (not self._dp or self._dp_graphs)
                and self.graph_fallback is None)

    def step(self) -> None:
        """One learner update (asynchronous on the current stream)."""
        graphs = self._graphs_enabled()
        if graphs and self._graphs is None:
            self.prepare_graphs(multi=False)
            graphs = self._graphs_enabled()
        if graphs and self._presample and self._sample_ver != self.replay.version:
            self._sample()     # host-side replay mutation since the pre-sample: redraw
        if graphs:
            self._graphs.replay()
        else:
            self._body()
        self.num_q_updates += 1
        L = self.cfg.Learner
        if self.num_q_updates % L.q_target_sync_freq == 0:
            self.sync_target()

    def steps(self, n: int) -> None:
        """``n`` learner updates.  With HIP graphs, chunks of ``Runtime.graph_steps``
        updates replay ONE graph holding that many steps (each graph launch costs
        ~9 us of idle GPU at its boundary); chunks never straddle a target-network
        sync.  Same updates as ``n`` calls of :meth:`step`."""
        k = int(self.rt.graph_steps)
        if k <= 1 or not self._graphs_enabled():
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
            self.prepare_graphs(multi=True)
            if not self._graphs_enabled():       # (the DP step fell back to eager)
                for _ in range(n):
                    self.step()
                return
            if self._presample and self._sample_ver != self.replay.version:
                self._sample()
            self._multi.replay()
            self.num_q_updates += k
            n -= k
            if self.num_q_updates % f == 0:
                self.sync_target()

    def prepare_graphs(self, multi: bool = True) -> int:
        """Capture every graph :meth:`step` / :meth:`steps` will replay (the one-update
        graph and, with ``multi``, the ``Runtime.graph_steps`` graph) now, so no
        capture lands in a timed region.  Learner state is unchanged.  Returns
        ``graph_captures``.

        Data parallel: the DP step's graphs hold RCCL collectives, and three phases
        differ in what a failure leaves behind:

        * the eager warm-up (real collectives) and the first replay of fresh graphs
          (real collectives) are not recoverable in process -- a rank that raises there
          has skipped collectives its peers are blocked in -- so an error propagates and
          the caller's watchdog (bench.py's ``PhaseWatchdog``, gpu_loop's chunk phase)
          aborts the communicator and exits non-zero;
        * the capture itself enqueues nothing: if it raises on ANY rank (agreed by a host
          all-reduce that every rank reaches), every rank drops its graphs and runs the
          eager DP step (``graph_fallback``).
        A NATIVE crash inside capture is caught before the parent process ever touches
        the GPU, by the out-of-process probe (``runtime/capture_probe.py``)."""
        if not self._graphs_enabled():
            return self.graph_captures
        k = int(self.rt.graph_steps)
        if not (self._graphs is None or (multi and k > 1 and self._multi is None) or not self._graphs_warm):
            return self.graph_captures
        if self._graphs is None:
            self._warmup_eager()
        if not self._dp:
            self._capture_graphs(multi)
        else:
            snap = self._snapshot()
            err = None
            try:
                self._capture_graphs(multi)
            except Exception as e:      # the capture of the DP step failed here
                err = e
            ok = err is None
            if self.comm is not None and getattr(self.comm, "active", False):
                ok = self.comm.allreduce_scalar(1.0 if ok else 0.0, "min") > 0.5
            if not ok:
                self._eager_fallback(err, snap)
                return self.graph_captures
        self._warm_graphs()
        return self.graph_captures

    def _eager_fallback(self, err, snap) -> None:
        import sys
        try:
            torch.cuda.synchronize(self.device)
        except Exception:  # pragma: no cover - a sticky error is reported below anyway
            pass
        self._graphs = self._multi = None
        self._params_pending, self._defer_params, self._gather_due = None, False, None
        self._restore(snap)
        if self._presample:
            self._sample()
        torch.cuda.synchronize(self.device)
        self.graph_fallback = repr(err) if err is not None else "a peer rank's DP graph capture failed"
        r = self.comm.rank if self.comm is not None else 0
        sys.stderr.write(f"[rank {r}] DP step graphs unavailable ({self.graph_fallback}); "
                         f"running the eager DP step\n")
        sys.stderr.flush()

    def _capture_graphs(self, multi: bool) -> None:
        """Capture the one-update graph (if missing) and, with ``multi``, the
        ``graph_steps`` graph.  Capture records without executing: state is unchanged.
        Thread-local capture mode: the torch.distributed RCCL watchdog thread queries its
        events at any time (in global mode one such query inside a capture invalidated it
        and aborted the process: hipErrorStreamCaptureUnsupported on the watchdog)."""
        if self._graphs is None:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                self._body()
                if self._inject_capture_failure:
                    raise RuntimeError("injected DP graph capture failure (test)")
            self._graphs = g
            self.graph_captures += 1
            self._graphs_warm = False
        k = int(self.rt.graph_steps)
        if multi and k > 1 and self._multi is None:
            g = torch.cuda.CUDAGraph()
            torch.cuda.synchronize(self.device)
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                try:
                    for i in range(k):
                        # (sharded DP update: the fc-row all-gather of every update but the
                        # last is joined by the next update's fc forward)
                        self._defer_params = i + 1 < k and self._step_hook is None
                        self._body()
                        if self._step_hook is not None:
                            self._step_hook(i)      # captured too (tests: per-update state copies)
                finally:
                    self._defer_params = False
                    self._wait_params()
            self._multi = g
            self.graph_captures += 1
            self._graphs_warm = False

    def _warm_graphs(self) -> None:
        """The first launch of a fresh graph uploads it (~ms): replay each graph once and
        restore the learner / replay state, so the first timed launch is warm."""
        if self._graphs_warm:
            return
        snap = self._snapshot()
        if self._presample and self._sample_ver != self.replay.version:
            self._sample()
        for gr in (self._graphs, self._multi):
            if gr is not None:
                gr.replay()
        torch.cuda.synchronize(self.device)
        self._restore(snap)
        if self._presample:
            self._sample()     # the pre-drawn batch of the restored state (same draw)
        torch.cuda.synchronize(self.device)
        self._graphs_warm = True

    def rewarm(self, replays: int) -> None:
        """Untimed, state-preserving GPU warm-up: replay the multi-step graph ``replays``
        times from a snapshot, then restore the learner / replay state (bench.py runs it
        right before its timed window so the clocks there are those of a busy GPU, as
        after a long warm-up; no update is kept)."""
        if replays <= 0 or not self._graphs_enabled():
            return
        self.prepare_graphs(multi=True)
        gr = self._multi if self._multi is not None else self._graphs
        snap = self._snapshot()
        if self._presample and self._sample_ver != self.replay.version:
            self._sample()
        for _ in range(replays):
            gr.replay()
        torch.cuda.synchronize(self.device)
        self._restore(snap)
        if self._presample:
            self._sample()
        torch.cuda.synchronize(self.device)

    def _warmup_eager(self) -> None:
        """Two eager updates on a side stream (allocator pools, workspaces, the
        communicator), then the state restored: the graphs start from the same state."""
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        snap = self._snapshot()
        with torch.cuda.stream(s):
            for _ in range(2):
                self._body()
        torch.cuda.current_stream(self.device).wait_stream(s)
        self._restore(snap)
        if self._presample:    # the graphs start from a drawn batch (their seg1 holds no sample)
            self._sample()
        torch.cuda.synchronize(self.device)

    def check_replicas(self) -> bool:
        """Data-parallel replicas must stay bit-identical (same all-reduced gradient,
        deterministic optimizer).  Compare a checksum of the fp32 master weights
        across ranks; on a mismatch (silent data corruption, a rank that skipped an
        update) re-broadcast rank 0's weights and optimizer state.  A collective:
        every rank calls it at the same step.  Returns True if the replicas agreed."""
        if not self._dp or self.world <= 1 or getattr(self.comm, "emulated", False):
            return True
        import torch.distributed as dist
        self.materialize()
        w = torch.arange(1, 65, device=self.device, dtype=torch.float64)
        p = self.p32.double()
        n = p.numel() // 64 * 64
        sig = torch.stack([p.sum(), (p[:n].view(-1, 64) * w).sum(), self.rms_v.double().sum()])
        lo, hi = sig.clone(), sig.clone()
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        if torch.equal(lo, hi):
            return True
        for t in (self.p32, self.rms_v, self.rms_m, self.t32):
            dist.broadcast(t, src=0)
        self._refresh_bf16()
        split_into(self.t32, self.tbf, self.tbf_lo)
        self._target_changed()
        return False

    def refresh_replay_stats(self) -> bool:
        """Re-gather the shard statistics (after host-side inserts / eviction; a
        collective: every rank calls it at the same point), and grow the per-rank rows if
        a shard's share of the mass outgrew them (:meth:`_fit_rows`).  Returns True when
        the rows grew: the step graphs were dropped, and the caller recaptures them
        (:meth:`prepare_graphs`) while no other thread launches GPU work."""
        if self._dp:
            self.replay.gather_shard_stats(coll=self.coll)
            return bool(self._fit_rows())
        return False

    def graph_matches_eager(self) -> Optional[bool]:
        """One update replayed from the captured one-update graph against the same update
        run eagerly from the same snapshot: parameters (fp32 + bf16 operands) and RMSprop
        state bit-identical?  The state is restored afterwards.  A collective with DP
        (every rank calls it; the answer is agreed by a host all-reduce).  None when the
        graphs are not in use."""
        if not self._graphs_enabled() or self._graphs is None:
            return None
        self._wait_params()
        torch.cuda.synchronize(self.device)
        snap = self._snapshot()
        state = (self.p32, self._pbf_all, self.rms_v, self.rms_m)
        if self._presample and self._sample_ver != self.replay.version:
            self._sample()
        self._graphs.replay()
        torch.cuda.synchronize(self.device)
        g = [t.clone() for t in state]
        self._restore(snap)
        if self._presample:
            self._sample()
        self._body()
        self._wait_params()
        torch.cuda.synchronize(self.device)
        same = all(torch.equal(a, b) for a, b in zip(g, state))
        self._restore(snap)
        if self._presample:
            self._sample()
        torch.cuda.synchronize(self.device)
        if self.comm is not None and getattr(self.comm, "active", False):
            same = self.comm.allreduce_scalar(1.0 if same else 0.0, "min") > 0.5
        return bool(same)

    def _snapshot(self):
        rp = self.replay
        return [t.clone() for t in (self.p32, self._pbf_all, self.rms_v, self.rms_m, rp.leaf, rp.nodes,
                                    rp.min_bits, rp.ctr)] + ([rp.shard_stats.clone()] if rp.sharded else [])

    def _restore(self, snap) -> None:
        rp = self.replay
        dst = [self.p32, self._pbf_all, self.rms_v, self.rms_m, rp.leaf, rp.nodes, rp.min_bits, rp.ctr]
        if rp.sharded:
            dst.append(rp.shard_stats)
        for t, src in zip(dst, snap):
            t.copy_(src)
        self._online_changed()

    def _refresh_bf16(self) -> None:
        """bf16 compute copy (and its lo plane) from the fp32 master weights."""
        split_into(self.p32, self.pbf, self.pbf_lo)
        self._online_changed()

    def sync_target(self) -> None:
        self.t32.copy_(self.p32)
        self._tbf_all.copy_(self._pbf_all)
        self._target_changed()

    # ------------------------------------------------------------ metrics
    def last_metrics(self) -> Dict[str, float]:
        return self._is_metrics()

    def q_values(self, frames_u8: torch.Tensor) -> torch.Tensor:
        """Greedy-evaluation helper: q for a (N, C, 84, 84) uint8 batch (fp32 module,
        scaled by ``Runtime.obs_scale`` as the learner's conv1 is)."""
        sd = self.reference_state_dict()
        net = DuellingDQN((self.C, 84, 84), self.A, conv1_channels=self.c1, obs_scale=self.rt.obs_scale)
        net = net.to(self.device)
        net.load_state_dict(sd)
        with torch.no_grad():
            return net(frames_u8.to(self.device))[2]

    # ------------------------------------------------------------- params
    def reference_state_dict(self):
        return flat_to_reference_state(self.P, self.c1)

    def load_reference_state_dict(self, sd) -> None:
        reference_state_to_flat(sd, self.P)
        self._refresh_bf16()

    def save(self, path: str, extra: Optional[Dict[str, Any]] = None) -> None:
        self._check_materialized()
        tgt = flat_to_reference_state(self.T, self.c1)
        save_checkpoint(path, self.reference_state_dict(), Q_target_state=tgt,
                        optimizer_state=pack_flat_state(layout_segments(self.layout), rms_v=self.rms_v, rms_m=self.rms_m),
                        num_q_updates=self.num_q_updates, config=self.cfg.to_dict(),
                        rng={"replay_ctr": int(self.replay.ctr.item()), "replay_seed": int(self.replay.seed)},
                        **(extra or {}))

    def load(self, path: str) -> bool:
        ck = load_checkpoint(path)
        if ck is None:
            return False
        if adopt_obs_scale(ck, self.rt):
            self._graphs = self._multi = None    # the input scale is a kernel argument: recapture
            self._setup_frag_out()               # (and folded into the conv1 operands)
        self.load_reference_state_dict(ck["Q_state"])
        if "Q_target_state" in ck:
            reference_state_to_flat(ck["Q_target_state"], self.T)
            split_into(self.t32, self.tbf, self.tbf_lo)
            self._target_changed()
        else:
            self.sync_target()
        opt = ck.get("optimizer_state")
        unpack_flat_state(opt, layout_segments(self.layout), untagged_network=checkpoint_network(ck),
                          network=self.cfg.network, rms_v=self.rms_v, rms_m=self.rms_m)
        self.num_q_updates = int(ck.get("num_q_updates", 0))
        rng = ck.get("rng")
        if isinstance(rng, dict) and "replay_ctr" in rng:
            self.replay.ctr.fill_(int(rng["replay_ctr"]))
        self._last_ckpt = ck
        return True
