"""MI355X learner for the IMPALA-deep ResNet dueling Q-net (BASELINE.json config 5).

Same GPU-resident step as ``fused_learner.FusedNatureLearner`` (sample ->
3-way forward -> fused DDQN head -> backward -> [DP all-reduce] -> clip +
centered RMSprop -> priority write-back), with the trunk on the small-channel
conv kernels of ``csrc/impala.hip``:

  per stack s (channels 16 / 32 / 32, input 84 / 42 / 21 px):
    p  = maxpool3x3s2(conv3x3(x))  one kernel (+ argmax codes for the backward);
                                 stack 1 reads the uint8 frame ring directly
    ya = conv(relu(p));  ra = p  + conv(relu(ya))   one kernel per block (ya in
    yb = conv(relu(ra)); o  = ra + conv(relu(yb))   LDS; kept in HBM for B rows)
  feat = relu(o_3) (planar, 3872 + 32 zero pad = 3904 per row)
  h = relu(feat @ Wfc^T + b)   (value | advantage streams, 2 x 256)

Backward per res block: the data gradient is the same correlation kernel with
transposed + flipped weight fragments and a (producer > 0) mask epilogue, the
skip gradient added in the same epilogue; weight gradients are image-tiled
split-K partials finalised in one pass per four convs.

Parameters live in one flat fp32 buffer in the kernels' layouts (conv OIHW,
fc columns in planar order); ``state_dict()`` converts to the
``ImpalaDuellingDQN`` module's keys.  Rows [0,B) = S_t and [B,2B) = S_{t+n}
use the online weights, rows [2B,3B) = S_{t+n} the target weights, switched
inside each launch.  Reference parity: ``learner.py:29-80`` semantics with the
defects fixed, exactly as the NatureCNN learner.
"""
from __future__ import annotations

import contextlib
from collections import OrderedDict
from typing import Dict, List, Optional

import torch

from ..config import ApexConfig
from ..models.dueling import ImpalaDuellingDQN
from ..models.flat_params import FlatLayout
from ..ops.fused_ops import HipBackend, TorchBackend, split_into
from ..ops.impala import ConvSpec, HipImpalaOps, TorchImpalaOps, frag_elems
from ..utils.checkpoint import (adopt_obs_scale, layout_segments, load_checkpoint, pack_flat_state,
                                save_checkpoint, unpack_flat_state, checkpoint_network)
from ..ops.switches import SW
from .fused_learner import _enable_sharding, dp_layout
from .is_norm import IsNormMixin

CH = (16, 32, 32)
HIDDEN = 256
FEAT = 2 * 11 * 11 * 16          # 3872
FEAT_LD = 3904                   # 61 x 64: the fc GEMM's K


def _stack_dims():
    out, cin, hw = [], 4, 84
    for c in CH:
        out.append((cin, c, hw, (hw + 1) // 2))
        cin, hw = c, (hw + 1) // 2
    return out   # (cin, cout, input hw, pooled hw)


def fc_column_perm(device=None) -> torch.Tensor:
    """torch flatten column j = c*121 + h*11 + w  ->  planar column of (c, h, w)."""
    c = torch.arange(32).view(32, 1, 1)
    h = torch.arange(11).view(1, 11, 1)
    w = torch.arange(11).view(1, 1, 11)
    k = ((c // 16) * 11 + h) * 176 + w * 16 + (c % 16)
    return k.reshape(-1).to(device)


class FusedImpalaLearner(IsNormMixin):
    kind = "impala"

    def __init__(self, cfg: ApexConfig, device, replay, comm=None, backend: Optional[str] = None,
                 batch_size: Optional[int] = None):
        self.cfg = cfg
        self.rt = cfg.Runtime
        self.device = torch.device(device)
        self.replay = replay
        self.comm = comm
        self.world, _, self.B, self.mcap = dp_layout(cfg, comm, batch_size, allow_force=False)
        self.C = cfg.frame_stack
        if self.C != 4 or tuple(cfg.env_conf.state_shape[1:]) != (84, 84):
            raise ValueError("the IMPALA kernels are built for 4 x 84 x 84 inputs")
        self.A = int(cfg.env_conf.action_dim)
        if backend is None:
            backend = "hip" if (self.device.type == "cuda" and self.rt.use_hip_kernels) else "torch"
        on_gpu = backend == "hip"
        if self.rt.dtype not in ("fp32", "bf16"):
            raise ValueError("Runtime.dtype must be fp32 or bf16")
        bf16_torch = self.device.type == "cuda" and self.rt.dtype == "bf16"
        self.ops = HipBackend(native_conv=True) if on_gpu else TorchBackend(
            torch.bfloat16 if bf16_torch else torch.float32)
        self.iops = HipImpalaOps() if on_gpu else TorchImpalaOps()
        # split mode (Runtime.dtype fp32 on the HIP kernels): fp32 trunk activations and
        # gradients, bf16 hi + lo weight fragments, three MFMAs per product
        # (csrc/impala_split.hip); the fc / heads run the NatureCNN split kernels on the
        # bf16 hi / lo planes of feat and h.  The torch backend is the fp32 oracle (bf16
        # on the GPU when asked for).
        self.split = on_gpu and self.rt.dtype == "fp32"
        if on_gpu:
            self.act_dtype = torch.float32 if self.split else torch.bfloat16
            self.op_dtype = torch.bfloat16                  # GEMM operand planes
        else:
            self.act_dtype = self.op_dtype = torch.bfloat16 if bf16_torch else torch.float32
        d = self.device

        # ---- flat parameter layout (conv trunk first: the DP fc/heads bucket starts at wfc)
        self.specs: List[List[ConvSpec]] = []
        segs = []
        for s, (cin, cout, hw, php) in enumerate(_stack_dims()):
            convs = [ConvSpec(f"s{s}c0", max(cin, 16), cout, cin, hw, hw)]
            for r in range(2):
                for k in range(2):
                    convs.append(ConvSpec(f"s{s}r{r}c{k}", cout, cout, cout, php, php))
            for cs in convs:
                segs += [(cs.name + ".w", (cs.cout, cs.cin_real, 3, 3)), (cs.name + ".b", (cs.cout,))]
            self.specs.append(convs)
        segs += [("wfc", (2 * HIDDEN, FEAT_LD)), ("bfc", (2 * HIDDEN,)), ("wv", (HIDDEN,)), ("bv", (1,)),
                 ("wa", (self.A, HIDDEN)), ("ba", (self.A,))]
        self.layout = FlatLayout(segs)
        n = self.layout.numel
        self.p32 = torch.zeros(n, dtype=torch.float32, device=d)
        # bf16 compute copies [hi | lo] of the online / target parameters (lo: split mode)
        nb = 2 * n if self.split else n
        self._pbf_all = torch.zeros(nb, dtype=self.op_dtype, device=d)
        self._tbf_all = torch.zeros(nb, dtype=self.op_dtype, device=d)
        self.pbf, self.tbf = self._pbf_all[:n], self._tbf_all[:n]
        self.pbf_lo = self._pbf_all[n:] if self.split else None
        self.tbf_lo = self._tbf_all[n:] if self.split else None
        self.g32 = torch.zeros(n, dtype=torch.float32, device=d)
        self.rms_v = torch.zeros(n, dtype=torch.float32, device=d)
        self.rms_m = torch.zeros(n, dtype=torch.float32, device=d)
        self.t32 = torch.zeros(n, dtype=torch.float32, device=d)
        self.P = self.layout.views(self.p32)
        self.Pb = self.layout.views(self.pbf)
        self.G = self.layout.views(self.g32)
        self.T = self.layout.views(self.t32)
        self.Tb = self.layout.views(self.tbf)
        self.Pl = self.layout.views(self.pbf_lo) if self.split else None
        self.Tl = self.layout.views(self.tbf_lo) if self.split else None
        self._perm = fc_column_perm(d)
        for convs in self.specs:
            for cs in convs:
                cs.w, cs.b, cs.wb = self.P[cs.name + ".w"], self.P[cs.name + ".b"], self.Pb[cs.name + ".w"]
                cs.extra["w_tgt"], cs.extra["b_tgt"] = self.Tb[cs.name + ".w"], self.T[cs.name + ".b"]
                if on_gpu:
                    cs.frag = torch.zeros(frag_elems(cs.cin, cs.cout), dtype=torch.bfloat16, device=d)
                    cs.fragT = torch.zeros(frag_elems(cs.cout, cs.cin), dtype=torch.bfloat16, device=d)
                    cs.frag_tgt = torch.zeros_like(cs.frag)
                if self.split:
                    cs.extra["wl"], cs.extra["w_tgt_lo"] = self.Pl[cs.name + ".w"], self.Tl[cs.name + ".w"]
                    cs.frag_lo, cs.fragT_lo = torch.zeros_like(cs.frag), torch.zeros_like(cs.fragT)
                    cs.frag_tgt_lo = torch.zeros_like(cs.frag)
        init = ImpalaDuellingDQN((self.C, 84, 84), self.A, channels=CH, hidden=HIDDEN)
        self.load_module_state(init.state_dict(), self.P)
        if comm is not None and comm.world_size > 1:
            comm.broadcast_flat(self.p32)
        self._refresh_bf16()
        self.num_q_updates = 0
        self._alloc(self.B)
        self.sync_target()
        self._graphs = None
        self._multi = None      # one rank: Runtime.graph_steps updates in one graph (steps())
        self.graph_captures = 0
        # one stream by default (see fused_learner: cross-stream edges in the HIP graph
        # cost more than the overlap); the head kernel writes the priorities back and
        # the optimizer launch draws the next batch (Runtime.presample)
        self._side = None
        # (the 15 conv weight gradients on a second stream beside the data-gradient chain
        # measured no gain -- 392.5 / 393.9 vs 395.6 / 395.4 steps/s fp32,
        # profiles/r4_ab_impala_bwd_branches.txt -- and were removed: the IMPALA kernels
        # fill the chip on their own)
        self._presample = bool(self.rt.presample)
        self._sample_ver = None
        self.partials = torch.zeros(1024, dtype=torch.float64, device=d)
        self.gnorm = torch.zeros(1, dtype=torch.float32, device=d)
        # DP: one global prioritized replay over the rank shards (see fused_learner)
        self._isw = bool(self.rt.use_is_weights) or self.world > 1
        self._dp = self.world > 1
        self._init_is_norm()
        if self.world > 1:
            _enable_sharding(replay, comm, self.rt, self.mcap)
            replay.gather_shard_stats()
        ls = cfg.Learner.load_saved_state
        if ls:
            self.load(ls)

    # ------------------------------------------------------------- buffers
    def _alloc(self, B: int) -> None:
        d, ad = self.device, self.act_dtype
        N3 = 3 * B
        self.S = self.replay.alloc_sample_buffers(B)
        self.slots = torch.zeros(N3, self.C, dtype=torch.int32, device=d)
        self.S["obs"] = self.slots[:B]
        self.S["nxt"] = self.slots[B:2 * B]
        self.fw, self.bw = [], []
        od = self.op_dtype
        # fc operand rows (pad columns stay 0); split mode: bf16 hi + lo planes written by
        # the last residual block, and the fc data gradient's planes merged to fp32
        self.feat = torch.zeros(N3, FEAT_LD, dtype=od if self.split else ad, device=d)
        self.feat_lo = torch.zeros(N3, FEAT_LD, dtype=od, device=d) if self.split else None
        self.dfeat = torch.zeros(B, FEAT_LD, dtype=od if self.split else ad, device=d)
        self.dfeat_lo = torch.zeros(B, FEAT_LD, dtype=od, device=d) if self.split else None
        self.dfeat32 = torch.zeros(B, FEAT_LD, dtype=torch.float32, device=d) if self.split else self.dfeat
        for s, (cin, cout, hw, php) in enumerate(_stack_dims()):
            P = cout // 16
            t = lambda n, h: torch.zeros(n, P, h, h, 16, dtype=ad, device=d)  # noqa: E731
            f = dict(p=t(N3, php), ya=t(N3, php), ra=t(N3, php), yb=t(N3, php),
                     amax=torch.zeros(N3, P, php, php, 16, dtype=torch.uint8, device=d))
            f["o"] = (self.feat[:, :FEAT].view(N3, P, php, php, 16) if s == 2 else t(N3, php))
            if s == 2 and self.split:
                f["o_lo"] = self.feat_lo[:, :FEAT].view(N3, P, php, php, 16)
            self.fw.append(f)
            b = dict(d_yb=t(B, php), d_ra=t(B, php), d_ya=t(B, php), d_p=t(B, php), d_c0=t(B, hw))
            if s < 2:
                b["d_o"] = t(B, php)    # gradient of this stack's output (the next stack's conv0 dgrad)
            self.bw.append(b)
        self.h = torch.zeros(N3, 2 * HIDDEN, dtype=od, device=d)
        self.dH = torch.zeros(B, 2 * HIDDEN, dtype=od, device=d)
        self.h_lo = torch.zeros(N3, 2 * HIDDEN, dtype=od, device=d) if self.split else None
        self.dH_lo = torch.zeros(B, 2 * HIDDEN, dtype=od, device=d) if self.split else None
        self.dhead = torch.zeros(B, self.A + 1, dtype=torch.float32, device=d)
        self.td_abs = torch.zeros(B, dtype=torch.float32, device=d)
        self.loss_b = torch.zeros(B, dtype=torch.float32, device=d)
        o0 = self.layout.offsets["wv"]
        o1 = self.layout.offsets["ba"] + self.A
        self.g_head_region = self.g32[o0:o1]

    # ------------------------------------------------------ weight packing
    def _pack_online(self) -> None:
        jobs = []
        for convs in self.specs:
            for cs in convs:
                planes = [(cs.wb, cs.frag, cs.fragT)]
                if self.split:
                    planes.append((cs.extra["wl"], cs.frag_lo, cs.fragT_lo))
                for w, f, fT in planes:
                    jobs.append((w, f, cs.cin, cs.cout, cs.cin_real, self._fwd_kind(cs)))
                    if cs.cin_real == cs.cin:   # the ring conv needs no data gradient
                        jobs.append((w, fT, cs.cin, cs.cout, cs.cin_real, 1))
        self.iops.pack(jobs)

    @staticmethod
    def _fwd_kind(cs: ConvSpec) -> int:
        return 2 if cs.cin_real < cs.cin else 0     # 4-frame ring conv: tap-pair fragments

    def _pack_target(self) -> None:
        jobs = []
        for convs in self.specs:
            for cs in convs:
                jobs.append((cs.extra["w_tgt"], cs.frag_tgt, cs.cin, cs.cout, cs.cin_real, self._fwd_kind(cs)))
                if self.split:
                    jobs.append((cs.extra["w_tgt_lo"], cs.frag_tgt_lo, cs.cin, cs.cout, cs.cin_real,
                                 self._fwd_kind(cs)))
        self.iops.pack(jobs)

    # ------------------------------------------------------------ forward
    def forward_all(self) -> None:
        """Online net on rows [0,2B), target net on rows [2B,3B)."""
        io, B, rt = self.iops, self.B, self.rt
        x = None
        for s, convs in enumerate(self.specs):
            f = self.fw[s]
            c0, r0a, r0b, r1a, r1b = convs
            tg = lambda cs: dict(second=cs.extra["b_tgt"], n_switch=2 * B)  # noqa: E731
            if s == 0:   # conv + max pool in one kernel, straight from the uint8 frame ring
                io.conv_pool(None, c0, f["p"], f["amax"], ring=self.replay.frames, slots=self.slots,
                             scale=rt.obs_scale, amax_rows=B, **tg(c0))
            else:
                io.conv_pool(x, c0, f["p"], f["amax"], amax_rows=B, **tg(c0))
            # residual blocks: one kernel each; the mid activations are kept for the
            # B training rows only (the backward's ReLU masks / weight-gradient inputs)
            io.resblock(f["p"], r0a, r0b, f["ra"], ysave=f["ya"], n_save=B, target=True, n_switch=2 * B)
            io.resblock(f["ra"], r1a, r1b, f["o"], ysave=f["yb"], n_save=B, target=True, n_switch=2 * B,
                        relu_out=(s == 2), **self._lo(out_lo=f.get("o_lo")))
            x = f["o"]
        self.ops.fc_fwd(self.feat, self.Pb["wfc"], self.P["bfc"], self.h, self.Tb["wfc"], self.T["bfc"], 2 * B,
                        **self._lo(x_lo=self.feat_lo, w_lo=self.Pl and self.Pl["wfc"],
                                   w2_lo=self.Tl and self.Tl["wfc"], out_lo=self.h_lo))

    def _lo(self, **kw):
        """Split-mode keyword arguments of an op (empty with bf16 operands)."""
        return kw if self.split else {}

    def _refresh_bf16(self) -> None:
        """bf16 compute copy (and its lo plane) from the fp32 master weights."""
        split_into(self.p32, self.pbf, self.pbf_lo)

    # ------------------------------------------------- actor-side inference
    def actor_param_set(self) -> Dict:
        """A private parameter slot for an actor group (fp32 + bf16 copies and, on
        the HIP path, packed fragments); refreshed by ``refresh_param_set``."""
        import dataclasses
        n = self.layout.numel
        p32, pall = self.p32.clone(), self._pbf_all.clone()
        V, Vb = self.layout.views(p32), self.layout.views(pall[:n])
        Vl = self.layout.views(pall[n:]) if self.split else None
        specs = []
        for convs in self.specs:
            row = []
            for cs in convs:
                c2 = dataclasses.replace(cs, w=V[cs.name + ".w"], b=V[cs.name + ".b"], wb=Vb[cs.name + ".w"],
                                         extra=dict(cs.extra))
                if cs.frag is not None:
                    c2.frag = torch.zeros_like(cs.frag)
                    c2.fragT = c2.frag_tgt = c2.fragT_lo = c2.frag_tgt_lo = None
                if self.split:
                    c2.extra["wl"] = Vl[cs.name + ".w"]
                    c2.frag_lo = torch.zeros_like(cs.frag_lo)
                row.append(c2)
            specs.append(row)
        ps = dict(p32=p32, pbf=pall, V=V, Vb=Vb, Vl=Vl, specs=specs)
        self.refresh_param_set(ps)
        return ps

    def refresh_param_set(self, ps: Dict) -> None:
        ps["p32"].copy_(self.p32)
        ps["pbf"].copy_(self._pbf_all)
        jobs = []
        for row in ps["specs"]:
            for cs in row:
                jobs.append((cs.wb, cs.frag, cs.cin, cs.cout, cs.cin_real, self._fwd_kind(cs)))
                if self.split:
                    jobs.append((cs.extra["wl"], cs.frag_lo, cs.cin, cs.cout, cs.cin_real, self._fwd_kind(cs)))
        self.iops.pack(jobs)

    def alloc_trunk(self, E: int) -> Dict:
        d, ad, od = self.device, self.act_dtype, self.op_dtype
        sp = self.split
        bufs = dict(stacks=[], feat=torch.zeros(E, FEAT_LD, dtype=od if sp else ad, device=d),
                    h=torch.zeros(E, 2 * HIDDEN, dtype=od, device=d),
                    feat_lo=torch.zeros(E, FEAT_LD, dtype=od, device=d) if sp else None,
                    h_lo=torch.zeros(E, 2 * HIDDEN, dtype=od, device=d) if sp else None)
        for s, (cin, cout, hw, php) in enumerate(_stack_dims()):
            P = cout // 16
            t = lambda: torch.zeros(E, P, php, php, 16, dtype=ad, device=d)  # noqa: E731
            st = dict(p=t(), ya=t(), ra=t(), yb=t())
            st["o"] = bufs["feat"][:, :FEAT].view(E, P, php, php, 16) if s == 2 else t()
            if s == 2 and sp:
                st["o_lo"] = bufs["feat_lo"][:, :FEAT].view(E, P, php, php, 16)
            bufs["stacks"].append(st)
        return bufs

    def trunk_forward(self, slots: torch.Tensor, ps: Dict, bufs: Dict) -> torch.Tensor:
        """Stream activations h (E, 512) of the frame stacks at ``slots`` with the
        parameter slot ``ps`` (actor inference: same kernels, no target rows)."""
        io, x = self.iops, None
        for s, convs in enumerate(ps["specs"]):
            f = bufs["stacks"][s]
            c0, r0a, r0b, r1a, r1b = convs
            if s == 0:
                io.conv_pool(None, c0, f["p"], None, ring=self.replay.frames, slots=slots, scale=self.rt.obs_scale)
            else:
                io.conv_pool(x, c0, f["p"], None)
            io.resblock(f["p"], r0a, r0b, f["ra"])
            io.resblock(f["ra"], r1a, r1b, f["o"], relu_out=(s == 2), **self._lo(out_lo=f.get("o_lo")))
            x = f["o"]
        self.ops.fc_fwd(bufs["feat"], ps["Vb"]["wfc"], ps["V"]["bfc"], bufs["h"],
                        **self._lo(x_lo=bufs["feat_lo"], w_lo=ps["Vl"] and ps["Vl"]["wfc"], out_lo=bufs["h_lo"]))
        return bufs["h"]

    def _head_params(self, V):
        return {k: V[k] for k in ("wv", "bv", "wa", "ba")}

    # ---------------------------------------------------------------- step
    def _seg1(self) -> None:
        B, rt, ops = self.B, self.rt, self.ops
        self._pack_online()
        if not self._presample or self._sample_ver != self.replay.version:
            self._sample()
        S = self.S
        self.forward_all()
        isw = S["weights"] if self._isw else None
        sp = self.split
        ops.head(self.h[:2 * B], self.h[2 * B:], self._head_params(self.P), self._head_params(self.T), S["act"],
                 S["rew"], S["gam"], isw, rt.loss == "huber", rt.huber_delta, 1.0 / (B * self.world),
                 self.td_abs, self.loss_b, self.dH, self.dhead, zero=self.g_head_region, isn=self._isn(),
                 **self._lo(lo=sp and (self.h_lo[:2 * B], self.h_lo[2 * B:], self.dH_lo)))
        # priority write-back in the head-wgrad launch (csrc/sumtree.hip head_wgrad_prio_kernel)
        with self._on_side():
            ops.head_wgrad(self.h, self.dhead, self.G, prio=(self.replay, S["idx"], S["gen"], self.td_abs),
                           **self._lo(Hon_lo=self.h_lo))
        ops.fc_wgrad(self.dH, self.feat[:B], self.G["wfc"], self.G["bfc"],
                     **self._lo(dh_lo=self.dH_lo, x_lo=sp and self.feat_lo[:B]))
        self._join_side()

    def _sample(self) -> None:
        self.replay.sample(self.B, out=self.S, nxt2=self.slots[2 * self.B:])
        self._sample_ver = self.replay.version

    def _seg2(self) -> None:
        """fc data gradient, then the three stacks backwards (one stream)."""
        B, io, G = self.B, self.iops, self.G
        sp = self.split
        self.ops.fc_dgrad(self.dH, self.feat[:B], self.Pb["wfc"], self.dfeat,
                          **self._lo(dh_lo=self.dH_lo, w_lo=sp and self.Pl["wfc"], dx_lo=self.dfeat_lo))
        if sp:
            io.merge(self.dfeat, self.dfeat_lo, self.dfeat32)
        jobs: list = []
        wgrad = io.wgrad
        dO = self.dfeat32[:, :FEAT].view(B, 2, 11, 11, 16)
        for s in (2, 1, 0):
            f, b = self.fw[s], self.bw[s]
            c0, r0a, r0b, r1a, r1b = self.specs[s]
            gw = lambda cs: (G[cs.name + ".w"], G[cs.name + ".b"])  # noqa: E731
            io.conv(dO, r1b, b["d_yb"], transpose=True, mask=f["yb"][:B])
            wgrad(dO, f["yb"][:B], r1b, *gw(r1b), jobs, relu_in=True)
            io.conv(b["d_yb"], r1a, b["d_ra"], transpose=True, mask=f["ra"][:B], add=dO)
            wgrad(b["d_yb"], f["ra"][:B], r1a, *gw(r1a), jobs, relu_in=True)
            io.conv(b["d_ra"], r0b, b["d_ya"], transpose=True, mask=f["ya"][:B])
            wgrad(b["d_ra"], f["ya"][:B], r0b, *gw(r0b), jobs, relu_in=True)
            io.conv(b["d_ya"], r0a, b["d_p"], transpose=True, mask=f["p"][:B], add=b["d_ra"])
            wgrad(b["d_ya"], f["p"][:B], r0a, *gw(r0a), jobs, relu_in=True)
            if s == 0 and SW.impala_pool_wgrad:
                # stack 1's conv has one consumer of its output gradient (the ring conv's
                # weight gradient): the max-pool backward runs inside that kernel's staging
                # (split) and the 84² gradient is never written
                wgrad(b["d_p"], None, c0, *gw(c0), jobs, ring=self.replay.frames, slots=self.slots[:B],
                      scale=self.rt.obs_scale, pool_amax=f["amax"][:B])
                continue
            # max-pool backward (gather form, csrc/impala_split.hip maxpool_bwd_split_kernel)
            io.maxpool_bwd(b["d_p"], f["amax"][:B], b["d_c0"])
            dc = b["d_c0"]
            if s == 0:
                wgrad(dc, None, c0, *gw(c0), jobs, ring=self.replay.frames, slots=self.slots[:B],
                         scale=self.rt.obs_scale)
            else:
                prev = self.fw[s - 1]["o"][:B]
                wgrad(dc, prev, c0, *gw(c0), jobs)
                dO = self.bw[s - 1]["d_o"]
                io.conv(dc, c0, dO, transpose=True)
        io.finalize(jobs)

    def _seg3(self) -> None:
        rt, ops = self.rt, self.ops
        nxt = (self.replay, self.B, self.S, self.slots[2 * self.B:]) if self._presample else None
        ops.optimizer(self.p32, self.g32, self.rms_v, self.rms_m, self.pbf, rt.lr, rt.rms_decay, rt.rms_eps,
                      rt.grad_clip, rt.centered_rmsprop, self.partials, self.gnorm, sample=nxt, wnorm=self._wnorm(),
                      **self._lo(pb_lo=self.pbf_lo))
        if self._presample:
            self._sample_ver = self.replay.version

    def _step_body(self) -> None:
        self._seg1()
        self._seg2()
        self._seg3()

    def _on_side(self):
        if self._side is None:
            return contextlib.nullcontext()
        self._side.wait_stream(torch.cuda.current_stream(self.device))
        return torch.cuda.stream(self._side)

    def _join_side(self) -> None:
        if self._side is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._side)

    def _dp_step(self, graphs: bool) -> None:
        import torch.distributed as dist
        cut = self.layout.offsets["wfc"]
        run = (lambda i: self._graphs[i].replay()) if graphs else (lambda i: (self._seg1, self._seg2,
                                                                                self._seg3)[i]())
        run(0)
        # shard statistics after this step's priority write-back: the next global draw
        # (inside the optimizer launch) sees exactly the trees it samples from
        w_st = self.replay.gather_shard_stats(async_op=True)
        w_fc = dist.all_reduce(self.g32[cut:], op=dist.ReduceOp.SUM, async_op=True)
        run(1)
        w_cv = dist.all_reduce(self.g32[:cut], op=dist.ReduceOp.SUM, async_op=True)
        w_st.wait()
        w_fc.wait()
        w_cv.wait()
        run(2)

    def step(self) -> None:
        graphs = self.rt.use_graphs and self.device.type == "cuda"
        if graphs and self._graphs is None:
            self._capture()
        if graphs and self._presample and self._sample_ver != self.replay.version:
            self._sample()     # host-side replay mutation since the in-graph draw: redraw
        if self.world > 1:
            self._dp_step(graphs)
        elif graphs:
            self._graphs[0].replay()
        else:
            self._step_body()
        self.num_q_updates += 1
        if self.num_q_updates % self.cfg.Learner.q_target_sync_freq == 0:
            self.sync_target()

    def steps(self, n: int) -> None:
        """``n`` updates.  On one rank with HIP graphs, chunks of ``Runtime.graph_steps``
        updates replay one graph holding that many steps (no launch boundary between
        them), never straddling a target sync -- learner/fused_learner.py ``steps``."""
        k = int(self.rt.graph_steps)
        if k <= 1 or self.world > 1 or not (self.rt.use_graphs and self.device.type == "cuda"):
            for _ in range(n):
                self.step()
            return
        f = self.cfg.Learner.q_target_sync_freq
        while n > 0:
            if n < k or f - self.num_q_updates % f < k:
                self.step()
                n -= 1
                continue
            if self._multi is None:
                self.prepare_graphs(multi=True)
            if self._presample and self._sample_ver != self.replay.version:
                self._sample()
            self._multi.replay()
            self.num_q_updates += k
            n -= k
            if self.num_q_updates % f == 0:
                self.sync_target()

    def _capture(self) -> None:
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
        segs = [self._step_body] if self.world == 1 else [self._seg1, self._seg2, self._seg3]
        self._graphs = []
        for seg in segs:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                seg()
            self._graphs.append(g)
            self.graph_captures += 1

    def prepare_graphs(self, multi: bool = True) -> int:
        """Capture the step's graphs now (outside any timed region); with ``multi`` on one
        rank also the ``graph_steps``-update graph, replayed once from a snapshot so its
        first timed launch is warm (the first launch of a fresh graph uploads it)."""
        if not (self.rt.use_graphs and self.device.type == "cuda"):
            return self.graph_captures
        if self._graphs is None:
            self._capture()
        k = int(self.rt.graph_steps)
        if multi and self.world == 1 and k > 1 and self._multi is None:
            torch.cuda.synchronize(self.device)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                for _ in range(k):
                    self._step_body()
            self._multi = g
            self.graph_captures += 1
            self.rewarm(1)
        return self.graph_captures

    def rewarm(self, replays: int) -> None:
        """Untimed, state-preserving warm-up: replay the multi-update graph ``replays``
        times from a snapshot, then restore the learner / replay state (bench.py, before
        its timed window; no update is kept)."""
        gr = self._multi if self._multi is not None else (self._graphs[0] if self._graphs and self.world == 1
                                                          else None)
        if replays <= 0 or gr is None:
            return
        snap = self._snapshot()
        if self._presample and self._sample_ver != self.replay.version:
            self._sample()
        for _ in range(replays):
            gr.replay()
        torch.cuda.synchronize(self.device)
        self._restore(snap)
        if self._presample:
            self._sample()     # the pre-drawn batch of the restored state (same draw)
        torch.cuda.synchronize(self.device)

    def _snapshot(self):
        rp = self.replay
        return [t.clone() for t in (self.p32, self._pbf_all, self.rms_v, self.rms_m, rp.leaf, rp.nodes,
                                    rp.min_bits, rp.ctr)] + ([rp.shard_stats.clone()] if rp.sharded else [])

    def _restore(self, snap) -> None:
        rp = self.replay
        for dst, src in zip((self.p32, self._pbf_all, self.rms_v, self.rms_m, rp.leaf, rp.nodes, rp.min_bits,
                             rp.ctr) + ((rp.shard_stats,) if rp.sharded else ()), snap):
            dst.copy_(src)

    def refresh_replay_stats(self) -> bool:
        """Re-gather the shard statistics (a collective).  Fixed rows: never resizes."""
        if self.world > 1:
            self.replay.gather_shard_stats()
        return False

    def sync_target(self) -> None:
        self.t32.copy_(self.p32)
        self._tbf_all.copy_(self._pbf_all)
        self._pack_target()

    # ------------------------------------------------------------ metrics
    def last_metrics(self) -> Dict[str, float]:
        return self._is_metrics()

    def profile_step(self) -> Dict[str, float]:
        if self.device.type != "cuda":
            return {}
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        self.step()
        e1.record()
        torch.cuda.synchronize(self.device)
        return {"total": e0.elapsed_time(e1)}

    # ------------------------------------------------------------- params
    def module_state(self, V: Optional[Dict[str, torch.Tensor]] = None) -> "OrderedDict[str, torch.Tensor]":
        """Engine layout -> ``ImpalaDuellingDQN.state_dict()`` (fp32, CPU)."""
        V = self.P if V is None else V
        sd = OrderedDict()
        for s, convs in enumerate(self.specs):
            names = ["conv", "res0.conv0", "res0.conv1", "res1.conv0", "res1.conv1"]
            for nm, cs in zip(names, convs):
                sd[f"stacks.{s}.{nm}.weight"] = V[cs.name + ".w"]
                sd[f"stacks.{s}.{nm}.bias"] = V[cs.name + ".b"]
        wfc = V["wfc"][:, self._perm]
        sd["value_stream_layer.0.weight"] = wfc[:HIDDEN]
        sd["value_stream_layer.0.bias"] = V["bfc"][:HIDDEN]
        sd["advantage_stream_layer.0.weight"] = wfc[HIDDEN:]
        sd["advantage_stream_layer.0.bias"] = V["bfc"][HIDDEN:]
        sd["value.weight"] = V["wv"].view(1, HIDDEN)
        sd["value.bias"] = V["bv"]
        sd["advantage.weight"] = V["wa"]
        sd["advantage.bias"] = V["ba"]
        return OrderedDict((k, t.detach().float().cpu().clone()) for k, t in sd.items())

    def load_module_state(self, sd, V: Optional[Dict[str, torch.Tensor]] = None) -> None:
        V = self.P if V is None else V
        with torch.no_grad():
            for s, convs in enumerate(self.specs):
                names = ["conv", "res0.conv0", "res0.conv1", "res1.conv0", "res1.conv1"]
                for nm, cs in zip(names, convs):
                    V[cs.name + ".w"].copy_(sd[f"stacks.{s}.{nm}.weight"])
                    V[cs.name + ".b"].copy_(sd[f"stacks.{s}.{nm}.bias"])
            wfc = torch.zeros_like(V["wfc"])
            perm = self._perm.to(wfc.device)
            wfc[:HIDDEN, perm] = sd["value_stream_layer.0.weight"].to(wfc)
            wfc[HIDDEN:, perm] = sd["advantage_stream_layer.0.weight"].to(wfc)
            V["wfc"].copy_(wfc)
            V["bfc"][:HIDDEN].copy_(sd["value_stream_layer.0.bias"])
            V["bfc"][HIDDEN:].copy_(sd["advantage_stream_layer.0.bias"])
            V["wv"].copy_(sd["value.weight"].reshape(HIDDEN))
            V["bv"].copy_(sd["value.bias"])
            V["wa"].copy_(sd["advantage.weight"])
            V["ba"].copy_(sd["advantage.bias"])

    def state_dict(self):
        return self.module_state()

    def q_values(self, frames_u8: torch.Tensor) -> torch.Tensor:
        net = ImpalaDuellingDQN((self.C, 84, 84), self.A, channels=CH, hidden=HIDDEN).to(self.device)
        net.load_state_dict(self.module_state())
        with torch.no_grad():
            return net(frames_u8.to(self.device))[2]

    def save(self, path: str, extra: Optional[Dict] = None) -> None:
        save_checkpoint(path, self.module_state(), Q_target_state=self.module_state(self.T),
                        optimizer_state=pack_flat_state(layout_segments(self.layout), rms_v=self.rms_v, rms_m=self.rms_m),
                        num_q_updates=self.num_q_updates, config=self.cfg.to_dict(),
                        rng={"replay_ctr": int(self.replay.ctr.item()), "replay_seed": int(self.replay.seed)},
                        **(extra or {}))

    def load(self, path: str) -> bool:
        ck = load_checkpoint(path)
        if ck is None:
            return False
        if adopt_obs_scale(ck, self.rt):
            self._graphs = self._multi = None     # the input scale is a kernel argument: recapture
        self.load_module_state(ck["Q_state"])
        self._refresh_bf16()
        if "Q_target_state" in ck:
            self.load_module_state(ck["Q_target_state"], self.T)
            split_into(self.t32, self.tbf, self.tbf_lo)
            self._pack_target()
        else:
            self.sync_target()
        opt = ck.get("optimizer_state")
        unpack_flat_state(opt, layout_segments(self.layout), untagged_network=checkpoint_network(ck),
                          network=self.cfg.network, rms_v=self.rms_v, rms_m=self.rms_m)
        self.num_q_updates = int(ck.get("num_q_updates", 0))
        rng = ck.get("rng")
        if isinstance(rng, dict) and "replay_ctr" in rng:
            self.replay.ctr.fill_(int(rng["replay_ctr"]))
        return True
