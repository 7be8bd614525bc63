"""Backends for the fused NatureCNN learner step.

``TorchBackend`` -- every op in PyTorch (CPU path, and the oracle);
``HipBackend``   -- the MI355X path: hand-written gfx950 kernels from
                    ``libapex_kernels.so`` for every op that has one.

Both write into preallocated output buffers so a whole learner step can be
captured in one HIP graph.

fp32-accurate ("split") mode: every activation, gradient and bf16 weight copy
comes as a hi plane (the usual tensor) plus a ``*_lo`` plane with
``value = hi + lo`` (csrc/mfma_common.h ``split_pk_bf16``).  The HIP kernels run
three bf16 MFMAs per fragment pair (hi.hi + lo.hi + hi.lo, fp32 accumulation); the
torch backend emulates the mode by joining the planes into fp32, computing in
fp32 and splitting the outputs again, so the learner's split plumbing runs (and is
tested) on the CPU.  Without ``*_lo`` arguments every op is the plain bf16 / fp32
op of before.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional

import torch

from . import _lib
from . import conv as C
from . import reference as R
from .switches import SW


def join(hi: torch.Tensor, lo: Optional[torch.Tensor]) -> torch.Tensor:
    """hi (+ lo) as fp32."""
    return hi.float() if lo is None else hi.float() + lo.float()


def split_into(v: torch.Tensor, hi: torch.Tensor, lo: Optional[torch.Tensor]) -> None:
    """Write fp32 ``v`` as hi = round(v), lo = round(v - hi) (or just hi when lo is None)."""
    hi.copy_(v.reshape(hi.shape))
    if lo is not None:
        lo.copy_((v.reshape(hi.shape).float() - hi.float()))


class TorchBackend:
    name = "torch"

    def __init__(self, dtype=torch.float32):
        self.dtype = dtype

    # ------------------------------------------------------------- forward
    def prepare(self, Pb) -> None:
        """Per-step weight preparation (nothing on either backend: the dgrad GEMMs read
        the natural weight tensors)."""

    def conv1_fwd(self, frames, w, b, scale, out, out_lo=None):
        dt = torch.float32 if out_lo is not None else self.dtype
        split_into(R.conv1_fwd(frames, w, b, scale, dt), out, out_lo)

    def conv1_fwd_ring(self, ring, slots, frames_buf, w, b, scale, out, w2=None, b2=None, rows_first=0, w32=None,
                       w2_32=None, out_lo=None, c2f=None):
        """conv1 on frame stacks addressed by replay-ring slots (N, C); rows >=
        ``rows_first`` use the second weight set (w2, b2) when given.  Split mode reads
        the fp32 master weights ``w32`` / ``w2_32``.  ``c2f``: conv2 weights the HIP
        backend pre-packs inside this launch (ignored here)."""
        from ..replay.gpu_replay import from_s2d
        frames = frames_buf[:slots.shape[0]]
        n, c = slots.shape
        frames.copy_(from_s2d(ring[slots.long()].reshape(n * c, 84, 84)).reshape(n, c, 84, 84))
        wa, wb = (w32, w2_32) if out_lo is not None else (w, w2)
        if w2 is None:
            self.conv1_fwd(frames, wa, b, scale, out, out_lo)
        else:
            r = rows_first
            self.conv1_fwd(frames[:r], wa, b, scale, out[:r], None if out_lo is None else out_lo[:r])
            self.conv1_fwd(frames[r:], wb, b2, scale, out[r:], None if out_lo is None else out_lo[r:])

    def conv12_pack(self, c1, c2, scale, sets=2, c3=None):
        """Repack the fused conv12 kernel's weight fragments of ``sets`` (bit 0 online, bit
        1 target; HIP backend only) -- after the target weights change; ``c3``: the fused
        conv3's too."""

    def conv12_fwd(self, ring, slots, frames_buf, scale, y1, y1_lo, y2, y2_lo, c1, c2, rows_first=0, copy_n=None,
                   pack_sets=3, c3=None, y3=None, y3_lo=None):
        """conv1 -> conv2 in split mode: ``c1 = (w1 fp32, b1, w1 target, b1 target)``, ``c2 =
        (w2, w2_lo, b2, w2 target, w2_lo target, b2 target)`` (target entries None: one
        set).  y1 rows < ``copy_n`` must hold conv1's output afterwards (the backward's
        input); the HIP backend keeps the other rows in LDS (csrc/conv12_fused.hip) and
        repacks the weight fragments of ``pack_sets`` first (the others come from the last
        ``conv12_pack``).  ``c3 = (w3, w3_lo, b3, w3 target, w3_lo target, b3 target)``:
        conv3 too, into ``y3`` / ``y3_lo``."""
        w1, b1, w1b, b1b = c1
        w2, w2l, b2, w2b, w2bl, b2b = c2
        self.conv1_fwd_ring(ring, slots, frames_buf, w1.to(y1.dtype), b1, scale, y1,
                            None if w1b is None else w1b.to(y1.dtype), b1b, rows_first, w32=w1, w2_32=w1b,
                            out_lo=y1_lo)
        self.conv_fwd(y1, w2, b2, 2, y2, w2b, b2b, rows_first, x_lo=y1_lo, w_lo=w2l, w2_lo=w2bl, out_lo=y2_lo)
        if c3 is not None:
            w3, w3l, b3, w3b, w3bl, b3b = c3
            self.conv_fwd(y2, w3, b3, 1, y3, w3b, b3b, rows_first, x_lo=y2_lo, w_lo=w3l, w2_lo=w3bl, out_lo=y3_lo)

    def conv_fwd(self, x, w, b, stride, out, w2=None, b2=None, rows_first=0, x_lo=None, w_lo=None, w2_lo=None,
                 out_lo=None):
        dt = torch.float32 if x_lo is not None else self.dtype
        xf = join(x, x_lo) if x_lo is not None else x
        if w2 is None:
            split_into(R.conv_fwd(xf, join(w, w_lo), b, stride, dt), out, out_lo)
        else:
            r = rows_first
            split_into(R.conv_fwd(xf[:r], join(w, w_lo), b, stride, dt), out[:r], None if out_lo is None else out_lo[:r])
            split_into(R.conv_fwd(xf[r:], join(w2, w2_lo), b2, stride, dt), out[r:],
                       None if out_lo is None else out_lo[r:])

    def fc_fwd(self, x, w, b, out, w2=None, b2=None, rows_first=0, x_lo=None, w_lo=None, w2_lo=None, out_lo=None,
               c2d=None, defer_head=False, ksplit=0):
        """``c2d = (conv2 weight, lo plane)``: weights of this step's conv2 data gradient,
        which the HIP backend pre-packs inside the fc launch; ``defer_head``: the HIP
        backend may leave the epilogue to the next :meth:`head` (both ignored here)."""
        dt = torch.float32 if x_lo is not None else self.dtype
        x = x.reshape(x.shape[0], -1)
        xf = join(x, x_lo.reshape(x.shape)) if x_lo is not None else x
        if w2 is None:
            split_into(R.fc_fwd(xf, join(w, w_lo), b, dt), out, out_lo)
        else:
            r = rows_first
            split_into(R.fc_fwd(xf[:r], join(w, w_lo), b, dt), out[:r], None if out_lo is None else out_lo[:r])
            split_into(R.fc_fwd(xf[r:], join(w2, w2_lo), b2, dt), out[r:], None if out_lo is None else out_lo[r:])

    # ---------------------------------------------------------------- head
    def head(self, Hon, Htg, Pon: Dict[str, torch.Tensor], Ptg: Dict[str, torch.Tensor], act, rew, gam, isw,
             huber: bool, kappa: float, grad_scale: float, td_abs, loss, dH, dhead, q_out=None,
             zero: Optional[torch.Tensor] = None, lo=None, isn=None):
        """``lo = (Hon_lo, Htg_lo, dH_lo)`` in split mode.  ``isn = (wscale, out[, count])``:
        batch-max IS normalisation, ``out[0] = max(isw) / wscale`` (the optimizer divides the
        gradient by it; csrc/ddqn_head.hip ``IsNorm``; ``out`` may be None), and ``count``
        (int64) += the rows with a non-zero weight (DP: the rows this rank drew)."""
        B = act.shape[0]
        A = Pon["wa"].shape[0]
        Hon = join(Hon, None if lo is None else lo[0])
        Htg = join(Htg, None if lo is None else lo[1])

        HS = Pon["wv"].numel()   # stream width (512 NatureCNN, 256 IMPALA)

        def q_of(h, P):
            v = h[:, :HS] @ P["wv"].float() + P["bv"].float()
            a = h[:, HS:] @ P["wa"].float().t() + P["ba"].float()
            return v[:, None] + a - a.mean(1, keepdim=True)

        q_t = q_of(Hon[:B], Pon)
        q_n = q_of(Hon[B:2 * B], Pon)
        q_g = q_of(Htg[:B], Ptg)
        a_star = q_n.argmax(1)
        G = rew.float() + gam.float() * q_g.gather(1, a_star[:, None]).squeeze(1)
        q_sa = q_t.gather(1, act.long()[:, None]).squeeze(1)
        delta = G - q_sa
        ad = delta.abs()
        if huber:
            lval = torch.where(ad <= kappa, 0.5 * delta * delta, kappa * (ad - 0.5 * kappa))
            dl = torch.where(ad <= kappa, delta, kappa * delta.sign())
        else:
            lval = 0.5 * delta * delta
            dl = delta
        w = isw.float() if isw is not None else torch.ones_like(delta)
        dq = -w * dl * grad_scale
        td_abs.copy_(ad)
        loss.copy_(w * lval)
        onehot = torch.nn.functional.one_hot(act.long(), A).float()
        dadv = dq[:, None] * (onehot - 1.0 / A)
        dhead[:, 0] = dq
        dhead[:, 1:] = dadv
        dv = dq[:, None] * Pon["wv"].float()[None, :]
        da = dadv @ Pon["wa"].float()
        dh = torch.cat([dv, da], 1) * (Hon[:B] > 0).float()
        split_into(dh, dH, None if lo is None else lo[2])
        if q_out is not None:
            q_out.copy_(q_t)
        if zero is not None:
            zero.zero_()
        if isn is not None:
            if isn[1] is not None:   # tensor ops only: no host sync (graph-capturable)
                ws = isn[0].reshape(-1)[0].double() if isn[0] is not None else torch.ones((), dtype=torch.float64,
                                                                                           device=w.device)
                m = w.max().double()
                isn[1].reshape(-1)[0] = torch.where(ws > 0, m / torch.where(ws > 0, ws, torch.ones_like(ws)),
                                                    torch.zeros_like(m))
            if len(isn) > 2 and isn[2] is not None:
                isn[2].add_((w > 0).sum())

    def head_wgrad(self, Hon, dhead, g: Dict[str, torch.Tensor], prio=None, Hon_lo=None, pack=None):
        """``prio = (replay, idx, gen, td_abs)``: also write the batch's priorities back
        (the HIP backend runs it as one extra block of the same launch).  ``pack = (dst,
        segs)``: also the :meth:`pack_rows` of the DP step's factor rows (HIP: tail blocks
        of the same launch)."""
        if pack is not None:
            self.pack_rows(*pack)
        if prio is not None:
            prio[0].update_priorities(prio[1], prio[3], prio[2])
        B = dhead.shape[0]
        HS = g["wv"].numel()
        h = join(Hon[:B], None if Hon_lo is None else Hon_lo[:B])
        g["wv"].add_(dhead[:, 0] @ h[:, :HS])
        g["bv"].add_(dhead[:, 0].sum().view(1))
        g["wa"].add_(dhead[:, 1:].t() @ h[:, HS:])
        g["ba"].add_(dhead[:, 1:].sum(0))

    def actor_head(self, H, P, eps, ctr, seed, q_out, a_out, H_lo=None):
        """Dueling q + epsilon-greedy per row (the oracle of csrc actor_head_kernel);
        ``H_lo``: split mode, the activations' lo plane."""
        h = join(H, H_lo)
        HS = P["wv"].numel()
        v = h[:, :HS] @ P["wv"].float() + P["bv"].float()
        a = h[:, HS:] @ P["wa"].float().t() + P["ba"].float()
        q = v[:, None] + a - a.mean(1, keepdim=True)
        q_out.copy_(q)
        E, A = q.shape
        gen = torch.Generator(device="cpu").manual_seed(int(seed) * 1000003 + int(ctr.item()))
        u = torch.rand(E, generator=gen).to(q.device)
        r = torch.randint(0, A, (E,), generator=gen).to(q.device)
        a_out.copy_(torch.where(u < eps.to(q.device), r, q.argmax(1)).to(a_out.dtype))

    # ------------------------------------------------------------ backward
    def fc_bwd(self, dh, x, w, dx_out, dw_out, db_out):
        self.fc_dgrad(dh, x, w, dx_out)
        self.fc_wgrad(dh, x, dw_out, db_out)

    def fc_dgrad(self, dh, x, w, dx_out, dh_lo=None, w_lo=None, dx_lo=None):
        """dx = (dh @ w) * (x > 0) (x = the ReLU'd fc input)."""
        xf = x.reshape(x.shape[0], -1)
        if dh_lo is not None:
            dx = (join(dh, dh_lo) @ join(w, w_lo)) * (xf > 0).float()
            split_into(dx, dx_out, dx_lo)
            return
        dx, _, _ = R.fc_bwd(dh, xf, w, xf, self.dtype)
        dx_out.copy_(dx.reshape(dx_out.shape))

    def fc_wgrad(self, dh, x, dw_out, db_out, norm=None, dh_lo=None, x_lo=None):
        """``norm = (partials, slot0)``: also the squared norm of what it writes, in fp64
        at ``partials[slot0]`` (one slot; the HIP kernel writes 4 per workgroup)."""
        xf = join(x.reshape(x.shape[0], -1), None if x_lo is None else x_lo.reshape(x.shape[0], -1))
        dhf = join(dh, dh_lo)
        dw_out.copy_(dhf.t() @ xf)
        db_out.copy_(dhf.sum(0))
        if norm is None:
            return 0
        part, s0 = norm
        part[s0] = dw_out.double().pow(2).sum() + db_out.double().pow(2).sum()
        return 1

    def fc_wgrad_split(self, dh, x, dw_out, db_out, jobs, split_rows: int, jnorm, dh_lo=None, x_lo=None,
                       cpb: int = -1) -> int:
        """The fc weight gradient as split-K partials reduced by the step's
        ``finalize_grads`` (HIP: a job appended to ``jobs``); its squared-norm partials go
        to ``jnorm`` (one per finalize block).  Returns the partial count.  The torch
        path computes it at once (one partial)."""
        return self.fc_wgrad(dh, x, dw_out, db_out, norm=(jnorm, 0), dh_lo=dh_lo, x_lo=x_lo)

    def fc_head_wgrad(self, dh, x, dw_out, db_out, Hon, dhead, g_head, prio, norm=None, dh_lo=None, x_lo=None,
                      Hon_lo=None) -> int:
        """fc weight gradient + head weight gradient (+ the priority write-back,
        ``prio = (replay, idx, gen, td_abs)``); returns the fc norm slots used."""
        self.head_wgrad(Hon, dhead, g_head, prio=prio, Hon_lo=Hon_lo)
        return self.fc_wgrad(dh, x, dw_out, db_out, norm=norm, dh_lo=dh_lo, x_lo=x_lo) or 0

    def finalize_grads(self, jobs, norm_range=None, norm=None) -> int:
        """Deferred split-K reductions (the torch path computes gradients directly)."""
        return 0

    def conv_dgrad(self, dy, w, stride, x_src, dx_out, dy_lo=None, w_lo=None, dx_lo=None):
        if dy_lo is not None:
            dx = R.conv_dgrad(join(dy, dy_lo), join(w, w_lo), tuple(x_src.shape), stride, x_src, torch.float32)
            split_into(dx, dx_out, dx_lo)
            return
        dx_out.copy_(R.conv_dgrad(dy, w, tuple(x_src.shape), stride, x_src, self.dtype))

    def conv_wgrad(self, dy, x, k, stride, dw_out, db_out, jobs=None, dy_lo=None, x_lo=None):
        dw, db = R.conv_wgrad(join(dy, dy_lo), join(x, x_lo), k, stride)
        dw_out.copy_(dw)
        db_out.copy_(db)

    def conv1_wgrad(self, dy, frames, scale, dw_out, db_out, dy_lo=None):
        dw, db = R.conv1_wgrad(join(dy, dy_lo), frames, scale)
        dw_out.copy_(dw)
        db_out.copy_(db)

    def conv1_wgrad_ring(self, dy, ring, slots, frames_buf, scale, dw_out, db_out, jobs=None, dy_lo=None):
        self.conv1_wgrad(dy, frames_buf[:slots.shape[0]], scale, dw_out, db_out, dy_lo=dy_lo)

    # ----------------------------------------------------------- optimizer
    def optimizer(self, p32, g32, v, m, pbf, lr, alpha, eps, clip, centered, partials, norm_out, norm_total=None,
                  sample=None, pb_lo=None, wnorm=None, frag_out=None, segs=None, norm_prefix=None):
        """``sample = (replay, B, out, nxt2)``: also draw the next
        batch after the update (the HIP backend fuses it into the optimizer launch).
        ``pb_lo``: split mode, the lo plane of the bf16 copy.  ``wnorm = (stats, n,
        stride)``: batch-max IS normalisation, the gradient is divided by the largest of
        the n per-rank maxima ``stats[k * stride]`` (csrc/rmsprop_common.h is_grad_scale).
        ``norm_total = (partials, n)``: the clip norm is sqrt(sum(partials[:n])) (squared-norm
        partials written by the gradient producers) instead of a pass over ``g32``.
        ``segs``: [(offset, length), ...] -- update only these ranges of the flat arrays
        (the sharded data-parallel update; needs ``norm_total``).  ``norm_prefix``: a
        gradient range whose squares join the partials' sum (summed inside the launch)."""
        self._optimizer(p32, g32, v, m, pbf, lr, alpha, eps, clip, centered, norm_out, pb_lo, wnorm, norm_total,
                        segs, norm_prefix)
        if sample is not None:
            rp, B, out, nxt2 = sample
            rp.sample(B, out=out, nxt2=nxt2)

    def _optimizer(self, p32, g32, v, m, pbf, lr, alpha, eps, clip, centered, norm_out, pb_lo=None, wnorm=None,
                   norm_total=None, segs=None, norm_prefix=None):
        sc = torch.ones((), dtype=torch.float32, device=g32.device)
        if wnorm is not None:     # tensor ops only: no host sync (graph-capturable)
            st, n, stride = wnorm
            mx = st.reshape(-1)[0:n * stride:stride].max().float()
            sc = torch.where(mx > 0, 1.0 / mx.clamp_min(1e-30), sc)
        if norm_total is not None:
            part, npart = norm_total if isinstance(norm_total, tuple) else (norm_total, 1)
            sq = part[:npart].double().sum()
            if norm_prefix is not None:
                sq = sq + norm_prefix.double().pow(2).sum()
        else:
            assert segs is None, "a sharded update needs the clip norm's partials (norm_total)"
            sq = g32.double().pow(2).sum()
        norm = sq.sqrt().float() * sc
        coef = torch.clamp(clip / (norm + 1e-6), max=1.0) if clip > 0 else torch.ones_like(norm)
        for o, n in (segs if segs is not None else [(0, p32.numel())]):
            r = slice(o, o + n)
            g = g32[r] * (coef * sc)
            vr, mr, pr = v[r], m[r], p32[r]
            vr.mul_(alpha).add_((1 - alpha) * g * g)
            if centered:
                mr.mul_(alpha).add_((1 - alpha) * g)
                var = vr - mr * mr
            else:
                var = vr
            pr.sub_(lr * g / (var.clamp_min(0).sqrt() + eps))
            split_into(pr, pbf[r], None if pb_lo is None else pb_lo[r])
        norm_out.copy_(norm.view(1))

    def gather_frames(self, replay, slots, out):
        replay.gather_frames(slots, out)

    # ------------------------------------------- data-parallel gradient factors
    def pack_rows(self, dst: torch.Tensor, segs) -> None:
        """dst[:, c0:c0 + n] = seg for the 2-D ``segs`` laid side by side (same row count)."""
        c0 = 0
        for t in segs:
            t2 = t.reshape(t.shape[0], -1)
            dst[:t2.shape[0], c0:c0 + t2.shape[1]].copy_(t2)
            c0 += t2.shape[1]

    def sqnorm_ranges(self, ranges, partials: torch.Tensor, nblk: int) -> int:
        """Squared-norm partials of the fp32 ``ranges`` into ``partials`` (fp64; the HIP
        kernel writes ``nblk`` block partials, this one slot).  Returns the slots written."""
        partials[0] = sum(r.double().pow(2).sum() for r in ranges if r is not None)
        return 1


class HipBackend(TorchBackend):
    """MI355X backend: the hand-written gfx950 kernels (``kernels`` lists the op
    families).  A missing kernel library is an error (``_lib.require_kernels``)."""

    name = "hip"

    def __init__(self, dtype=torch.bfloat16, native_conv: bool = True):
        super().__init__(dtype)
        self.lib = _lib.require_kernels()
        self.native_conv = native_conv and hasattr(self.lib, "apex_conv_fwd")
        self.kernels = ["replay", "head", "head_wgrad", "optimizer", "actor_head"]
        if self.native_conv:
            self.kernels += ["conv_fwd", "conv_dgrad", "conv_wgrad", "fc_fwd", "fc_bwd"]
        self.ws = C.Workspace()

    # --------------------------------------------------- native conv family
    def conv1_fwd_ring(self, ring, slots, frames_buf, w, b, scale, out, w2=None, b2=None, rows_first=0, w32=None,
                       w2_32=None, out_lo=None, c2f=None):
        if not self.native_conv:
            return super().conv1_fwd_ring(ring, slots, frames_buf, w, b, scale, out, w2, b2, rows_first, w32, w2_32,
                                          out_lo)
        c2f = c2f if (c2f is not None and SW.c2f_pack) else None
        C.conv1_s2d_fwd(self.lib, self.ws, ring, slots, w, b, scale, out, w2, b2, rows_first, w32=w32, w2_32=w2_32,
                        out_lo=out_lo, c2f=c2f)
        if c2f is not None:   # this step's split conv2 forward finds its weights packed
            self._c2f_packed = tuple(_lib.ptr(t) for t in c2f)

    def _conv12_native(self) -> bool:
        return self.native_conv and SW.conv12_fused and hasattr(self.lib, "apex_conv12_fused_fwd")

    def conv12_pack(self, c1, c2, scale, sets=2, c3=None):
        if not self._conv12_native():
            return
        w1, b1, w1b, b1b = c1
        w2, w2l, b2, w2b, w2bl, b2b = c2
        C.conv12_pack(self.lib, self.ws, w1, b1, w2, w2l, b2, scale, w1b=w1b, b1b=b1b, w2b=w2b, w2b_lo=w2bl,
                      b2b=b2b, sets=sets, c3=c3)

    def conv12_fwd(self, ring, slots, frames_buf, scale, y1, y1_lo, y2, y2_lo, c1, c2, rows_first=0, copy_n=None,
                   pack_sets=3, c3=None, y3=None, y3_lo=None):
        if not self._conv12_native():
            return super().conv12_fwd(ring, slots, frames_buf, scale, y1, y1_lo, y2, y2_lo, c1, c2, rows_first,
                                      copy_n, c3=c3, y3=y3, y3_lo=y3_lo)
        w1, b1, w1b, b1b = c1
        w2, w2l, b2, w2b, w2bl, b2b = c2
        n = slots.shape[0] if copy_n is None else int(copy_n)
        C.conv12_fused_fwd(self.lib, self.ws, ring, slots, w1, b1, w2, w2l, b2, scale, y2, y2_lo, y1=y1, y1_lo=y1_lo,
                           copy_n=n, w1b=w1b, b1b=b1b, w2b=w2b, w2b_lo=w2bl, b2b=b2b, rows_first=rows_first,
                           pack_sets=pack_sets, c3=c3, y3=y3, y3_lo=y3_lo)

    def conv_fwd(self, x, w, b, stride, out, w2=None, b2=None, rows_first=0, x_lo=None, w_lo=None, w2_lo=None,
                 out_lo=None):
        if not self.native_conv:
            return super().conv_fwd(x, w, b, stride, out, w2, b2, rows_first, x_lo, w_lo, w2_lo, out_lo)
        key = (_lib.ptr(w), _lib.ptr(w_lo), _lib.ptr(w2), _lib.ptr(w2_lo))
        packed = stride == 2 and getattr(self, "_c2f_packed", None) == key
        if packed:
            self._c2f_packed = None
        C.conv_fwd(self.lib, x, w, b, stride, out, w2, b2, rows_first, x_lo=x_lo, w_lo=w_lo, w2_lo=w2_lo,
                   out_lo=out_lo, packed=packed)

    def fc_fwd(self, x, w, b, out, w2=None, b2=None, rows_first=0, x_lo=None, w_lo=None, w2_lo=None, out_lo=None,
               c2d=None, defer_head=False, ksplit=0):
        """``ksplit`` > 0: that K split instead of the one that fills the chip (the actors:
        a throughput job beside the learner, where fewer partial planes cost less)."""
        if not self.native_conv:
            return super().fc_fwd(x, w, b, out, w2, b2, rows_first, x_lo, w_lo, w2_lo, out_lo)
        M, K = x.shape[0], x[0].numel()
        if w.shape[0] % 128 == 0 and K % 64 == 0 and hasattr(self.lib, "apex_fc_gemm128"):
            # 128x128 tiles, K split in two, loader waves: fc forward 40.6 -> 36.2 us
            # (split) / 25.7 -> 22.5 (bf16) at the learner shape (scripts/bench_fc128.py)
            defer = defer_head and w2 is not None and b is not None and b2 is not None and \
                2 * (M // 3) == rows_first and M % 3 == 0
            # K splits so the launch fills the chip: 2 at the learner's 1536 rows (96 tiles,
            # 192 blocks), more for the few row tiles of a small per-rank batch (global-batch
            # DP: 74 rows per rank -> 24 tiles x 10 splits)
            tiles = C.row_tiles_host(M, rows_first if w2 is not None else None, 128) * (w.shape[0] // 128)
            if ksplit > 0:
                ks = int(ksplit)
            else:
                ks = max(2, 256 // max(tiles, 1))
                if SW.fc_ksplit_max > 0:
                    ks = max(1, min(ks, SW.fc_ksplit_max))
            r = C.dense_fwd128(self.lib, self.ws, x.reshape(M, K), w, b, out, True, w2, b2, rows_first, ks, True,
                               x_lo=None if x_lo is None else x_lo.reshape(M, K), w_lo=w_lo, w2_lo=w2_lo,
                               out_lo=out_lo, c2d_pack=None if defer else c2d, no_epilogue=defer)
            if defer:
                # the split-K epilogue (and the conv2 pack) move into the next head launch
                self._fc_part = dict(part=r[0], nz=r[1], zstride=M * w.shape[0], b=b, b2=b2,
                                     two_b=rows_first, out=out, c2d=c2d)
                return
            # the conv2 data gradient of this step finds its weights packed (the key is
            # checked there, so a different weight tensor still packs its own)
            if c2d is not None:
                self._c2d_packed = (c2d[0].data_ptr(), _lib.ptr(c2d[1]))
            return
        C.dense_fwd(self.lib, x.reshape(x.shape[0], -1), w, b, out, relu=True, w2=w2, b2=b2,
                    rows_first=rows_first, ws=self.ws,
                    x_lo=None if x_lo is None else x_lo.reshape(x.shape[0], -1), w_lo=w_lo, w2_lo=w2_lo,
                    out_lo=out_lo)

    def fc_dgrad(self, dh, x, w, dx_out, dh_lo=None, w_lo=None, dx_lo=None):
        if not self.native_conv:
            return super().fc_dgrad(dh, x, w, dx_out, dh_lo, w_lo, dx_lo)
        xf = x.reshape(x.shape[0], -1)
        C.dense_dgrad(self.lib, dh, w, dx_out.reshape(dh.shape[0], -1), xf, dh_lo=dh_lo, w_lo=w_lo,
                      out_lo=None if dx_lo is None else dx_lo.reshape(dh.shape[0], -1))

    def fc_wgrad(self, dh, x, dw_out, db_out, norm=None, dh_lo=None, x_lo=None):
        if not self.native_conv:
            return super().fc_wgrad(dh, x, dw_out, db_out, dh_lo=dh_lo, x_lo=x_lo)
        return C.dense_wgrad(self.lib, dh, x.reshape(x.shape[0], -1), dw_out, db_out, norm=norm, dy_lo=dh_lo,
                             x_lo=None if x_lo is None else x_lo.reshape(x.shape[0], -1))

    def fc_wgrad_split(self, dh, x, dw_out, db_out, jobs, split_rows: int, jnorm, dh_lo=None, x_lo=None,
                       cpb: int = -1) -> int:
        if not self.native_conv:
            return super().fc_wgrad_split(dh, x, dw_out, db_out, jobs, split_rows, jnorm, dh_lo, x_lo, cpb)
        M = dh.shape[0]
        return C.dense_wgrad_split(self.lib, self.ws, dh, x.reshape(M, -1), max(1, -(-M // int(split_rows))),
                                   dw_out, db_out, jobs, dy_lo=dh_lo,
                                   x_lo=None if x_lo is None else x_lo.reshape(M, -1), cpb=cpb, jnorm=jnorm)

    def fc_head_wgrad(self, dh, x, dw_out, db_out, Hon, dhead, g_head, prio, norm=None, dh_lo=None, x_lo=None,
                      Hon_lo=None) -> int:
        if self.native_conv and prio is not None and prio[0].use_hip:
            rp, idx, gen, td = prio
            r = C.dense_wgrad_head_prio(self.lib, dh, x.reshape(x.shape[0], -1), dw_out, db_out, norm, Hon, dhead,
                                        g_head, rp, idx, gen, td, dy_lo=dh_lo,
                                        x_lo=None if x_lo is None else x_lo.reshape(x.shape[0], -1), Hon_lo=Hon_lo)
            if r is not None:
                return r
        return super().fc_head_wgrad(dh, x, dw_out, db_out, Hon, dhead, g_head, prio, norm, dh_lo, x_lo, Hon_lo)

    def finalize_grads(self, jobs, norm_range=None, norm=None) -> int:
        """Returns the number of squared-norm partial slots written (``slot0`` + blocks)."""
        if not jobs and norm is None:
            return 0
        if norm is None:
            C.finalize_grads(self.lib, jobs)
            return 0
        return norm["slot0"] + C.finalize_grads(self.lib, jobs, norm_range, norm["part"], norm["slot0"],
                                                norm.get("total"))

    def conv_dgrad(self, dy, w, stride, x_src, dx_out, dy_lo=None, w_lo=None, dx_lo=None):
        if not self.native_conv:
            return super().conv_dgrad(dy, w, stride, x_src, dx_out, dy_lo, w_lo, dx_lo)
        if stride == 1:
            C.conv3_dgrad(self.lib, dy, w, x_src, dx_out, dy_lo=dy_lo, w_lo=w_lo, out_lo=dx_lo)
        else:
            key = (w.data_ptr(), _lib.ptr(w_lo))
            packed = getattr(self, "_c2d_packed", None) == key
            self._c2d_packed = None
            C.conv2_dgrad(self.lib, dy, w, x_src, dx_out, dy_lo=dy_lo, w_lo=w_lo, out_lo=dx_lo, ws=self.ws,
                          packed=packed)

    def conv_wgrad(self, dy, x, k, stride, dw_out, db_out, jobs=None, dy_lo=None, x_lo=None):
        if not self.native_conv:
            return super().conv_wgrad(dy, x, k, stride, dw_out, db_out, dy_lo=dy_lo, x_lo=x_lo)
        C.conv_wgrad(self.lib, self.ws, dy, x, k, stride, dw_out, db_out, jobs=jobs, dy_lo=dy_lo, x_lo=x_lo)

    def conv1_wgrad_ring(self, dy, ring, slots, frames_buf, scale, dw_out, db_out, jobs=None, dy_lo=None):
        if not self.native_conv:
            return super().conv1_wgrad_ring(dy, ring, slots, frames_buf, scale, dw_out, db_out, dy_lo=dy_lo)
        C.conv1_wgrad_ring(self.lib, self.ws, dy, ring, slots, scale, dw_out, db_out, jobs=jobs, dy_lo=dy_lo)

    @staticmethod
    def _hp(P):
        h = _lib.HeadParams()
        h.wv, h.bv, h.wa, h.ba = (P["wv"].data_ptr(), P["bv"].data_ptr(), P["wa"].data_ptr(),
                                  P["ba"].data_ptr())
        return h

    def head(self, Hon, Htg, Pon, Ptg, act, rew, gam, isw, huber, kappa, grad_scale, td_abs, loss, dH,
             dhead, q_out=None, zero=None, lo=None, isn=None):
        B = act.shape[0]
        A = Pon["wa"].shape[0]
        args = (Hon.data_ptr(), Htg.data_ptr(), self._hp(Pon), self._hp(Ptg), act.data_ptr(), rew.data_ptr(),
                gam.data_ptr(), _lib.ptr(isw), B, A, int(huber), float(kappa), float(grad_scale),
                td_abs.data_ptr(), loss.data_ptr(), _lib.ptr(q_out), dH.data_ptr(), dhead.data_ptr(),
                _lib.ptr(zero), 0 if zero is None else zero.numel(), Pon["wv"].numel())
        hl = _lib.head_lo(*(lo if lo is not None else (None, None, None)))
        hp, pk = _lib.HeadPart(), _lib.C2dPack()
        fp = getattr(self, "_fc_part", None)
        if fp is not None:
            # the deferred fc epilogue: h rows [0, B) (+ lo plane) are written by this launch
            self._fc_part = None
            assert fp["out"].data_ptr() == Hon.data_ptr() and fp["two_b"] == 2 * B
            hp.part, hp.zstride, hp.nz = fp["part"].data_ptr(), int(fp["zstride"]), int(fp["nz"])
            hp.bias_on, hp.bias_tg, hp.two_b = fp["b"].data_ptr(), fp["b2"].data_ptr(), int(fp["two_b"])
            hp.hon, hp.hon_lo = Hon.data_ptr(), _lib.ptr(None if lo is None else lo[0])
            if fp["c2d"] is not None:
                pk.w, pk.w_lo = fp["c2d"][0].data_ptr(), _lib.ptr(fp["c2d"][1])
                pk.out = C.c2d_wfrag_buffer(self.ws, Hon.device).data_ptr()
                self._c2d_packed = (fp["c2d"][0].data_ptr(), _lib.ptr(fp["c2d"][1]))
        isn_s = _lib.IsNorm()
        if isn is not None:
            isn_s.wscale, isn_s.out = _lib.ptr(isn[0]), _lib.ptr(isn[1])
            isn_s.valid_count = _lib.ptr(isn[2]) if len(isn) > 2 else None
        _lib.check(self.lib.apex_ddqn_head(*args, hl, hp, pk, isn_s, _lib.stream_ptr()), "ddqn_head")

    def head_wgrad(self, Hon, dhead, g, prio=None, Hon_lo=None, pack=None):
        B, A1 = dhead.shape
        if prio is not None and prio[0].use_hip and B <= 1024:
            rp, idx, gen, td = prio
            pk = self._pack_args(*pack) if pack is not None else (None, None, None, 0, 0, None, 0)
            _lib.check(self.lib.apex_head_wgrad_prio(
                Hon.data_ptr(), dhead.data_ptr(), B, A1 - 1, g["wv"].data_ptr(), g["bv"].data_ptr(),
                g["wa"].data_ptr(), g["ba"].data_ptr(), g["wv"].numel(), rp.tree_desc(), idx.data_ptr(),
                td.data_ptr(), _lib.ptr(gen), rp.gen.data_ptr(), rp.alpha, rp.eps, rp.ctr.data_ptr(),
                _lib.ptr(Hon_lo), _lib.ptr(rp.local_stats), *pk, _lib.stream_ptr()), "head_wgrad_prio")
            return
        if pack is not None:
            self.pack_rows(*pack)
        if prio is not None:
            prio[0].update_priorities(prio[1], prio[3], prio[2])
        _lib.check(self.lib.apex_head_wgrad(Hon.data_ptr(), dhead.data_ptr(), B, A1 - 1, g["wv"].data_ptr(),
                                            g["bv"].data_ptr(), g["wa"].data_ptr(), g["ba"].data_ptr(),
                                            g["wv"].numel(), _lib.ptr(Hon_lo), _lib.stream_ptr()), "head_wgrad")

    def actor_head(self, H, P, eps, ctr, seed, q_out, a_out, H_lo=None):
        E, A = q_out.shape
        _lib.check(self.lib.apex_actor_head(H.data_ptr(), self._hp(P), E, A, eps.data_ptr(), int(seed),
                                            ctr.data_ptr(), q_out.data_ptr(), a_out.data_ptr(),
                                            P["wv"].numel(), _lib.ptr(H_lo), _lib.stream_ptr()), "actor_head")

    def optimizer(self, p32, g32, v, m, pbf, lr, alpha, eps, clip, centered, partials, norm_out, norm_total=None,
                  sample=None, pb_lo=None, wnorm=None, frag_out=None, segs=None, norm_prefix=None) -> bool:
        """``frag_out`` (ops/conv.py conv12_frag_out): the launch also stores the updated
        w1 / w2 in the fused forward's fragment order.  Returns whether it did (the fused
        optimizer + sample launch only).  ``segs``: the ranges to update (the sharded DP
        update: one launch, csrc/sumtree.hip ``RmsSegs``)."""
        n = p32.numel()
        if segs is not None:
            if norm_total is None:
                raise ValueError("a sharded update needs the clip norm's partials (norm_total)")
            if sample is None or not sample[0].use_hip:
                raise ValueError("the sharded update runs in the fused optimizer + sample launch")
            sg = _lib.RmsSegs()
            sg.nseg = len(segs)
            assert 1 <= sg.nseg <= 3
            for k, (o, ln) in enumerate(segs):
                sg.off[k], sg.len[k] = int(o), int(ln)
            segp = ctypes.byref(sg)
        else:
            segp = None
        st = _lib.stream_ptr()
        lo = _lib.ptr(pb_lo)
        wn = (wnorm[0].data_ptr(), int(wnorm[1]), int(wnorm[2])) if wnorm is not None else (None, 0, 0)
        if frag_out is not None and not (sample is not None and sample[0].use_hip):
            raise ValueError("frag_out needs the fused optimizer + sample launch (a HIP replay)")
        if sample is not None and sample[0].use_hip:
            # the next batch's draw rides in the optimizer launch (csrc/sumtree.hip: rmsprop_sample_kernel)
            rp, B, out, nxt2 = sample
            if norm_total is None:
                _lib.check(self.lib.apex_grad_sqnorm_partials(g32.data_ptr(), n, partials.data_ptr(), st), "sqnorm")
                part, npart = partials, partials.numel()
            elif isinstance(norm_total, tuple):   # (producer partials, count): summed in the launch
                part, npart = norm_total
            else:
                part, npart = norm_total, 1
            _lib.check(self.lib.apex_rmsprop_sample(
                p32.data_ptr(), g32.data_ptr(), v.data_ptr(), m.data_ptr(), pbf.data_ptr(), n, part.data_ptr(), npart,
                float(lr), float(alpha), float(eps), float(clip), int(centered), norm_out.data_ptr(),
                *rp.sample_launch_args(B, out, nxt2), lo, *wn, frag_out if frag_out is not None else _lib.CfFragOut(),
                segp, _lib.ptr(norm_prefix), 0 if norm_prefix is None else norm_prefix.numel(), st), "rmsprop_sample")
            return frag_out is not None
        if norm_prefix is not None:
            raise ValueError("norm_prefix runs in the fused optimizer + sample launch")
        if sample is not None:
            self.optimizer(p32, g32, v, m, pbf, lr, alpha, eps, clip, centered, partials, norm_out, norm_total,
                           pb_lo=pb_lo, wnorm=wnorm)
            rp, B, out, nxt2 = sample
            rp.sample(B, out=out, nxt2=nxt2)
            return
        if norm_total is not None:   # squared norm already summed by the gradient producers
            part, npart = norm_total if isinstance(norm_total, tuple) else (norm_total, 1)
            _lib.check(self.lib.apex_rmsprop_step_np(p32.data_ptr(), g32.data_ptr(), v.data_ptr(), m.data_ptr(),
                                                     pbf.data_ptr(), n, part.data_ptr(), npart, float(lr),
                                                     float(alpha), float(eps), float(clip), int(centered),
                                                     norm_out.data_ptr(), lo, *wn, st), "rmsprop_np")
            return
        _lib.check(self.lib.apex_grad_sqnorm_partials(g32.data_ptr(), n, partials.data_ptr(), st), "sqnorm")
        _lib.check(self.lib.apex_rmsprop_step(p32.data_ptr(), g32.data_ptr(), v.data_ptr(), m.data_ptr(),
                                              pbf.data_ptr(), n, partials.data_ptr(), float(lr), float(alpha),
                                              float(eps), float(clip), int(centered), norm_out.data_ptr(), lo, *wn,
                                              st),
                   "rmsprop")

    def _pack_args(self, dst: torch.Tensor, segs):
        """(src*, ld*, cols*, nseg, rows, dst, dst ld) of a row pack (csrc/pack_rows.h); the
        ctypes arrays stay referenced by this backend until the next call."""
        assert dst.dtype in (torch.bfloat16, torch.float16) and len(segs) <= 4
        n = len(segs)
        src = (ctypes.c_void_p * 4)(*[t.data_ptr() for t in segs])
        ld = (ctypes.c_int64 * 4)(*[t.stride(0) for t in segs])
        cols = (ctypes.c_int * 4)(*[t.reshape(t.shape[0], -1).shape[1] for t in segs])
        for t in segs:
            assert t.dtype == dst.dtype and t.reshape(t.shape[0], -1).stride(1) == 1 and t.shape[0] == segs[0].shape[0]
        self._pack_keep = (src, ld, cols)
        return (ctypes.addressof(src), ctypes.addressof(ld), ctypes.addressof(cols), n, int(segs[0].shape[0]),
                dst.data_ptr(), int(dst.stride(0)))

    def pack_rows(self, dst: torch.Tensor, segs) -> None:
        if dst.dtype not in (torch.bfloat16, torch.float16) or len(segs) > 4:
            return super().pack_rows(dst, segs)
        _lib.check(self.lib.apex_pack_rows(*self._pack_args(dst, segs), _lib.stream_ptr()), "pack_rows")

    def grad_sqnorm_partials(self, g32, partials) -> int:
        """Squared-norm partials of the whole gradient (the optimizer's own pass);
        returns the partial count."""
        _lib.check(self.lib.apex_grad_sqnorm_partials(g32.data_ptr(), g32.numel(), partials.data_ptr(),
                                                      _lib.stream_ptr()), "sqnorm")
        return partials.numel()

    def sqnorm_ranges(self, ranges, partials: torch.Tensor, nblk: int) -> int:
        (a, b) = (list(ranges) + [None])[:2]
        _lib.check(self.lib.apex_sqnorm_ranges(a.data_ptr(), a.numel(), _lib.ptr(b), 0 if b is None else b.numel(),
                                               partials.data_ptr(), int(nblk), _lib.stream_ptr()), "sqnorm_ranges")
        return int(nblk)

    def cast_bf16(self, x32, hi, lo=None) -> None:
        """hi = bf16(x32) (and lo = bf16(x32 - hi)) with one kernel."""
        _lib.check(self.lib.apex_cast_bf16(x32.data_ptr(), hi.data_ptr(), x32.numel(), _lib.ptr(lo),
                                           _lib.stream_ptr()), "cast_bf16")
