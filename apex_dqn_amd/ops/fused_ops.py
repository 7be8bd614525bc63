"""Backends for the fused NatureCNN learner step.

``TorchBackend`` -- every op in PyTorch (CPU path, and the oracle);
``HipBackend``   -- the MI355X path: hand-written gfx950 kernels from
                    ``libapex_kernels.so`` for every op that has one.

Both write into preallocated output buffers so a whole learner step can be
captured in one HIP graph.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from . import _lib
from . import conv as C
from . import reference as R


class TorchBackend:
    name = "torch"

    def __init__(self, dtype=torch.float32):
        self.dtype = dtype

    # ------------------------------------------------------------- forward
    def prepare(self, Pb) -> None:
        """Per-step weight preparation (packed dgrad copies on the HIP path)."""

    def conv1_fwd(self, frames, w, b, scale, out):
        out.copy_(R.conv1_fwd(frames, w, b, scale, self.dtype))

    def conv1_fwd_ring(self, ring, slots, frames_buf, w, b, scale, out, w2=None, b2=None, rows_first=0):
        """conv1 on frame stacks addressed by replay-ring slots (N, C); rows >=
        ``rows_first`` use the second weight set (w2, b2) when given."""
        from ..replay.gpu_replay import from_s2d
        frames = frames_buf[:slots.shape[0]]
        n, c = slots.shape
        frames.copy_(from_s2d(ring[slots.long()].reshape(n * c, 84, 84)).reshape(n, c, 84, 84))
        if w2 is None:
            self.conv1_fwd(frames, w, b, scale, out)
        else:
            self.conv1_fwd(frames[:rows_first], w, b, scale, out[:rows_first])
            self.conv1_fwd(frames[rows_first:], w2, b2, scale, out[rows_first:])

    def conv_fwd(self, x, w, b, stride, out, w2=None, b2=None, rows_first=0):
        if w2 is None:
            out.copy_(R.conv_fwd(x, w, b, stride, self.dtype))
        else:
            out[:rows_first].copy_(R.conv_fwd(x[:rows_first], w, b, stride, self.dtype))
            out[rows_first:].copy_(R.conv_fwd(x[rows_first:], w2, b2, stride, self.dtype))

    def fc_fwd(self, x, w, b, out, w2=None, b2=None, rows_first=0):
        x = x.reshape(x.shape[0], -1)
        if w2 is None:
            out.copy_(R.fc_fwd(x, w, b, self.dtype))
        else:
            out[:rows_first].copy_(R.fc_fwd(x[:rows_first], w, b, self.dtype))
            out[rows_first:].copy_(R.fc_fwd(x[rows_first:], w2, b2, self.dtype))

    # ---------------------------------------------------------------- head
    def head(self, Hon, Htg, Pon: Dict[str, torch.Tensor], Ptg: Dict[str, torch.Tensor], act, rew, gam, isw,
             huber: bool, kappa: float, grad_scale: float, td_abs, loss, dH, dhead, q_out=None,
             zero: Optional[torch.Tensor] = None, prio=None):
        """``prio = (replay, idx, gen)``: also write the batch's priorities back
        (the HIP backend fuses it into the head kernel)."""
        B = act.shape[0]
        A = Pon["wa"].shape[0]
        Hon = Hon.float()
        Htg = Htg.float()

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
        dH.copy_(dh)
        if q_out is not None:
            q_out.copy_(q_t)
        if zero is not None:
            zero.zero_()
        if prio is not None:
            prio[0].update_priorities(prio[1], td_abs, prio[2])

    def head_wgrad(self, Hon, dhead, g: Dict[str, torch.Tensor], prio=None):
        """``prio = (replay, idx, gen, td_abs)``: also write the batch's priorities back
        (the HIP backend runs it as one extra block of the same launch)."""
        if prio is not None:
            prio[0].update_priorities(prio[1], prio[3], prio[2])
        B = dhead.shape[0]
        HS = g["wv"].numel()
        h = Hon[:B].float()
        g["wv"].add_(dhead[:, 0] @ h[:, :HS])
        g["bv"].add_(dhead[:, 0].sum().view(1))
        g["wa"].add_(dhead[:, 1:].t() @ h[:, HS:])
        g["ba"].add_(dhead[:, 1:].sum(0))

    def actor_head(self, H, P, eps, ctr, seed, q_out, a_out):
        """Dueling q + epsilon-greedy per row (the oracle of csrc actor_head_kernel)."""
        h = H.float()
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

    def fc_dgrad(self, dh, x, w, dx_out):
        """dx = (dh @ w) * (x > 0) (x = the ReLU'd fc input)."""
        xf = x.reshape(x.shape[0], -1)
        dx, _, _ = R.fc_bwd(dh, xf, w, xf, self.dtype)
        dx_out.copy_(dx.reshape(dx_out.shape))

    def fc_wgrad(self, dh, x, dw_out, db_out, norm=None):
        xf = x.reshape(x.shape[0], -1)
        dw_out.copy_(dh.t().float() @ xf.float())
        db_out.copy_(dh.float().sum(0))
        return 0

    def fc_head_wgrad(self, dh, x, dw_out, db_out, Hon, dhead, g_head, prio, norm=None) -> int:
        """fc weight gradient + head weight gradient (+ the priority write-back,
        ``prio = (replay, idx, gen, td_abs)``); returns the fc norm slots used."""
        self.head_wgrad(Hon, dhead, g_head, prio=prio)
        return self.fc_wgrad(dh, x, dw_out, db_out, norm=norm) or 0

    def finalize_grads(self, jobs, norm_range=None, norm=None) -> int:
        """Deferred split-K reductions (the torch path computes gradients directly)."""
        return 0

    def conv_dgrad(self, dy, w, stride, x_src, dx_out):
        dx_out.copy_(R.conv_dgrad(dy, w, tuple(x_src.shape), stride, x_src, self.dtype))

    def conv_wgrad(self, dy, x, k, stride, dw_out, db_out, jobs=None):
        dw, db = R.conv_wgrad(dy, x, k, stride)
        dw_out.copy_(dw)
        db_out.copy_(db)

    def conv1_wgrad(self, dy, frames, scale, dw_out, db_out):
        dw, db = R.conv1_wgrad(dy, frames, scale)
        dw_out.copy_(dw)
        db_out.copy_(db)

    def conv1_wgrad_ring(self, dy, ring, slots, frames_buf, scale, dw_out, db_out, jobs=None):
        self.conv1_wgrad(dy, frames_buf[:slots.shape[0]], scale, dw_out, db_out)

    # ----------------------------------------------------------- optimizer
    def optimizer(self, p32, g32, v, m, pbf, lr, alpha, eps, clip, centered, partials, norm_out, norm_total=None,
                  sample=None):
        """``sample = (replay, B, out, ratio_min_global, nxt2)``: also draw the next
        batch after the update (the HIP backend fuses it into the optimizer launch)."""
        self._optimizer(p32, g32, v, m, pbf, lr, alpha, eps, clip, centered, norm_out)
        if sample is not None:
            rp, B, out, ratio, nxt2 = sample
            rp.sample(B, out=out, ratio_min_global=ratio, nxt2=nxt2)

    def _optimizer(self, p32, g32, v, m, pbf, lr, alpha, eps, clip, centered, norm_out):
        norm = g32.double().pow(2).sum().sqrt().float()
        coef = torch.clamp(clip / (norm + 1e-6), max=1.0) if clip > 0 else torch.ones_like(norm)
        g = g32 * coef
        v.mul_(alpha).add_((1 - alpha) * g * g)
        if centered:
            m.mul_(alpha).add_((1 - alpha) * g)
            var = v - m * m
        else:
            var = v
        p32.sub_(lr * g / (var.clamp_min(0).sqrt() + eps))
        pbf.copy_(p32)
        norm_out.copy_(norm.view(1))

    def gather_frames(self, replay, slots, out):
        replay.gather_frames(slots, out)


class HipBackend(TorchBackend):
    """MI355X backend.  Ops without a hand-written kernel yet run on torch
    (MIOpen / hipBLASLt) in bf16; each kernel family switches on here as it
    lands (``kernels`` lists what is native)."""

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
    # prepare(): nothing to do -- the dgrad GEMMs read the natural weight tensors
    # K-major (transposed LDS reads) and conv1 reads OIHW w1 directly.

    def conv1_fwd_ring(self, ring, slots, frames_buf, w, b, scale, out, w2=None, b2=None, rows_first=0):
        if not self.native_conv:
            return super().conv1_fwd_ring(ring, slots, frames_buf, w, b, scale, out, w2, b2, rows_first)
        C.conv1_s2d_fwd(self.lib, self.ws, ring, slots, w, b, scale, out, w2, b2, rows_first)

    def conv_fwd(self, x, w, b, stride, out, w2=None, b2=None, rows_first=0):
        if not self.native_conv:
            return super().conv_fwd(x, w, b, stride, out, w2, b2, rows_first)
        C.conv_fwd(self.lib, x, w, b, stride, out, w2, b2, rows_first)

    def fc_fwd(self, x, w, b, out, w2=None, b2=None, rows_first=0):
        if not self.native_conv:
            return super().fc_fwd(x, w, b, out, w2, b2, rows_first)
        C.dense_fwd(self.lib, x.reshape(x.shape[0], -1), w, b, out, relu=True, w2=w2, b2=b2,
                    rows_first=rows_first, ws=self.ws)

    def fc_dgrad(self, dh, x, w, dx_out):
        if not self.native_conv:
            return super().fc_dgrad(dh, x, w, dx_out)
        xf = x.reshape(x.shape[0], -1)
        C.dense_dgrad(self.lib, dh, w, dx_out.reshape(dh.shape[0], -1), xf)

    def fc_wgrad(self, dh, x, dw_out, db_out, norm=None):
        if not self.native_conv:
            return super().fc_wgrad(dh, x, dw_out, db_out)
        return C.dense_wgrad(self.lib, dh, x.reshape(x.shape[0], -1), dw_out, db_out, norm=norm)

    def fc_head_wgrad(self, dh, x, dw_out, db_out, Hon, dhead, g_head, prio, norm=None) -> int:
        if self.native_conv and prio is not None and prio[0].use_hip:
            rp, idx, gen, td = prio
            r = C.dense_wgrad_head_prio(self.lib, dh, x.reshape(x.shape[0], -1), dw_out, db_out, norm, Hon, dhead,
                                        g_head, rp, idx, gen, td)
            if r is not None:
                return r
        return super().fc_head_wgrad(dh, x, dw_out, db_out, Hon, dhead, g_head, prio, norm)

    def finalize_grads(self, jobs, norm_range=None, norm=None) -> int:
        """Returns the number of squared-norm partial slots written (``slot0`` + blocks)."""
        if not jobs and norm is None:
            return 0
        if norm is None:
            C.finalize_grads(self.lib, jobs)
            return 0
        return norm["slot0"] + C.finalize_grads(self.lib, jobs, norm_range, norm["part"], norm["slot0"],
                                                norm.get("total"))

    def conv_dgrad(self, dy, w, stride, x_src, dx_out):
        if not self.native_conv:
            return super().conv_dgrad(dy, w, stride, x_src, dx_out)
        if stride == 1:
            C.conv3_dgrad(self.lib, dy, w, x_src, dx_out)
        else:
            C.conv2_dgrad(self.lib, dy, w, x_src, dx_out)

    def conv_wgrad(self, dy, x, k, stride, dw_out, db_out, jobs=None):
        if not self.native_conv:
            return super().conv_wgrad(dy, x, k, stride, dw_out, db_out)
        C.conv_wgrad(self.lib, self.ws, dy, x, k, stride, dw_out, db_out, jobs=jobs)

    def conv1_wgrad_ring(self, dy, ring, slots, frames_buf, scale, dw_out, db_out, jobs=None):
        if not self.native_conv:
            return super().conv1_wgrad_ring(dy, ring, slots, frames_buf, scale, dw_out, db_out)
        C.conv1_wgrad_ring(self.lib, self.ws, dy, ring, slots, scale, dw_out, db_out, jobs=jobs)

    @staticmethod
    def _hp(P):
        h = _lib.HeadParams()
        h.wv, h.bv, h.wa, h.ba = (P["wv"].data_ptr(), P["bv"].data_ptr(), P["wa"].data_ptr(),
                                  P["ba"].data_ptr())
        return h

    def head(self, Hon, Htg, Pon, Ptg, act, rew, gam, isw, huber, kappa, grad_scale, td_abs, loss, dH,
             dhead, q_out=None, zero=None, prio=None):
        B = act.shape[0]
        A = Pon["wa"].shape[0]
        args = (Hon.data_ptr(), Htg.data_ptr(), self._hp(Pon), self._hp(Ptg), act.data_ptr(), rew.data_ptr(),
                gam.data_ptr(), _lib.ptr(isw), B, A, int(huber), float(kappa), float(grad_scale),
                td_abs.data_ptr(), loss.data_ptr(), _lib.ptr(q_out), dH.data_ptr(), dhead.data_ptr(),
                _lib.ptr(zero), 0 if zero is None else zero.numel(), Pon["wv"].numel())
        if prio is not None and prio[0].use_hip:
            # priority write-back in the head kernel (csrc/sumtree.hip: ddqn_head_prio_kernel)
            _lib.check(self.lib.apex_ddqn_head_prio(*args, *prio[0].prio_launch_args(prio[1], prio[2]),
                                                    _lib.stream_ptr()), "ddqn_head_prio")
            return
        _lib.check(self.lib.apex_ddqn_head(*args, _lib.stream_ptr()), "ddqn_head")
        if prio is not None:
            prio[0].update_priorities(prio[1], td_abs, prio[2])

    def head_wgrad(self, Hon, dhead, g, prio=None):
        B, A1 = dhead.shape
        if prio is not None and prio[0].use_hip and B <= 1024:
            rp, idx, gen, td = prio
            _lib.check(self.lib.apex_head_wgrad_prio(
                Hon.data_ptr(), dhead.data_ptr(), B, A1 - 1, g["wv"].data_ptr(), g["bv"].data_ptr(),
                g["wa"].data_ptr(), g["ba"].data_ptr(), g["wv"].numel(), rp.tree_desc(), idx.data_ptr(),
                td.data_ptr(), _lib.ptr(gen), rp.gen.data_ptr(), rp.alpha, rp.eps, rp.ctr.data_ptr(),
                _lib.stream_ptr()), "head_wgrad_prio")
            return
        if prio is not None:
            prio[0].update_priorities(prio[1], prio[3], prio[2])
        _lib.check(self.lib.apex_head_wgrad(Hon.data_ptr(), dhead.data_ptr(), B, A1 - 1, g["wv"].data_ptr(),
                                            g["bv"].data_ptr(), g["wa"].data_ptr(), g["ba"].data_ptr(),
                                            g["wv"].numel(), _lib.stream_ptr()), "head_wgrad")

    def actor_head(self, H, P, eps, ctr, seed, q_out, a_out):
        E, A = q_out.shape
        _lib.check(self.lib.apex_actor_head(H.data_ptr(), self._hp(P), E, A, eps.data_ptr(), int(seed),
                                            ctr.data_ptr(), q_out.data_ptr(), a_out.data_ptr(),
                                            P["wv"].numel(), _lib.stream_ptr()), "actor_head")

    def optimizer(self, p32, g32, v, m, pbf, lr, alpha, eps, clip, centered, partials, norm_out, norm_total=None,
                  sample=None):
        n = p32.numel()
        st = _lib.stream_ptr()
        if sample is not None and sample[0].use_hip:
            # the next batch's draw rides in the optimizer launch (csrc/sumtree.hip: rmsprop_sample_kernel)
            rp, B, out, ratio, nxt2 = sample
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
                *rp.sample_launch_args(B, out, ratio, nxt2), st), "rmsprop_sample")
            return
        if sample is not None:
            self.optimizer(p32, g32, v, m, pbf, lr, alpha, eps, clip, centered, partials, norm_out, norm_total)
            rp, B, out, ratio, nxt2 = sample
            rp.sample(B, out=out, ratio_min_global=ratio, nxt2=nxt2)
            return
        if norm_total is not None:   # squared norm already summed by the gradient producers
            part, npart = norm_total if isinstance(norm_total, tuple) else (norm_total, 1)
            _lib.check(self.lib.apex_rmsprop_step_np(p32.data_ptr(), g32.data_ptr(), v.data_ptr(), m.data_ptr(),
                                                     pbf.data_ptr(), n, part.data_ptr(), npart, float(lr),
                                                     float(alpha), float(eps), float(clip), int(centered),
                                                     norm_out.data_ptr(), st), "rmsprop_np")
            return
        _lib.check(self.lib.apex_grad_sqnorm_partials(g32.data_ptr(), n, partials.data_ptr(), st), "sqnorm")
        _lib.check(self.lib.apex_rmsprop_step(p32.data_ptr(), g32.data_ptr(), v.data_ptr(), m.data_ptr(),
                                              pbf.data_ptr(), n, partials.data_ptr(), float(lr), float(alpha),
                                              float(eps), float(clip), int(centered), norm_out.data_ptr(), st),
                   "rmsprop")
