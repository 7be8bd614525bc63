"""GPU-resident learner for any image network (IMPALA-deep ResNet, nature32, ...).

The NatureCNN has the fully hand-written learner (``fused_learner.py``).  Every
other image network runs here with the same GPU-first structure:

* samples come from the HBM replay shard (``csrc/sumtree.hip`` sampling, frame
  gather straight from the uint8 ring) -- no host round trip;
* the network is a torch module whose parameters and gradients are VIEWS into
  one flat fp32 buffer each, so the clip + centered RMSprop step is the fused
  HIP optimizer kernel over the whole model (``csrc/optimizer.hip``) and the DP
  all-reduce is one flat RCCL call;
* forward/backward run in fp32 (``Runtime.dtype = fp32``, the reference's precision) or
  bf16 autocast (``bf16``) on MIOpen / hipBLASLt convs and GEMMs -- the vendor-library
  baseline the hand-written NatureCNN learner is measured against (``bench.py
  --learner graph``);
* the whole update -- sample, gather, 3 forwards, DDQN Huber*IS loss, backward,
  optimizer, priority write-back -- is captured in ONE HIP graph (two segments
  around the gradient all-reduce with data parallelism).

Reference semantics are those of ``learner.py:29-80`` with the defects fixed
(SURVEY Appendix A): terminal mask via Gamma, IS weights, Huber, centered
RMSprop with decay 0.95, target sync every ``q_target_sync_freq`` steps.
"""
from __future__ import annotations

import copy
from typing import Dict, List, Optional

import torch

from ..config import ApexConfig
from ..models.dueling import build_network
from ..ops.fused_ops import HipBackend, TorchBackend
from ..utils.checkpoint import (adopt_obs_scale, checkpoint_network, load_checkpoint, pack_flat_state, save_checkpoint,
                                unpack_flat_state)
from .fused_learner import _enable_sharding, dp_layout
from .losses import ddqn_loss


def _flatten_module(module: torch.nn.Module, device) -> torch.Tensor:
    """Move every parameter of ``module`` into one contiguous fp32 buffer (params
    become views of it).  Returns the buffer."""
    params = list(module.parameters())
    n = sum(p.numel() for p in params)
    flat = torch.zeros(n, dtype=torch.float32, device=device)
    off = 0
    for p in params:
        k = p.numel()
        flat[off:off + k].copy_(p.data.reshape(-1))
        p.data = flat[off:off + k].view_as(p)
        off += k
    return flat


class GraphLearner:
    kind = "graph"

    def __init__(self, cfg: ApexConfig, device, replay, comm=None, batch_size: Optional[int] = None):
        self.cfg = cfg
        self.rt = cfg.Runtime
        self.device = torch.device(device)
        self.replay = replay
        self.comm = comm
        self.world, _, self.B, self.mcap = dp_layout(cfg, comm, batch_size, allow_force=False)
        self.C = cfg.frame_stack
        self.A = int(cfg.env_conf.action_dim)
        d = self.device
        self.Q = build_network(cfg.network, cfg.env_conf.state_shape, self.A, obs_scale=self.rt.obs_scale).to(d)
        self.p32 = _flatten_module(self.Q, d)
        if comm is not None and comm.world_size > 1:
            comm.broadcast_flat(self.p32)
        self.g32 = torch.zeros_like(self.p32)
        for p, g in zip(self.Q.parameters(), self._views(self.g32)):
            p.grad = g
        self.Q_target = copy.deepcopy(self.Q)
        for p in self.Q_target.parameters():
            p.requires_grad_(False)
        self.t32 = _flatten_module(self.Q_target, d)
        self.rms_v = torch.zeros_like(self.p32)
        self.rms_m = torch.zeros_like(self.p32)
        self.pbf = torch.zeros(self.p32.numel(), dtype=torch.bfloat16, device=d)
        self.partials = torch.zeros(1024, dtype=torch.float64, device=d)
        self.gnorm = torch.zeros(1, dtype=torch.float32, device=d)
        self.ops = HipBackend(native_conv=False) if (d.type == "cuda" and self.rt.use_hip_kernels) else \
            TorchBackend(torch.float32)
        # fp32: plain fp32 library kernels (gfx950 has no xf32 / TF32 path); bf16: autocast
        self.amp_dtype = torch.bfloat16 if (d.type == "cuda" and self.rt.dtype == "bf16") else None
        self.graph_captures = 0
        self.S = replay.alloc_sample_buffers(self.B)
        self.td_abs = torch.zeros(self.B, dtype=torch.float32, device=d)
        self.loss_b = torch.zeros(1, dtype=torch.float32, device=d)
        # DP: one global prioritized replay over the rank shards (see fused_learner)
        self._isw = bool(self.rt.use_is_weights) or self.world > 1
        # batch-max IS normalisation (learner/is_norm.py): the loss keeps the sampler's
        # global-min weights, the optimizer divides the gradient by the batch's largest
        # (p / p_min)^-beta (with DP its max over the ranks, all-reduced beside the gradient)
        self._is_bmax = bool(self.rt.use_is_weights) and self.rt.is_normalise == "batch_max"
        self.wmax = torch.zeros(1, dtype=torch.float64, device=d)
        if self.world > 1:
            _enable_sharding(replay, comm, self.rt, self.mcap)
            replay.gather_shard_stats()
        self.num_q_updates = 0
        self._graphs: Optional[List[torch.cuda.CUDAGraph]] = None
        ls = cfg.Learner.load_saved_state
        if ls:
            self.load(ls)

    def _views(self, flat: torch.Tensor) -> List[torch.Tensor]:
        out, off = [], 0
        for p in self.Q.parameters():
            k = p.numel()
            out.append(flat[off:off + k].view_as(p))
            off += k
        return out

    # ---------------------------------------------------------------- step
    def _forward_backward(self) -> None:
        rt, B = self.rt, self.B
        S = self.replay.sample(B, out=self.S)
        obs = self.replay.gather_frames(S["obs"])
        nxt = self.replay.gather_frames(S["nxt"])
        self.g32.zero_()
        # cache_enabled=False: autocast's weight-cast cache must not outlive a graph capture
        amp = torch.autocast(device_type="cuda", dtype=self.amp_dtype, cache_enabled=False) \
            if self.amp_dtype is not None else torch.autocast(device_type=self.device.type, enabled=False)
        with amp:
            q_t = self.Q(obs)[2]
            with torch.no_grad():
                q_n = self.Q(nxt)[2]
                q_g = self.Q_target(nxt)[2]
        w = S["weights"] if self._isw else None
        if self._is_bmax:
            self.wmax.copy_(S["weights"].max().double() / S["wscale"].double().clamp_min(1e-30))
        loss, td = ddqn_loss(q_t.float(), q_n.float(), q_g.float(), S["act"], S["rew"], S["gam"], w,
                             loss=rt.loss, kappa=rt.huber_delta)
        (loss / self.world).backward()     # SUM all-reduce of 1/world-scaled grads = mean
        self.td_abs.copy_(td)
        self.loss_b.copy_(loss.detach().view(1))

    def _apply(self) -> None:
        rt = self.rt
        self.ops.optimizer(self.p32, self.g32, self.rms_v, self.rms_m, self.pbf, rt.lr, rt.rms_decay, rt.rms_eps,
                           rt.grad_clip, rt.centered_rmsprop, self.partials, self.gnorm,
                           wnorm=(self.wmax, 1, 1) if self._is_bmax else None)
        self.replay.update_priorities(self.S["idx"], self.td_abs, self.S["gen"])

    def _allreduce(self) -> None:
        import torch.distributed as dist
        dist.all_reduce(self.g32, op=dist.ReduceOp.SUM)
        if self._is_bmax:
            dist.all_reduce(self.wmax, op=dist.ReduceOp.MAX)

    def _capture(self) -> None:
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        snap = [t.clone() for t in (self.p32, self.rms_v, self.rms_m, self.replay.leaf, self.replay.nodes,
                                    self.replay.min_bits, self.replay.ctr)]
        with torch.cuda.stream(s):
            for _ in range(2):
                self._forward_backward()
                if self.world > 1:
                    self._allreduce()
                self._apply()
        torch.cuda.current_stream(self.device).wait_stream(s)
        for dst, src in zip((self.p32, self.rms_v, self.rms_m, self.replay.leaf, self.replay.nodes,
                             self.replay.min_bits, self.replay.ctr), snap):
            dst.copy_(src)
        torch.cuda.synchronize(self.device)
        segs = [self._forward_backward, self._apply] if self.world > 1 else \
            [lambda: (self._forward_backward(), self._apply())]
        self._graphs = []
        for seg in segs:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                seg()
            self._graphs.append(g)
            self.graph_captures += 1

    def prepare_graphs(self, multi: bool = True) -> int:
        """Capture the step's graphs now (outside any timed region)."""
        if self.rt.use_graphs and self.device.type == "cuda" and self._graphs is None:
            self._capture()
        return self.graph_captures

    def step(self) -> None:
        graphs = self.rt.use_graphs and self.device.type == "cuda"
        if graphs and self._graphs is None:
            self._capture()
        if graphs:
            self._graphs[0].replay()
            if self.world > 1:
                self._allreduce()
                self._graphs[1].replay()
        else:
            self._forward_backward()
            if self.world > 1:
                self._allreduce()
            self._apply()
        if self.world > 1:
            self.replay.gather_shard_stats()
        self.num_q_updates += 1
        if self.num_q_updates % self.cfg.Learner.q_target_sync_freq == 0:
            self.sync_target()

    # --------------------------------------------------- replay statistics
    def refresh_replay_stats(self) -> bool:
        """Re-gather the shard statistics (a collective).  Fixed rows: never resizes."""
        if self.world > 1:
            self.replay.gather_shard_stats()
        return False

    def sync_target(self) -> None:
        self.t32.copy_(self.p32)

    # ------------------------------------------------------------- metrics
    def last_metrics(self) -> Dict[str, float]:
        w = float(self.S["weights"].mean()) if self._isw else 1.0
        if self._is_bmax:    # the effective weights: the optimizer divides the gradient by wmax
            wm = float(self.wmax[0])
            w = w / wm if wm > 0 else w
        return {"loss": float(self.loss_b[0]), "td_abs_mean": float(self.td_abs.mean()),
                "grad_norm": float(self.gnorm[0]), "is_weight_mean": w}

    def profile_step(self) -> Dict[str, float]:
        if self.device.type != "cuda":
            return {}
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        self.step()
        e1.record()
        torch.cuda.synchronize(self.device)
        return {"total": e0.elapsed_time(e1)}

    # ------------------------------------------------------------------ io
    def actor_forward(self, net: torch.nn.Module, frames: torch.Tensor) -> torch.Tensor:
        amp = torch.autocast(device_type="cuda", dtype=self.amp_dtype) if self.amp_dtype is not None \
            else torch.autocast(device_type=self.device.type, enabled=False)
        with torch.no_grad(), amp:
            return net(frames)[2].float()

    def _segments(self):
        """(parameter name, flat offset, numel) of the flat buffers (module parameter order)."""
        out, o = [], 0
        for name, p in self.Q.named_parameters():
            out.append((name, o, p.numel()))
            o += p.numel()
        return out

    def save(self, path: str, extra: Optional[Dict] = None) -> None:
        save_checkpoint(path, self.Q.state_dict(), Q_target_state=self.Q_target.state_dict(),
                        optimizer_state=pack_flat_state(self._segments(), rms_v=self.rms_v, rms_m=self.rms_m),
                        num_q_updates=self.num_q_updates, config=self.cfg.to_dict(),
                        rng={"replay_ctr": int(self.replay.ctr.item()), "replay_seed": int(self.replay.seed)},
                        **(extra or {}))

    def load(self, path: str) -> bool:
        ck = load_checkpoint(path)
        if ck is None:
            return False
        if adopt_obs_scale(ck, self.rt):
            for net in (self.Q, self.Q_target):
                if hasattr(net, "pre"):
                    net.pre.scale = self.rt.obs_scale
            self._graphs = None
        with torch.no_grad():
            for p, v in zip(self.Q.state_dict().values(), ck["Q_state"].values()):
                p.copy_(v)
            if "Q_target_state" in ck:
                for p, v in zip(self.Q_target.state_dict().values(), ck["Q_target_state"].values()):
                    p.copy_(v)
            else:
                self.sync_target()
            unpack_flat_state(ck.get("optimizer_state"), self._segments(), untagged_network=checkpoint_network(ck),
                              network=self.cfg.network, rms_v=self.rms_v, rms_m=self.rms_m)
        self.num_q_updates = int(ck.get("num_q_updates", 0))
        rng = ck.get("rng")
        if isinstance(rng, dict) and "replay_ctr" in rng:
            self.replay.ctr.fill_(int(rng["replay_ctr"]))
        return True
