"""Generic learner over any dueling ``nn.Module`` (CPU path, MLP/IMPALA nets,
and the correctness oracle for the fused MI355X learner).

Reference parity: ``Learner`` (``learner.py:10-80``) -- double-DQN loss
(:29-52), optimizer step + target sync (:54-61), checkpoint load (:18-23).
Fixed: target net starts as a copy of the online net (A30), target sync on
``n % freq == 0`` (A17), centered RMSprop with decay 0.95 (A16), grad-norm
clip, Huber + IS weights (A18), no ``requires_grad_`` on inputs (A20).
Data parallel: gradients are all-reduced across ranks
(``parallel/dist.py``) before the optimizer step.
"""
from __future__ import annotations

import copy
from typing import Any, Dict, Optional

import numpy as np
import torch

from ..config import ApexConfig
from ..models.dueling import build_network
from ..utils.checkpoint import adopt_obs_scale, load_checkpoint, save_checkpoint
from .losses import ddqn_loss


def make_optimizer(params, rt) -> torch.optim.Optimizer:
    return torch.optim.RMSprop(params, lr=rt.lr, alpha=rt.rms_decay, eps=rt.rms_eps,
                               centered=rt.centered_rmsprop)


class TorchLearner:
    def __init__(self, cfg: ApexConfig, device: torch.device, comm=None):
        self.cfg = cfg
        self.rt = cfg.Runtime
        self.device = torch.device(device)
        self.comm = comm
        shape = cfg.env_conf.state_shape
        self.Q = build_network(cfg.network, shape, cfg.env_conf.action_dim,
                               obs_scale=self.rt.obs_scale).to(self.device)
        if comm is not None and comm.world_size > 1:
            comm.broadcast_module(self.Q)
        self.Q_target = copy.deepcopy(self.Q)
        for p in self.Q_target.parameters():
            p.requires_grad_(False)
        self.optimizer = make_optimizer(self.Q.parameters(), self.rt)
        self.num_q_updates = 0
        ls = cfg.Learner.load_saved_state
        if ls:
            self.load(ls)

    # ---------------------------------------------------------------- io
    def _to(self, x, dtype=None):
        t = torch.as_tensor(x)
        if dtype is not None:
            t = t.to(dtype)
        return t.to(self.device, non_blocking=True)

    def q_values(self, obs) -> torch.Tensor:
        with torch.no_grad():
            return self.Q(self._to(obs))[2]

    # -------------------------------------------------------------- step
    def compute_loss_and_priorities(self, batch: Dict[str, Any]):
        S_t = self._to(batch["S_t"])
        S_tpn = self._to(batch["S_tpn"])
        A = self._to(batch["A_t"], torch.long)
        R = self._to(batch["R"], torch.float32)
        G = self._to(batch["Gamma"], torch.float32)
        w = self._to(batch["weights"], torch.float32) if (
            self.rt.use_is_weights and "weights" in batch) else None
        with torch.no_grad():
            q_next_online = self.Q(S_tpn)[2]
            q_next_target = self.Q_target(S_tpn)[2]
        q_t = self.Q(S_t)[2]
        return ddqn_loss(q_t, q_next_online, q_next_target, A, R, G, w,
                         loss=self.rt.loss, kappa=self.rt.huber_delta)

    def update_Q(self, loss: torch.Tensor) -> float:
        self.optimizer.zero_grad(set_to_none=False)
        loss.backward()
        if self.comm is not None and self.comm.world_size > 1:
            self.comm.allreduce_grads([p.grad for p in self.Q.parameters()])
        gnorm = 0.0
        if self.rt.grad_clip and self.rt.grad_clip > 0:
            gnorm = float(torch.nn.utils.clip_grad_norm_(self.Q.parameters(), self.rt.grad_clip))
        self.optimizer.step()
        self.num_q_updates += 1
        if self.num_q_updates % self.cfg.Learner.q_target_sync_freq == 0:
            self.sync_target()
        return gnorm

    def sync_target(self) -> None:
        self.Q_target.load_state_dict(self.Q.state_dict())

    def step(self, batch: Dict[str, Any]) -> Dict[str, Any]:
        loss, td = self.compute_loss_and_priorities(batch)
        gnorm = self.update_Q(loss)
        return {"loss": float(loss.detach()), "td_abs": td.cpu().numpy(), "grad_norm": gnorm}

    # --------------------------------------------------------- params
    def state_dict_for_actors(self) -> Dict[str, torch.Tensor]:
        return {k: v.detach() for k, v in self.Q.state_dict().items()}

    def save(self, path: str, extras: bool = True) -> None:
        ex: Dict[str, Any] = {}
        if extras:
            ex = dict(Q_target_state=self.Q_target.state_dict(),
                      optimizer_state=self.optimizer.state_dict(),
                      num_q_updates=self.num_q_updates,
                      config=self.cfg.to_dict())
        save_checkpoint(path, self.Q.state_dict(), **ex)

    def load(self, path: str) -> bool:
        ck = load_checkpoint(path)
        if ck is None:
            return False
        if adopt_obs_scale(ck, self.rt):
            for net in (self.Q, self.Q_target):
                if hasattr(net, "pre"):
                    net.pre.scale = self.rt.obs_scale
        self.Q.load_state_dict(ck["Q_state"])
        if "Q_target_state" in ck:
            self.Q_target.load_state_dict(ck["Q_target_state"])
        else:
            self.sync_target()
        if "optimizer_state" in ck:
            self.optimizer.load_state_dict(ck["optimizer_state"])
        self.num_q_updates = int(ck.get("num_q_updates", 0))
        return True
