"""Double-DQN n-step loss (PyTorch oracle).

Reference ``learner.py:29-52`` computes ``G = R + Gamma * Q_double(S_tpn)[argmax Q(S_tpn)]``
and ``0.5*delta^2`` with no terminal mask, no IS weights and a broken
priority dict.  This module is the intended version:
terminal masking through Gamma=0 (set by the n-step builder), Huber (or
0.5*delta^2 for parity) weighted by IS weights, one |delta| per sample.
The fused HIP head kernel (``ops/kernels.py::ddqn_head``) is tested against
this function.
"""
from __future__ import annotations

from typing import Tuple

import torch


def huber(delta: torch.Tensor, kappa: float = 1.0) -> torch.Tensor:
    a = delta.abs()
    return torch.where(a <= kappa, 0.5 * delta * delta, kappa * (a - 0.5 * kappa))


def ddqn_targets(q_online_next: torch.Tensor, q_target_next: torch.Tensor,
                 R: torch.Tensor, Gamma: torch.Tensor) -> torch.Tensor:
    a_star = q_online_next.argmax(dim=1, keepdim=True)
    return R + Gamma * q_target_next.gather(1, a_star).squeeze(1)


def ddqn_loss(q_online_t: torch.Tensor, q_online_next: torch.Tensor,
              q_target_next: torch.Tensor, A: torch.Tensor, R: torch.Tensor,
              Gamma: torch.Tensor, weights: torch.Tensor = None, loss: str = "huber",
              kappa: float = 1.0) -> Tuple[torch.Tensor, torch.Tensor]:
    """Return (scalar loss, |delta| per sample)."""
    with torch.no_grad():
        G = ddqn_targets(q_online_next.float(), q_target_next.float(), R.float(), Gamma.float())
    q_sa = q_online_t.float().gather(1, A.long().view(-1, 1)).squeeze(1)
    delta = G - q_sa
    per = huber(delta, kappa) if loss == "huber" else 0.5 * delta * delta
    if weights is not None:
        per = per * weights.float()
    return per.mean(), delta.detach().abs()
