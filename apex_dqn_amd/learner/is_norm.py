"""Importance-sampling weight normalisation shared by the fused learners.

The reference exposes ``importance_sampling_exponent`` (beta,
``parameters.json:30``) but never uses it (``replay.py:8-16``, defect A18).  The
samplers here write w_i = (p_i / p_min)^-beta, i.e. the weights normalised by
their maximum over the WHOLE replay (the global minimum priority).  With the
default priority floor (``Runtime.priority_eps`` = 1e-6) one stale leaf near the
floor makes every weight tiny: the mean weight of a live run was 0.036, an update
~28x smaller than the configured learning rate.

``Runtime.is_normalise = "batch_max"`` (default) divides instead by the largest
weight of the sampled batch -- the PER / Ape-X papers' ``1 / max_i w_i`` over the
minibatch; with data parallelism, over the GLOBAL batch of all ranks.  The loss
is linear in the weights, so the learners keep the global-min weights in the loss
kernel and divide the *gradient* by m = max_j (p_j / p_min)^-beta once, inside the
optimizer launch, before the clip:

* the head kernel (``csrc/ddqn_head.hip`` ``IsNorm``) leaves m of its local batch
  -- one rank: in ``wmax``; DP: in this rank's slot of the replay-shard statistics
  (``GpuReplayShard.local_stats[2]``), which the step all-gathers anyway;
* the optimizer (``csrc/rmsprop_common.h`` ``is_grad_scale``) takes the max over
  the ranks' slots and scales the gradient (and its clip norm) by 1 / m.

No extra collective, launch or pass over the weights.  ``global_min`` keeps the
old normalisation.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch


class IsNormMixin:
    """Needs ``self.rt``, ``self.replay``, ``self.S`` (sample buffers with
    ``weights`` / ``wscale``), ``self.device`` and ``self._dp`` / ``self.world``."""

    def _init_is_norm(self) -> None:
        self._is_bmax = bool(self.rt.use_is_weights) and self.rt.is_normalise == "batch_max"
        self.wmax = torch.zeros(1, dtype=torch.float64, device=self.device)
        # DP: rows this rank drew, summed over steps by the head kernel (the global batch of
        # a DP step is M = sum over ranks <= W B; bench.py reports it)
        self.valid_rows_total = torch.zeros(1, dtype=torch.int64, device=self.device)

    def _isn(self):
        """(wscale, out, valid counter) for the head kernel, or None."""
        sharded = self.replay.sharded
        if not self._is_bmax and not sharded:
            return None
        out = None
        if self._is_bmax:
            out = self.replay.local_stats[2:3] if sharded else self.wmax
        return (self.S["wscale"], out, self.valid_rows_total if sharded else None)

    def _wnorm(self) -> Optional[Tuple[torch.Tensor, int, int]]:
        """(stats, n, stride) the optimizer reads the normaliser from, or None."""
        if not self._is_bmax:
            return None
        if self.replay.sharded:
            from ..replay.gpu_replay import SHARD_STATS
            return (self.replay.shard_stats[2:], self.replay.shard_world, SHARD_STATS)
        return (self.wmax, 1, 1)

    def is_scale(self) -> float:
        """1 / (batch-max normaliser) of the last step (1 with global_min)."""
        wn = self._wnorm()
        if wn is None:
            return 1.0
        m = float(wn[0].reshape(-1)[0:wn[1] * wn[2]:wn[2]].max())
        return 1.0 / m if m > 0 else 1.0

    def _is_metrics(self) -> Dict[str, float]:
        """Loss / |delta| / IS-weight means over the rows this rank actually drew (with
        DP the rest belong to other shards and carry weight 0)."""
        sc = self.is_scale()
        w = self.S["weights"]
        sharded = self.replay.sharded
        valid = (w > 0) if sharded else torch.ones_like(w, dtype=torch.bool)
        nv = max(int(valid.sum()), 1)
        return {"loss": float(self.loss_b.sum()) * sc / nv,
                "td_abs_mean": float(self.td_abs[valid].sum()) / nv,
                "grad_norm": float(self.gnorm[0]),
                "is_weight_mean": float(w[valid].sum()) * sc / nv,
                "valid_rows": int(valid.sum())}
