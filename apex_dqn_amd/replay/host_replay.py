"""CPU prioritized replay (CartPole / CPU configs and the semantic oracle for
the HBM shard).

Reference parity (``replay.py:8-84``): ``add`` (:59), ``sample`` (:44),
``set_priorities`` (:32), ``remove_to_fit`` (:71, FIFO to ``soft_capacity``),
``size`` (:82).  Intended semantics instead of the
defects: P(i) = p_i^alpha / sum p^alpha through a sum-tree, IS weights
w_i = (N P(i))^-beta / max_j w_j (``importance_sampling_exponent`` is never
read by the reference) -- max over the sampled batch (``is_normalise =
"batch_max"``, the default) or over the whole replay (``"global_min"``) -- and
eviction that also drops the priority (A5).
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np

from .sumtree import SumTree


def _make_tree(cap: int) -> SumTree:
    """C++ sum-tree (csrc/runtime) when the native runtime builds, numpy otherwise."""
    from ..runtime.native import make_sum_tree
    return make_sum_tree(cap)


class PrioritizedReplay:
    def __init__(self, soft_capacity: int, priority_exponent: float = 0.6,
                 importance_sampling_exponent: float = 0.4, capacity: Optional[int] = None,
                 priority_eps: float = 1e-6, seed: int = 0, is_normalise: str = "batch_max"):
        self.soft_capacity = int(soft_capacity)
        self.cap = int(capacity or max(soft_capacity + 1, int(soft_capacity * 1.25)))
        self.alpha = float(priority_exponent)
        self.beta = float(importance_sampling_exponent)
        self.eps = float(priority_eps)
        if is_normalise not in ("batch_max", "global_min"):
            raise ValueError("is_normalise must be 'batch_max' or 'global_min'")
        self.is_normalise = is_normalise
        self.tree = _make_tree(self.cap)
        self.rng = np.random.default_rng(seed)
        self.storage: Dict[str, np.ndarray] = {}
        self.head = 0
        self.live = 0
        self.total_inserted = 0

    # ------------------------------------------------------------ storage
    def _ensure_storage(self, batch: Dict[str, np.ndarray]) -> None:
        if self.storage:
            return
        for k, v in batch.items():
            if k == "priority":
                continue
            v = np.asarray(v)
            self.storage[k] = np.zeros((self.cap,) + v.shape[1:], v.dtype)

    def priority_to_leaf(self, p) -> np.ndarray:
        return (np.abs(np.asarray(p, np.float64)) + self.eps) ** self.alpha

    def add(self, batch: Dict[str, np.ndarray], priorities=None) -> np.ndarray:
        """Insert a batch of n-step transitions; returns the slots written."""
        self._ensure_storage(batch)
        n = len(batch["A_t"])
        if n == 0:
            return np.zeros(0, np.int64)
        if n > self.cap:
            batch = {k: np.asarray(v)[-self.cap:] for k, v in batch.items()}
            n = self.cap
        slots = (self.head + np.arange(n)) % self.cap
        for k, arr in self.storage.items():
            arr[slots] = batch[k]
        pr = batch.get("priority") if priorities is None else priorities
        if pr is None:
            # new experience without actor priority: max priority so it is seen once
            pr_leaf = np.full(n, max(self.tree.sum[self.tree.size2:].max(), 1.0))
        else:
            pr_leaf = self.priority_to_leaf(pr)
        self.tree.update(slots, pr_leaf)
        self.head = int((self.head + n) % self.cap)
        self.live = min(self.live + n, self.cap)
        self.total_inserted += n
        return slots

    def size(self) -> int:
        return int(self.live)

    def __len__(self) -> int:
        return self.size()

    # ----------------------------------------------------------- sampling
    def sample(self, batch_size: int) -> Dict[str, np.ndarray]:
        if self.live == 0:
            raise RuntimeError("replay is empty")
        idx = self.tree.sample_stratified(batch_size, self.rng)
        out = {k: arr[idx] for k, arr in self.storage.items()}
        p = self.tree.get(idx)
        total = self.tree.total
        pmin = self.tree.min_positive
        N = self.live
        prob = p / total
        w = (N * prob) ** (-self.beta)
        wmax = w.max() if self.is_normalise == "batch_max" else (N * pmin / total) ** (-self.beta)
        out["weights"] = (w / wmax).astype(np.float32)
        out["idx"] = idx.astype(np.int64)
        out["prob"] = prob.astype(np.float32)
        return out

    def set_priorities(self, idx, priorities) -> None:
        """Write back |delta|-based priorities for sampled slots."""
        idx = np.asarray(idx, np.int64)
        leaf = self.priority_to_leaf(priorities)
        # never resurrect a slot that was evicted after it was sampled
        alive = self.tree.get(idx) > 0
        self.tree.update(idx[alive], leaf[alive])

    update_priorities = set_priorities

    def remove_to_fit(self) -> int:
        """FIFO-evict down to ``soft_capacity`` (reference ``replay.py:71-80``)."""
        excess = self.live - self.soft_capacity
        if excess <= 0:
            return 0
        oldest = (self.head - self.live) % self.cap
        slots = (oldest + np.arange(excess)) % self.cap
        self.tree.update(slots, np.zeros(excess))
        self.live -= excess
        return int(excess)

    def state_dict(self) -> Dict[str, np.ndarray]:
        d = {f"storage.{k}": v for k, v in self.storage.items()}
        d.update(tree_sum=self.tree.sum, tree_min=self.tree.min,
                 meta=np.array([self.head, self.live, self.total_inserted], np.int64))
        return d

    def load_state_dict(self, d: Dict[str, np.ndarray]) -> None:
        self.storage = {k[len("storage."):]: np.array(v) for k, v in d.items()
                        if k.startswith("storage.")}
        self.tree.sum[:] = d["tree_sum"]
        self.tree.min[:] = d["tree_min"]
        self.head, self.live, self.total_inserted = (int(x) for x in d["meta"])
