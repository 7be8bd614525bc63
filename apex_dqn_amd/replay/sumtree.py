"""Host (numpy) sum-tree: the oracle for the HIP 64-ary tree and the storage
behind the CPU prioritized replay.

Replaces the reference's dict-of-priorities + O(N^2) probability recompute
(``replay.py:18-30``, defects A1-A4) with O(log N) updates and O(B log N)
vectorised stratified sampling (reference ``replay.py:44-57`` is O(B*N)).
"""
from __future__ import annotations

import numpy as np


class SumTree:
    """Binary sum-tree + min-tree over ``capacity`` leaves (vectorised).

    ``update`` resolves duplicate indices in one call deterministically: the
    last occurrence wins (same rule as the HIP kernel).
    """

    def __init__(self, capacity: int):
        cap = 1
        while cap < capacity:
            cap *= 2
        self.capacity = int(capacity)
        self.size2 = cap
        self.sum = np.zeros(2 * cap, np.float64)
        self.min = np.full(2 * cap, np.inf, np.float64)

    @property
    def total(self) -> float:
        return float(self.sum[1])

    @property
    def min_positive(self) -> float:
        return float(self.min[1])

    def get(self, idx) -> np.ndarray:
        return self.sum[self.size2 + np.asarray(idx, np.int64)]

    def update(self, idx, values) -> None:
        idx = np.asarray(idx, np.int64).ravel()
        values = np.asarray(values, np.float64).ravel()
        if idx.size == 0:
            return
        if idx.min() < 0 or idx.max() >= self.capacity:
            raise IndexError("sum-tree index out of range")
        # last-writer-wins dedupe
        rev_idx = idx[::-1]
        uniq, first_in_rev = np.unique(rev_idx, return_index=True)
        vals = values[::-1][first_in_rev]
        nodes = uniq + self.size2
        self.sum[nodes] = vals
        self.min[nodes] = np.where(vals > 0, vals, np.inf)
        nodes = np.unique(nodes // 2)
        while nodes[0] >= 1:
            self.sum[nodes] = self.sum[2 * nodes] + self.sum[2 * nodes + 1]
            self.min[nodes] = np.minimum(self.min[2 * nodes], self.min[2 * nodes + 1])
            if nodes[0] == 1:
                break
            nodes = np.unique(nodes // 2)

    def find_prefix(self, u) -> np.ndarray:
        """Smallest leaf i with cumsum(leaves)[i] > u (vectorised descent)."""
        u = np.asarray(u, np.float64).copy()
        node = np.ones(u.shape, np.int64)
        while node[0] < self.size2:
            left = 2 * node
            lv = self.sum[left]
            # go right when u passes the left mass, but never into an empty
            # subtree (guards fp round-off at the top of the range)
            go_right = (u >= lv) & (self.sum[left + 1] > 0)
            u = np.where(go_right, u - lv, u)
            node = np.where(go_right, left + 1, left)
        return np.minimum(node - self.size2, self.capacity - 1)

    def sample_stratified(self, batch: int, rng: np.random.Generator) -> np.ndarray:
        total = self.total
        if total <= 0:
            raise RuntimeError("cannot sample from an empty sum-tree")
        seg = total / batch
        u = (np.arange(batch) + rng.random(batch)) * seg
        u = np.minimum(u, np.nextafter(total, 0))
        return self.find_prefix(u)


def inverse_cdf_oracle(leaves: np.ndarray, u: np.ndarray) -> np.ndarray:
    """Brute-force reference: smallest i with cumsum(leaves)[i] > u."""
    c = np.cumsum(np.asarray(leaves, np.float64))
    return np.minimum(np.searchsorted(c, u, side="right"), len(leaves) - 1)
