"""Zero-copy parameter publication from the learner to actor processes.

Reference: the learner pickles the whole 13.3 MB ``state_dict`` into a
Manager dict every step (``learner.py:74``, 6.1 ms) and actors unpickle it
every 500 steps (``actor.py:189-191``).  Here the learner copies its flat
parameters into one shared-memory tensor and bumps a version counter; actors
copy only when the version changed.  A seqlock (odd version = write in
progress) keeps readers from observing a torn copy.
"""
from __future__ import annotations

import math
import multiprocessing as mp
from typing import Dict, List, Tuple

import torch


class SharedParams:
    def __init__(self, template: Dict[str, torch.Tensor], ctx=None):
        ctx = ctx or mp.get_context("spawn")
        self.spec: List[Tuple[str, Tuple[int, ...], int]] = []
        off = 0
        for k, v in template.items():
            n = v.numel()
            self.spec.append((k, tuple(v.shape), off))
            off += n
        self.numel = off
        self.flat = torch.zeros(off, dtype=torch.float32).share_memory_()
        self.version = ctx.Value("q", 0, lock=False)
        # native seqlock (csrc/runtime): release/acquire fences around the copy
        from . import native
        self.native = native.available()
        if self.native:
            self.seq = torch.zeros(1, dtype=torch.int64).share_memory_()
        self.publish(template)

    def __setstate__(self, st):
        self.__dict__.update(st)
        if self.native:
            from . import native
            self.native = native.available()

    def publish(self, state: Dict[str, torch.Tensor]) -> None:
        if self.native:
            from .native import SeqLock
            stage = torch.cat([state[k].detach().reshape(-1).float().cpu() for k, _, _ in self.spec])
            SeqLock(self.seq, self.flat).write(stage)
            return
        self.version.value += 1          # odd: writing
        for k, shape, off in self.spec:
            v = state[k]
            self.flat[off:off + v.numel()].copy_(v.detach().reshape(-1).float().cpu())
        self.version.value += 1          # even: stable

    def read(self, last_version: int = -1):
        """Return (version, state_dict) or (last_version, None) if unchanged."""
        if self.native:
            from .native import SeqLock
            snap = torch.empty_like(self.flat)
            v = SeqLock(self.seq, self.flat).read_into(snap, last_version)
            if v < 0:
                return last_version, None
            return v, {k: snap[off:off + math.prod(shape)].view(shape) for k, shape, off in self.spec}
        for _ in range(1000):
            v0 = self.version.value
            if v0 == last_version:
                return last_version, None
            if v0 % 2:
                continue
            snap = self.flat.clone()
            if self.version.value == v0:
                out = {k: snap[off:off + math.prod(shape)].view(shape)
                       for k, shape, off in self.spec}
                return v0, out
        return last_version, None
