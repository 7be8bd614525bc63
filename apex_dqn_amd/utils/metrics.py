"""Structured metrics (JSONL) and wall-clock phase timers.

The reference only prints (``actor.py:170,177``, ``main.py:34-35``); a
per-step ``\\r`` print in the actor hot loop is a throughput killer.  Here:
a JSONL stream on rank 0 plus the familiar per-episode console line.
"""
from __future__ import annotations

import json
import time
from collections import defaultdict
from contextlib import contextmanager
from typing import Any, Dict, Optional


class MetricsLogger:
    def __init__(self, path: Optional[str] = None, rank: int = 0, echo: bool = False):
        self.rank = rank
        self.echo = echo
        self.f = open(path, "a") if (path and rank == 0) else None
        self.t0 = time.time()

    def log(self, kind: str, **fields: Any) -> None:
        rec = {"t": round(time.time() - self.t0, 4), "kind": kind}
        rec.update({k: (float(v) if hasattr(v, "__float__") and not isinstance(v, (int, bool)) else v)
                    for k, v in fields.items()})
        if self.f is not None:
            self.f.write(json.dumps(rec) + "\n")
            self.f.flush()
        if self.echo and self.rank == 0:
            print(json.dumps(rec), flush=True)

    def episode(self, actor_id: int, t: int, ep_len: int, ep_reward: float) -> None:
        # same console line as reference actor.py:177
        if self.rank == 0:
            print("Actor#:", actor_id, "t:", t, "  ep_len:", ep_len, "  ep_reward:", ep_reward)
        self.log("episode", actor=actor_id, t=t, ep_len=ep_len, ep_reward=ep_reward)

    def close(self) -> None:
        if self.f is not None:
            self.f.close()


class PhaseTimer:
    """Accumulating wall timers per phase (host-side; synchronise first for GPU phases)."""

    def __init__(self):
        self.acc: Dict[str, float] = defaultdict(float)
        self.cnt: Dict[str, int] = defaultdict(int)

    @contextmanager
    def phase(self, name: str, sync=None):
        if sync is not None:
            sync()
        t = time.perf_counter()
        yield
        if sync is not None:
            sync()
        self.acc[name] += time.perf_counter() - t
        self.cnt[name] += 1

    def summary(self) -> Dict[str, float]:
        return {k: 1e3 * v / max(self.cnt[k], 1) for k, v in self.acc.items()}

    def reset(self) -> None:
        self.acc.clear()
        self.cnt.clear()
