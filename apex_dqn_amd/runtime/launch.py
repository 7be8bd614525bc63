"""Single-node elastic launcher with restart-from-checkpoint.

The reference has no failure handling at all: a dead learner or inserter
leaves the others spinning forever (``learner.py:64-65``).  On a
GPU node the framework runs under ``torchrun --max-restarts K``: when any rank
dies, torchrun tears the group down and restarts every rank, and each rank
resumes from the shared checkpoint (``Runtime.resume``,
``runtime/gpu_loop.py``), so the data-parallel replicas stay identical.

``run_elastic`` implements the same contract without torchrun (CPU / gloo
tests, hosts without the launcher): spawn ``world_size`` ranks with a fresh
file:// rendezvous per attempt; if any rank exits non-zero the surviving
ranks of that attempt are terminated (by their own PIDs) and the whole group
is restarted, up to ``max_restarts`` times.
"""
from __future__ import annotations

import os
import tempfile
import time
from typing import Any, Callable, Dict, Sequence

import torch.multiprocessing as mp


def _rank_main(target: Callable, rank: int, world: int, init_method: str, attempt: int, args: Sequence[Any],
               backend: str) -> None:
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), APEX_RESTART_ATTEMPT=str(attempt))
    from ..parallel.dist import Comm
    comm = Comm.init(rank, world, init_method, backend=backend)
    try:
        target(comm, attempt, *args)
    finally:
        comm.shutdown()


def run_elastic(target: Callable, world_size: int, args: Sequence[Any] = (), max_restarts: int = 3,
                backend: str = "gloo", timeout_s: float = 900.0, poll_s: float = 0.2) -> Dict[str, Any]:
    """Run ``target(comm, attempt, *args)`` on ``world_size`` ranks; restart the
    whole group when a rank fails.  Returns {"attempts", "failures"}."""
    ctx = mp.get_context("spawn")
    failures = []
    rdzv_dir = tempfile.mkdtemp(prefix="apex_rdzv_")
    t_end = time.time() + timeout_s
    for attempt in range(max_restarts + 1):
        init = f"file://{os.path.join(rdzv_dir, f'rdzv_{attempt}')}"
        procs = [ctx.Process(target=_rank_main, args=(target, r, world_size, init, attempt, tuple(args), backend))
                 for r in range(world_size)]
        for p in procs:
            p.start()
        failed = None
        while True:
            codes = [p.exitcode for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                failed = bad
                break
            if all(c == 0 for c in codes):
                break
            if time.time() > t_end:
                failed = [(-1, "timeout")]
                break
            time.sleep(poll_s)
        if failed is None:
            return {"attempts": attempt + 1, "failures": failures}
        failures.append({"attempt": attempt, "ranks": failed})
        for p in procs:               # tear the group down: exact PIDs of this attempt only
            if p.is_alive():
                p.terminate()
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
                p.join(timeout=10)
        if failed and failed[0][0] == -1:
            break
    raise RuntimeError(f"elastic run failed after {len(failures)} attempt(s): {failures}")
