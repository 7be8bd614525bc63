"""Actor group on its own host thread, decoupled from the learner.

The reference runs N actor processes concurrently with the learner process
(``main.py:46-58``): neither waits for the other.  On a GPU rank the actor group
(env stepping on the host, batched inference on its own HIP stream, n-step
building, inserts on the compute stream) runs here, on a thread, while the
learner thread replays its step graphs back to back:

* the env step (numpy), the n-step builder (native C++ through ctypes, which
  drops the GIL) and the stream waits (HIP synchronise, GIL released) overlap
  the learner thread's graph launches; the learner keeps at most
  ``max_inflight`` graph chunks queued so the actor's inserts never wait behind
  a long queue;
* the replay shard's host state is guarded by ``GpuReplayShard.lock``, and every
  kernel a locked section enqueues lands on the compute stream in the order the
  sections ran, so the compute stream stays the single writer of the tree and
  records (inserts, evictions, the learner's priority write-back);
* heartbeat: the thread stamps ``beat`` after every group step; the learner
  loop calls :meth:`check`, which restarts a thread that died with an exception
  (up to ``max_restarts``, fresh env episodes) and raises when one is stalled
  for ``timeout`` seconds (the rank then fails and torchrun's elastic restart
  resumes every rank from the last checkpoint, ``runtime/launch.py``).
"""
from __future__ import annotations

import threading
import time
import traceback
from typing import Callable, List, Optional


class ActorRunner:
    def __init__(self, group, max_steps: int, timeout: float = 60.0, max_restarts: int = 3,
                 on_event: Optional[Callable[..., None]] = None):
        self.group = group
        self.max_steps = int(max_steps)
        self.timeout = float(timeout)
        self.max_restarts = int(max_restarts)
        self.on_event = on_event
        self.steps = 0
        self.restarts = 0
        self.beat = time.time()
        self.errors: List[str] = []
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._failed = False

    # ------------------------------------------------------------- thread body
    def _run(self) -> None:
        try:
            while not self._stop.is_set() and self.steps < self.max_steps:
                self.group.step()
                self.steps += 1
                self.beat = time.time()
        except BaseException:   # noqa: BLE001 - reported to the learner thread by check()
            self.errors.append(traceback.format_exc())
            self._failed = True

    def start(self) -> "ActorRunner":
        self._stop.clear()
        self._failed = False
        self.beat = time.time()
        self._thread = threading.Thread(target=self._run, name="apex-actor", daemon=True)
        self._thread.start()
        return self

    def stop(self, timeout: float = 30.0) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout)

    def pause(self, timeout: float = 60.0) -> None:
        """Quiesce: let the thread finish its current group step and end (the learner
        thread then launches alone, e.g. to recapture its graphs); :meth:`resume` starts a
        fresh thread that continues the step count."""
        self.stop(timeout)
        if self.alive:
            raise RuntimeError("actor thread did not stop within %.0f s" % timeout)

    def resume(self) -> None:
        if not self.done:
            self.start()

    # ----------------------------------------------------------------- health
    @property
    def done(self) -> bool:
        return self.steps >= self.max_steps

    @property
    def alive(self) -> bool:
        return self._thread is not None and self._thread.is_alive()

    def check(self) -> None:
        """Learner-side supervision: restart a crashed actor thread, fail on a stall."""
        if self._failed:
            if self.restarts >= self.max_restarts:
                raise RuntimeError("actor thread failed %d times; last error:\n%s"
                                   % (self.restarts + 1, self.errors[-1]))
            self.restarts += 1
            if self.on_event is not None:
                self.on_event("actor_restart", restarts=self.restarts, error=self.errors[-1].splitlines()[-1])
            self.group.reset_episodes()    # fresh episodes: the crashed step's env state is unknown
            self.start()
            return
        if self.alive and not self.done and time.time() - self.beat > self.timeout:
            raise RuntimeError("actor thread stalled: no group step for %.0f s" % (time.time() - self.beat))

