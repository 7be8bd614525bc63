"""Phase watchdog for multi-rank GPU runs (bench.py; the learner loop has its own
per-chunk wait in ``runtime/gpu_loop.py``).

A rank whose peer died blocks forever inside a collective -- in the host call
(communicator init, a barrier) or in a ``synchronize`` behind a hung RCCL kernel.  The
reference has no failure detection at all.  ``PhaseWatchdog`` runs a
daemon thread that knows the current phase and its deadline; when a phase overruns it
names the rank and the phase on stderr, aborts the communicators (so no teardown
blocks) and ends the process with ``WATCHDOG_EXIT_CODE`` -- non-zero, so the driver or
torchrun sees the failure instead of a silent hang.
"""
from __future__ import annotations

import os
import sys
import threading
import time
from contextlib import contextmanager
from typing import Optional

WATCHDOG_EXIT_CODE = 75


class PhaseWatchdog:
    def __init__(self, rank: int = 0, comm=None, exit_code: int = WATCHDOG_EXIT_CODE, _exit=None):
        self.rank = int(rank)
        self.comm = comm
        self.exit_code = int(exit_code)
        self._exit = _exit or os._exit       # (tests substitute a recorder)
        self._lock = threading.Lock()
        self._phase: Optional[str] = None
        self._deadline = 0.0
        self._timeout = 0.0
        self._seq = 0
        self._stop = threading.Event()
        self.fired: Optional[str] = None
        self._thread = threading.Thread(target=self._run, name="apex-phase-watchdog", daemon=True)
        self._thread.start()

    @contextmanager
    def phase(self, name: str, timeout: float):
        """Run the body under a deadline of ``timeout`` seconds (<= 0: no deadline)."""
        with self._lock:
            self._seq += 1
            seq = self._seq
            prev = (self._phase, self._deadline, self._timeout)
            self._phase, self._timeout = name, float(timeout)
            self._deadline = time.monotonic() + float(timeout) if timeout > 0 else float("inf")
        try:
            yield
        finally:
            with self._lock:
                if self._seq == seq:
                    self._phase, self._deadline, self._timeout = prev

    def _run(self) -> None:
        while not self._stop.wait(0.5):
            with self._lock:
                phase, deadline, timeout = self._phase, self._deadline, self._timeout
            if phase is not None and time.monotonic() > deadline:
                self._fire(phase, timeout)
                return

    def _fire(self, phase: str, timeout: float) -> None:
        msg = f"[rank {self.rank}] watchdog: phase '{phase}' did not finish in {timeout:.0f} s; exiting\n"
        self.fired = phase
        sys.stderr.write(msg)
        sys.stderr.flush()
        try:
            if self.comm is not None and hasattr(self.comm, "abort"):
                self.comm.abort()
        except Exception:  # pragma: no cover - best effort on the failure path
            pass
        self._exit(self.exit_code)

    def close(self) -> None:
        self._stop.set()
