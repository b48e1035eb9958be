"""Failure handling: a test-only fault hook and numeric guards.

``SHIFU_FAULT_AT_ITER=n`` (optionally ``SHIFU_FAULT_RANK=r`` or ``*``) makes the training loop of
rank r terminate abruptly (``os._exit``, no cleanup, like a killed worker) right after iteration
n's checkpoint was written; re-running the same command resumes from that checkpoint.  The
reference has no fault injection; its recovery paths (NNMaster.initOrRecoverParams :331-362,
DTMaster.recoverMasterStatus :1118-1154) are reproduced by checkpoint + resume.
"""
from __future__ import annotations

import math
import os
import threading
import time

from ..utils.log import get_logger

_log = get_logger("runtime.fault")
FAULT_EXIT_CODE = 17
WATCHDOG_EXIT_CODE = 18


def maybe_fault(iteration: int, rank: int = 0) -> None:
    hang = os.environ.get("SHIFU_FAULT_HANG_AT_ITER")      # test hook: a rank that stops progressing
    if hang and int(hang) == iteration and os.environ.get("SHIFU_FAULT_RANK", "0") in ("*", str(rank)):
        _log.error("fault injection: rank %d hangs at iteration %d", rank, iteration)
        while True:
            time.sleep(1.0)
    at = os.environ.get("SHIFU_FAULT_AT_ITER")
    if not at:
        return
    who = os.environ.get("SHIFU_FAULT_RANK", "0")
    if int(at) == iteration and (who == "*" or int(who) == rank):
        _log.error("fault injection: rank %d exits at iteration %d", rank, iteration)
        os._exit(FAULT_EXIT_CODE)


def check_finite(name: str, value: float, iteration: int) -> None:
    """NaN/Inf guard: a diverged model stops the job with a clear error instead of writing NaN weights."""
    if not math.isfinite(value):
        raise FloatingPointError(f"{name} is {value} at iteration {iteration}; lower LearningRate or check data")


class IterationWatchdog:
    """Per-iteration time limit, the ``@ComputableMonitor`` timeouts of the reference (NNWorker
    3600 s, J/core/dtrain/nn/NNWorker.java:52; DTWorker 800 s, J/core/dtrain/dt/DTWorker.java:105):
    a daemon thread aborts the process (``WATCHDOG_EXIT_CODE``) when no ``tick()`` arrived within
    ``limit_s`` - a hung collective or a stuck rank then fails the job instead of blocking the
    node, and the run is resumed from its last checkpoint (possibly with another world size: rows
    are re-sharded on load and the optimizer state is replicated).  ``limit_s <= 0`` disables."""

    def __init__(self, limit_s: float, what: str = "iteration"):
        self.limit, self.what = float(limit_s), what
        self.last = time.monotonic()
        self._stop = threading.Event()
        self._t = None

    def __enter__(self):
        if self.limit > 0:
            self._t = threading.Thread(target=self._run, daemon=True, name="shifu-watchdog")
            self._t.start()
        return self

    def tick(self):
        self.last = time.monotonic()

    def _run(self):
        period = min(1.0, self.limit / 4)
        while not self._stop.wait(period):
            idle = time.monotonic() - self.last
            if idle > self.limit:
                _log.error("watchdog: no %s progress for %.1f s (limit %.1f s); aborting", self.what, idle, self.limit)
                os._exit(WATCHDOG_EXIT_CODE)

    def __exit__(self, *exc):
        self._stop.set()
        return False


def iteration_limit(default_s: float) -> float:
    """``shifu.train.iteration.timeout`` / ``SHIFU_ITERATION_TIMEOUT`` seconds (0 disables)."""
    from ..config import environment
    v = os.environ.get("SHIFU_ITERATION_TIMEOUT") or environment.get("shifu.train.iteration.timeout", None)
    return float(v) if v not in (None, "") else float(default_s)
