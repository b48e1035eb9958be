"""Wall-clock timers.  Step timings mirror the reference's "Step Finished: X with N ms"
lines (e.g. ``J/core/processor/TrainModelProcessor.java:213-215``)."""
from __future__ import annotations

import time
from contextlib import contextmanager

from .log import get_logger

_log = get_logger("timer")


class Timer:
    def __init__(self):
        self.t0 = time.perf_counter()

    def elapsed(self) -> float:
        return time.perf_counter() - self.t0

    def ms(self) -> float:
        return self.elapsed() * 1e3


class StepTimer:
    """Accumulates named phase timings (seconds)."""

    def __init__(self):
        self.totals: dict[str, float] = {}
        self.counts: dict[str, int] = {}

    @contextmanager
    def phase(self, name: str, sync=None):
        if sync:
            sync()
        t0 = time.perf_counter()
        try:
            yield
        finally:
            if sync:
                sync()
            dt = time.perf_counter() - t0
            self.totals[name] = self.totals.get(name, 0.0) + dt
            self.counts[name] = self.counts.get(name, 0) + 1

    def summary(self) -> dict:
        return {k: {"total_s": v, "count": self.counts[k]} for k, v in self.totals.items()}


@contextmanager
def step_finished(step_name: str):
    t = Timer()
    yield
    _log.info("Step Finished: %s with %d ms", step_name, int(t.ms()))
