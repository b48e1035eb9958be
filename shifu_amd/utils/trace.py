"""Tracing: roctx ranges around steps, epochs, kernels groups and collectives.

On ROCm ``torch.cuda.nvtx`` is backed by roctx, so the ranges show up in
``rocprofv3 --marker-trace`` / ``--sys-trace`` timelines next to the kernels.  Ranges are no-ops
on the CPU path and cost one host call on the GPU path; ``SHIFU_TRACE=0`` disables them.
Step wall times are also logged as ``Step Finished: <name> with <ms> ms`` (the reference's
processor log line) and appended to the JSONL metrics stream when one is active.
"""
from __future__ import annotations

import contextlib
import os
import time

import torch

from .log import get_logger

_log = get_logger("trace")
_ENABLED = os.environ.get("SHIFU_TRACE", "1") != "0"


def _gpu():
    return torch.cuda.is_available() and os.environ.get("SHIFU_FORCE_CPU") != "1"


@contextlib.contextmanager
def trace_range(name: str):
    pushed = False
    if _ENABLED and _gpu():
        try:
            torch.cuda.nvtx.range_push(name)
            pushed = True
        except Exception:   # noqa: BLE001 - tracing must never break a run
            pushed = False
    try:
        yield
    finally:
        if pushed:
            torch.cuda.nvtx.range_pop()


@contextlib.contextmanager
def step_timer(step: str):
    """``Step Start: x`` / ``Step Finished: x with N ms`` around a processor (+ roctx range)."""
    _log.info("Step Start: %s", step)
    t0 = time.perf_counter()
    with trace_range(f"shifu.{step}"):
        yield
    _log.info("Step Finished: %s with %d ms", step, int((time.perf_counter() - t0) * 1000))
