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

from ..utils.log import get_logger

_log = get_logger("runtime.fault")
FAULT_EXIT_CODE = 17


def maybe_fault(iteration: int, rank: int = 0) -> None:
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
