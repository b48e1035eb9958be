"""Shared utilities: logging, timers, JSONL metrics, roctx ranges, device helpers."""
from .log import get_logger, setup_logging
from .timer import Timer, StepTimer
from .metrics import MetricsWriter
from .device import default_device, is_gpu_available, sync

__all__ = [
    "get_logger", "setup_logging", "Timer", "StepTimer", "MetricsWriter",
    "default_device", "is_gpu_available", "sync",
]
