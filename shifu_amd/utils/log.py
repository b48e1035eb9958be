"""Logging setup.

The reference logs through SLF4J/log4j to console plus a rolling ``logs/shifu.log``
(``src/main/resources/conf/log4j.properties``).  We keep the same human-readable
progress lines ("Trainer i Epoch #n Training Error: ... Validation Error: ...",
``J/core/dtrain/nn/NNOutput.java:219-237``) on the Python ``logging`` module and add a
machine-readable JSONL stream (see :mod:`shifu_amd.utils.metrics`).
"""
from __future__ import annotations

import logging
import logging.handlers
import os
import sys

_CONFIGURED = False
FORMAT = "%(asctime)s %(levelname)s [%(name)s] %(message)s"


def setup_logging(level: str | int | None = None, log_dir: str | None = None) -> None:
    global _CONFIGURED
    if _CONFIGURED:
        return
    lvl = level or os.environ.get("SHIFU_LOG_LEVEL", "INFO")
    if isinstance(lvl, str):
        lvl = getattr(logging, lvl.upper(), logging.INFO)
    root = logging.getLogger("shifu_amd")
    root.setLevel(lvl)
    h = logging.StreamHandler(sys.stderr)
    h.setFormatter(logging.Formatter(FORMAT))
    root.addHandler(h)
    if log_dir:
        os.makedirs(log_dir, exist_ok=True)
        fh = logging.handlers.RotatingFileHandler(
            os.path.join(log_dir, "shifu.log"), maxBytes=10 << 20, backupCount=10)
        fh.setFormatter(logging.Formatter(FORMAT))
        root.addHandler(fh)
    root.propagate = False
    _CONFIGURED = True


def get_logger(name: str) -> logging.Logger:
    if not name.startswith("shifu_amd"):
        name = "shifu_amd." + name
    setup_logging()
    return logging.getLogger(name)
