"""Opt-in usage records (A3).

The reference appends one record per invocation to ``/tmp/shifu`` on HDFS
(``B/shifu_statistics.sh``) and kills the YARN applications of an interrupted run
(``B/cleanup.sh``, trap in ``B/shifu:105-109, 206``).  Here, when enabled with
``SHIFU_TELEMETRY=1`` (or ``-Dshifu.telemetry=true``), every CLI invocation appends one JSON line
(time, verb, arguments, exit code, seconds, world size) to the model set's own
``logs/usage.jsonl`` (or ``$SHIFU_STATS_DIR/usage.jsonl`` when that is set).  Off by default,
nothing leaves the model set.  The interrupt cleanup lives in ``bin/shifu`` (the torchrun child
is signalled and reaped on SIGINT/SIGTERM).
"""
from __future__ import annotations

import json
import os
import time

from ..config import environment


def enabled() -> bool:
    if os.environ.get("SHIFU_TELEMETRY", "0") == "1":
        return True
    return environment.get_bool("shifu.telemetry", False)


def stats_path(model_set_dir: str = ".") -> str:
    base = os.environ.get("SHIFU_STATS_DIR") or os.path.join(model_set_dir, "logs")
    return os.path.join(base, "usage.jsonl")


def record_usage(cmd: str, args, rc: int, seconds: float, world_size: int = 1, rank: int = 0,
                 model_set_dir: str = ".") -> str | None:
    """Append one usage record (rank 0, enabled, inside a model set); never raises."""
    if rank != 0 or not enabled():
        return None
    if not os.environ.get("SHIFU_STATS_DIR") and not os.path.exists(os.path.join(model_set_dir, "ModelConfig.json")):
        return None
    rec = {"ts": time.strftime("%Y-%m-%dT%H:%M:%S"), "model_set": os.path.basename(os.path.abspath(model_set_dir)),
           "cmd": cmd, "args": list(args), "rc": int(rc), "seconds": round(float(seconds), 3),
           "world_size": int(world_size)}
    path = stats_path(model_set_dir)
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "a") as fh:
            fh.write(json.dumps(rec) + "\n")
    except OSError:
        return None
    return path
