"""Layered global flags (C4): ``$SHIFU_HOME/conf/shifuconfig`` -> ``/etc/shifuconfig`` ->
``~/.shifuconfig`` -> CLI ``-Dk=v`` (``J/util/Environment.java:92-106``, ``J/ShifuCLI.java:430-453``).

Hadoop/Guagua/Pig-specific keys are accepted and ignored with a one-time warning; shifu.*
keys are honoured (e.g. ``shifu.train.bagging.inparallel``, ``shifu.gridsearch.threshold``,
``shifu.train.val.steps.ratio``, ``shifu.train.earlystop.window.size``).
"""
from __future__ import annotations

import os
import threading

from ..utils.log import get_logger

_log = get_logger("config.environment")

DEFAULTS = {
    "localNumParallel": "6",
    "shifu.train.bagging.inparallel": "5",
    "shifu.gridsearch.threshold": "30",
    "shifu.namespace.strict.mode": "false",
    "shifu.eval.score.multithread": "false",
    "shifu.train.nn.inputlayerdropout.enable": "true",
    "shifu.train.val.steps.ratio": "0.1",
    "shifu.train.earlystop.window.size": "20",
    "shifu.tree.checkpoint.interval": "100",
    "shifu.combo.max.retry": "3",
    "shifu.stats.corr.reuse": "false",
    "shifu.stats.streaming": "auto",
    "shifu.stats.streamThresholdGB": "8",
    "shifu.stats.binning.parity": "false",
    "shifu.varsel.se.reuse": "false",
    "shifu.tree.regeninput": "false",
}
IGNORED_PREFIXES = ("mapreduce.", "guagua.", "pig.", "hadoop", "zookeeper", "mapred.", "yarn.")

_lock = threading.Lock()
_props: dict | None = None
_warned: set = set()


def _parse_props(path):
    out = {}
    if not path or not os.path.isfile(path):
        return out
    with open(path, encoding="utf-8") as f:
        for line in f:
            line = line.strip()
            if not line or line.startswith("#") or "=" not in line:
                continue
            k, v = line.split("=", 1)
            out[k.strip()] = v.strip()
    return out


def _load():
    props = dict(DEFAULTS)
    home = os.environ.get("SHIFU_HOME")
    for p in ([os.path.join(home, "conf", "shifuconfig")] if home else []) + \
             ["/etc/shifuconfig", os.path.expanduser("~/.shifuconfig")]:
        props.update(_parse_props(p))
    return props


def props() -> dict:
    global _props
    with _lock:
        if _props is None:
            _props = _load()
        return _props


def reload():
    global _props
    with _lock:
        _props = None
    return props()


def set_property(k: str, v):
    p = props()
    if k.startswith(IGNORED_PREFIXES) and k not in _warned:
        _warned.add(k)
        _log.warning("property %s is Hadoop/Guagua/Pig specific and has no effect on MI355X", k)
    p[k] = str(v)


def get(k: str, default=None):
    v = os.environ.get("SHIFU_PROP_" + k.replace(".", "_"))
    if v is not None:
        return v
    return props().get(k, default)


def get_int(k, default=0) -> int:
    try:
        return int(float(get(k, default)))
    except (TypeError, ValueError):
        return default


def get_float(k, default=0.0) -> float:
    try:
        return float(get(k, default))
    except (TypeError, ValueError):
        return default


def get_bool(k, default=False) -> bool:
    v = get(k, None)
    if v is None:
        return default
    return str(v).strip().lower() in ("1", "true", "yes", "y", "on")


def apply_cli_overrides(args):
    """Consume ``-Dk=v`` tokens from an argv list (returns the remaining args)."""
    rest = []
    for a in args:
        if a.startswith("-D") and "=" in a:
            k, v = a[2:].split("=", 1)
            set_property(k, v)
        else:
            rest.append(a)
    return rest
