"""Jackson-compatible JSON IO for ModelConfig.json / ColumnConfig.json.

The reference serializes with Jackson's default pretty printer (2-space indent, ``"k" : v``
separators, primitive arrays on one line ``[ 1, 2 ]``, object arrays as ``[ {`` ... ``}, {``
... ``} ]``) and writes non-finite doubles as strings (``"-Infinity"`` in ``binBoundary``,
see ``src/test/resources/example/wdbc/wdbcModelSetLocal/ColumnConfig.json``).  We reproduce
that so files written by shifu_amd diff cleanly against files written by Shifu.
"""
from __future__ import annotations

import json
import math
from decimal import Decimal
from collections import OrderedDict


def java_double_str(x: float) -> str:
    """Java ``Double.toString`` formatting (decimal for 1e-3 <= |x| < 1e7, else x.yE±n)."""
    if x != x:
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    if x == 0:
        return "-0.0" if math.copysign(1.0, x) < 0 else "0.0"
    ax = abs(x)
    r = repr(float(x))
    if 1e-3 <= ax < 1e7:
        if "e" in r or "E" in r:
            r = f"{x:.17f}".rstrip("0")
            if r.endswith("."):
                r += "0"
        elif "." not in r:
            r += ".0"
        return r
    # shortest round-trip digits (repr) re-positioned as d.dddE±n without float arithmetic
    sign, digits, exp10 = Decimal(repr(float(ax))).as_tuple()
    ds = "".join(map(str, digits)).rstrip("0") or "0"
    e = exp10 + len(digits) - 1
    m = ("-" if x < 0 else "") + ds[0] + "." + (ds[1:] or "0")
    if "." not in m:
        m += ".0"
    return f"{m}E{int(e)}"


def _scalar(v) -> str:
    if v is None:
        return "null"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, int):
        return str(v)
    if isinstance(v, float):
        if math.isnan(v) or math.isinf(v):
            return json.dumps(java_double_str(v))
        return java_double_str(v)
    return json.dumps(v, ensure_ascii=False)


def _is_primitive(v) -> bool:
    return not isinstance(v, (dict, list, tuple))


def dumps(obj, indent: int = 0) -> str:
    pad = "  " * indent
    if isinstance(obj, dict):
        if not obj:
            return "{ }"
        items = []
        for k, v in obj.items():
            items.append(f'{pad}  {json.dumps(str(k), ensure_ascii=False)} : {dumps(v, indent + 1)}')
        return "{\n" + ",\n".join(items) + f"\n{pad}}}"
    if isinstance(obj, (list, tuple)):
        if not obj:
            return "[ ]"
        if all(_is_primitive(v) for v in obj):
            return "[ " + ", ".join(_scalar(v) for v in obj) + " ]"
        parts = [dumps(v, indent) for v in obj]
        return "[ " + ", ".join(parts) + " ]"
    return _scalar(obj)


def _hook(pairs):
    return OrderedDict(pairs)


def loads(text: str):
    return json.loads(text, object_pairs_hook=_hook)


def load(path):
    with open(path, encoding="utf-8") as f:
        return loads(f.read())


def dump(obj, path):
    """Write atomically (temp file in the same directory + rename): ranks / processes that read
    a ModelConfig / ColumnConfig while rank 0 rewrites it see the old or the new file, never a
    truncated one."""
    import os
    import tempfile
    path = os.path.realpath(path)              # a symlinked config: update the link's target
    d = os.path.dirname(path)
    fd, tmp = tempfile.mkstemp(prefix=".tmp_", suffix=".json", dir=d)
    try:
        with os.fdopen(fd, "w", encoding="utf-8") as f:
            f.write(dumps(obj))
        if os.path.exists(path):
            mode = os.stat(path).st_mode & 0o777
        else:                                   # a new file: 0666 minus the process umask
            um = os.umask(0)
            os.umask(um)
            mode = 0o666 & ~um
        os.chmod(tmp, mode)                     # mkstemp creates 0600
        os.replace(tmp, path)
    except BaseException:
        if os.path.exists(tmp):
            os.unlink(tmp)
        raise


def to_double(v):
    """Decode a Jackson double that may be a string (``"-Infinity"``, ``"NaN"``)."""
    if v is None:
        return None
    if isinstance(v, str):
        t = v.strip()
        if t in ("-Infinity", "-inf"):
            return float("-inf")
        if t in ("Infinity", "inf", "+Infinity"):
            return float("inf")
        if t == "NaN":
            return float("nan")
        return float(t)
    return float(v)
