"""Segment expansion (C6): ``dataSet.segExpressionFile`` lists filter expressions; every raw column
gets one copy per segment, named ``<column>_<k>`` (k = 1..S) with column number ``k * size + i``
(``AddColumnNumAndFilterUDF.exec`` J/udf/AddColumnNumAndFilterUDF.java:160-185, updaters
``TrainUpdater``/``VarSelUpdater`` J/util/updater/*).  A copy carries the row's value when the row
passes segment k's filter and is missing otherwise, so its stats / bins / WOE describe that
segment only and a model can learn per-segment effects.  Segments are supported for NN and LR
(``BasicModelProcessor.setUp`` :140-155)."""
from __future__ import annotations

import re

import numpy as np

from .expr import Evaluator
from .reader import Column

_SUFFIX = re.compile(r"^(.*)_(\d+)$")


def split_name(name: str, n_segments: int, raw_names: set):
    """``col_3`` -> ("col", 3) when it is a segment copy of a raw column; else (name, 0)."""
    m = _SUFFIX.match(name)
    if m and n_segments and name not in raw_names:
        base, k = m.group(1), int(m.group(2))
        if 1 <= k <= n_segments and base in raw_names:
            return base, k
    return name, 0


def needed_base_columns(names, exprs, raw_names: set):
    """Raw columns to parse for ``names`` (segment copies map to their base) + filter columns."""
    base, kinds = set(), set()
    for n in names:
        b, k = split_name(n, len(exprs), raw_names)
        base.add(b)
        if k:
            kinds.add(k)
    expr_cols = set()
    for k in kinds:
        try:
            expr_cols |= set(Evaluator(exprs[k - 1]).columns())
        except Exception:    # noqa: BLE001 - reported when evaluated
            pass
    return base, expr_cols


def expand(table, names, exprs, raw_names: set):
    """Add the requested segment copies to ``table`` (in place) and return it."""
    masks = {}
    for n in names:
        b, k = split_name(n, len(exprs), raw_names)
        if not k or n in table.columns or b not in table.columns:
            continue
        if k not in masks:
            masks[k] = Evaluator(exprs[k - 1]).mask(table)
        src = table[b]
        keep = masks[k]
        if src.kind == "num":
            vals = np.where(keep, src.values, np.nan)
        else:
            vals = np.where(keep, src.values, -1).astype(src.values.dtype)
        table.columns[n] = Column(n, src.kind, vals, src.dictionary)
    return table
