"""Purify / tag / sample / weight (H6).

* filter: ``DataPurifier.isFilter`` (J/core/DataPurifier.java:103-145) -> :mod:`.expr`
* tags: pos/neg tag groups (``a|b`` = one class), invalid tags dropped
  (``INVALID_TAG`` counter); multi-class = index into the tag list; linear target = float
* sampling: ``DataSampler.isNotSampled`` (J/core/DataSampler.java:112-153), ``sampleNegOnly``
* weight: column or JEXL expression (``NormalizeUDF.evaluateWeight`` J/udf/NormalizeUDF.java:640-661),
  invalid -> 1.0
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from ..utils.log import get_logger
from .expr import Evaluator
from .reader import RawTable, read_header, read_table, first_line_is_header

_log = get_logger("data.purifier")


@dataclass
class Counters:
    """Hadoop-counter equivalents (SHIFU_GROUP_COUNTER)."""
    total: int = 0
    filtered_out: int = 0
    invalid_tag: int = 0
    not_sampled: int = 0
    weight_exception: int = 0
    valid: int = 0
    pos: int = 0
    neg: int = 0

    def as_dict(self):
        return dict(TOTAL_VALID_COUNT=self.valid, FILTER_OUT_COUNT=self.filtered_out, INVALID_TAG=self.invalid_tag,
                    NOT_SAMPLED=self.not_sampled, WEIGHT_EXCEPTION=self.weight_exception, TOTAL=self.total,
                    POSTAGS=self.pos, NEGTAGS=self.neg)


@dataclass
class ModelData:
    table: RawTable
    y: np.ndarray                # float32: binary 1/0, multi-class index, or regression target
    w: np.ndarray                # float64 significance
    tag_index: np.ndarray        # int32 class index (-1 linear)
    counters: Counters = field(default_factory=Counters)

    @property
    def n(self):
        return self.table.n


def tag_index(values_str: np.ndarray, set_tags: list) -> np.ndarray:
    lut = {}
    for i, s in enumerate(set_tags):
        for t in s:
            lut[str(t).strip()] = i
    return np.array([lut.get(str(v).strip(), -1) if v is not None else -1 for v in values_str], dtype=np.int32)


def row_uniform(seed: int, row0: int, n: int) -> np.ndarray:
    """Uniform [0, 1) draws for raw rows row0 .. row0 + n - 1: a counter-based generator
    (splitmix64 of seed and the global row index), so a row's sampling decision is the same whether
    the data set is read whole, in chunks, or split over ranks by byte range."""
    with np.errstate(over="ignore"):
        x = (np.arange(row0, row0 + n, dtype=np.uint64) + np.uint64((int(seed) * 0x9E3779B97F4A7C15) % (1 << 64)))
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
    return (x >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


def purify(mc, table: RawTable, target: str, weight_expr: str | None = None, filter_expr: str | None = None,
           sample_rate: float = 1.0, sample_neg_only: bool = False, seed: int = 0,
           require_target: bool = True, row_offset: int = 0) -> ModelData:
    c = Counters(total=table.n)
    keep = np.ones(table.n, dtype=bool)
    if filter_expr and str(filter_expr).strip():
        try:
            m = Evaluator(filter_expr).mask(table)
            c.filtered_out = int((~m).sum())
            keep &= m
        except Exception as e:  # reference logs and keeps the row on expression errors
            _log.warning("filter expression %r failed (%s); no rows filtered", filter_expr, e)
    # target / tags
    ti = np.full(table.n, -1, dtype=np.int32)
    if target in table.columns:
        tcol = table[target]
        if mc.is_linear_target():
            y = tcol.numeric().astype(np.float64)
            bad = np.isnan(y)
            c.invalid_tag = int((bad & keep).sum())
            if require_target:
                keep &= ~bad
            y = np.nan_to_num(y)
        else:
            ti = tag_index(tcol.strings(), mc.set_tags())
            bad = ti < 0
            c.invalid_tag = int((bad & keep).sum())
            if require_target:
                keep &= ~bad
            if mc.is_binary():
                npos = len(mc.pos_tags)
                y = (ti < npos).astype(np.float64)   # pos tag groups come first in tags()
                y[ti < 0] = 0
            else:
                y = ti.astype(np.float64)
    else:
        if require_target:
            raise KeyError(f"target column {target!r} not in data header")
        y = np.zeros(table.n)
    # sampling
    if sample_rate < 1.0:
        r = row_uniform(seed, row_offset, table.n)
        if sample_neg_only and mc.is_binary():
            drop = (y == 0) & (r > sample_rate)
        else:
            drop = r > sample_rate
        c.not_sampled = int((drop & keep).sum())
        keep &= ~drop
    # weight
    w = np.ones(table.n)
    if weight_expr and str(weight_expr).strip():
        we = str(weight_expr).strip()
        if we in table.columns:
            wv = table[we].numeric()
        else:
            try:
                wv = Evaluator(we).values(table)
            except Exception as e:
                _log.warning("weight expression %r failed (%s); weight = 1", we, e)
                wv = np.ones(table.n)
        bad = ~np.isfinite(wv)
        c.weight_exception = int((bad & keep).sum())
        w = np.where(bad, 1.0, wv)
    idx = np.nonzero(keep)[0]
    c.valid = int(len(idx))
    if c.valid == table.n:
        # every row kept (the common case): no copy of the table (a full gather of every column
        # was ~7 % of a streamed stats / norm pass at 2M x 1600)
        t, yk, wk, tk = table, y.astype(np.float32), w.astype(np.float64, copy=False), ti
    else:
        t, yk, wk, tk = table.take(idx), y[idx].astype(np.float32), w[idx].astype(np.float64), ti[idx]
    if mc.is_binary():
        c.pos = int((yk == 1).sum())
        c.neg = int((yk == 0).sum())
    return ModelData(t, yk, wk, tk, c)


@dataclass
class DatasetPlan:
    """What to parse from one data set section and how to purify it (shared by the whole-table
    loader and the streamed chunk reader, data/stream.py)."""
    data_path: str
    delim: str
    header: list
    skip_header_line: bool
    target: str | None
    weight: str | None
    filt: str | None
    nums: list
    strs: list
    seg_names: list
    seg_exprs: list
    missing: list


def plan_dataset(mc, data_conf, columns_num=None, columns_str=None, extra_filter=None) -> DatasetPlan:
    data_path = mc.resolve(data_conf.get("dataPath"))
    delim = data_conf.get("dataDelimiter") or "|"
    hpath = data_conf.get("headerPath")
    header = read_header(mc.resolve(hpath) if hpath else None, data_conf.get("headerDelimiter") or "|",
                         data_path, delim)
    skip = (not hpath) and first_line_is_header(data_path, header, delim)
    target = data_conf.get("targetColumnName") or mc.dataSet.get("targetColumnName")
    weight = data_conf.get("weightColumnName")
    filt = data_conf.get("filterExpressions")
    if extra_filter:
        filt = f"({filt}) && ({extra_filter})" if filt else extra_filter
    strs = set(columns_str or [])
    nums = set(columns_num or [])
    seg_exprs = mc.segment_filter_expressions()
    seg_names = []
    if seg_exprs:                    # segment copies "<col>_<k>" are derived from their base column
        from . import segments
        raw = set(header)
        seg_names = [n for n in list(nums) + list(strs) if segments.split_name(n, len(seg_exprs), raw)[1]]
        base, expr_cols = segments.needed_base_columns(seg_names, seg_exprs, raw)
        for n in seg_names:
            b = segments.split_name(n, len(seg_exprs), raw)[0]
            (nums if n in nums else strs).add(b)
            nums.discard(n)
            strs.discard(n)
        strs |= {c for c in expr_cols if c in raw and c not in nums}
    if target:
        strs.add(target)
        nums.discard(target)
    needed_expr = []
    for e in (filt, weight):
        if e and str(e).strip():
            try:
                needed_expr += Evaluator(str(e)).columns()
            except Exception:
                pass
    from ..config.updater import simple_name
    hmap = {simple_name(h): h for h in header}
    for nm in needed_expr:
        h = nm if nm in header else hmap.get(simple_name(nm))
        if h and h not in nums:
            strs.add(h)
    if weight and weight in header:
        nums.add(weight)
        strs.discard(weight)
    return DatasetPlan(data_path, delim, header, skip, target, weight, filt, [h for h in header if h in nums],
                       [h for h in header if h in strs], seg_names, seg_exprs, list(mc.missing_values))


def finish_table(mc, plan: DatasetPlan, table, sample_rate=1.0, sample_neg_only=False, seed=0,
                 require_target=True, row_offset: int = 0) -> ModelData:
    """Segment expansion + purification of a parsed table (whole data set or one chunk whose first
    raw row is global row ``row_offset``)."""
    if plan.seg_names:
        from . import segments
        segments.expand(table, plan.seg_names, plan.seg_exprs, set(plan.header))
    return purify(mc, table, plan.target, plan.weight, plan.filt, sample_rate, sample_neg_only, seed,
                  require_target, row_offset)


def load_dataset(mc, data_conf, columns_num=None, columns_str=None, sample_rate=1.0, sample_neg_only=False,
                 seed=0, require_target=True, extra_filter=None, max_rows=None) -> ModelData:
    """Read + purify one data set section (``dataSet`` or an eval's ``dataSet``)."""
    plan = plan_dataset(mc, data_conf, columns_num, columns_str, extra_filter)
    table = read_table(plan.data_path, plan.header, plan.delim, numeric=plan.nums, strings=plan.strs,
                       missing=plan.missing, skip_header_line=plan.skip_header_line, max_rows=max_rows)
    return finish_table(mc, plan, table, sample_rate, sample_neg_only, seed, require_target)
