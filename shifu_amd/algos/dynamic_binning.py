"""IV-keeping re-binning of an existing ColumnConfig binning (``shifu stats -rebin``).

Same semantics as the reference's ``ColumnConfigDynamicBinning.run``
(J/core/binning/ColumnConfigDynamicBinning.java:35-68) with ``AutoDynamicBinning.merge``
(J/core/binning/AutoDynamicBinning.java:20-110):

1. the column's bins (numeric: by left boundary; categorical: one bin per category, sorted by
   positive rate) are merged pairwise, always the adjacent pair whose merge loses the least
   entropy, until at most ``expected_bins`` remain (``expected_bins <= 0``: no cap);
2. bins with fewer than ``min_inst_cnt`` instances are merged into the neighbour with the closer
   positive rate (first / last bin into their only neighbour);
3. while merging one more pair keeps IV >= ``iv_keep_ratio`` x the IV after step 2, merge.

The missing-value bin (last slot of every ``binCount*`` list) never takes part in merging; it is
carried over unchanged and counts in the IV.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

EPS = 1e-6                      # AutoDynamicBinning.EPS
CATEGORICAL_GROUP_VAL_DELIMITER = "@^"   # Constants.CATEGORICAL_GROUP_VAL_DELIMITER


@dataclass
class BinInfo:
    pos: float
    neg: float
    wpos: float
    wneg: float
    left: float = 0.0                       # numeric: left threshold
    values: list = field(default_factory=list)   # categorical: member categories

    @property
    def total(self) -> float:
        return self.pos + self.neg

    @property
    def pos_rate(self) -> float:
        return self.pos / self.total if self.total > 0 else 0.0

    def merge_right(self, o: "BinInfo") -> None:
        self.pos += o.pos
        self.neg += o.neg
        self.wpos += o.wpos
        self.wneg += o.wneg
        self.values = self.values + o.values

    def clone(self) -> "BinInfo":
        return BinInfo(self.pos, self.neg, self.wpos, self.wneg, self.left, list(self.values))


def _info_value(b: BinInfo, total: float) -> float:
    if b.total == 0:
        return 0.0
    pct = b.total / total
    pr = (b.pos + EPS) / b.total
    nr = (b.neg + EPS) / b.total
    return -pct * (pr * math.log2(pr) + nr * math.log2(nr))


def auto_dynamic_merge(bins: list[BinInfo], expected: int) -> list[BinInfo]:
    """AutoDynamicBinning.merge: adjacent merges with the smallest entropy change."""
    bins = list(bins)
    if len(bins) <= expected:
        return bins
    total = sum(b.total for b in bins)
    while len(bins) > expected:
        ent = sum(_info_value(b, total) for b in bins)
        best, best_red = 0, math.inf
        for pos in range(1, len(bins)):
            cur, nxt = bins[pos - 1], bins[pos]
            tmp = cur.clone()
            tmp.merge_right(nxt)
            merged = ent - _info_value(cur, total) - _info_value(nxt, total) + _info_value(tmp, total)
            red = merged - ent
            if red < best_red:
                best, best_red = pos, red
        if best <= 0:
            break
        bins[best - 1].merge_right(bins[best])
        del bins[best]
    return bins


def merge_small_bins(bins: list[BinInfo], min_cnt: float) -> list[BinInfo]:
    i = 0
    while i < len(bins):
        b = bins[i]
        if min_cnt > 0 and b.total < min_cnt and len(bins) > 1:
            if i == 0:
                b.merge_right(bins[1])
                del bins[1]
            elif i == len(bins) - 1:
                bins[i - 1].merge_right(b)
                del bins[i]
            else:
                prev, nxt = bins[i - 1], bins[i + 1]
                if abs(prev.pos_rate - b.pos_rate) < abs(b.pos_rate - nxt.pos_rate):
                    prev.merge_right(b)
                    del bins[i]
                else:
                    b.merge_right(nxt)
                    del bins[i + 1]
        else:
            i += 1
    return bins


def _iv(bins: list[BinInfo], missing: BinInfo) -> float:
    from .stats import column_metrics
    import numpy as np
    neg = np.array([b.neg for b in bins] + [missing.neg], float)
    pos = np.array([b.pos for b in bins] + [missing.pos], float)
    m = column_metrics(neg, pos)
    return m[1] if m else 0.0


def column_bin_infos(categorical: bool, boundaries_or_cats, cpos, cneg, wpos, wneg) -> tuple[list[BinInfo], BinInfo]:
    n = len(boundaries_or_cats)
    bins = []
    for i in range(n):
        b = BinInfo(float(cpos[i]), float(cneg[i]), float(wpos[i]), float(wneg[i]))
        if categorical:
            b.values = [boundaries_or_cats[i]]
        else:
            b.left = float(boundaries_or_cats[i])
        bins.append(b)
    bins.sort(key=(lambda b: b.pos_rate) if categorical else (lambda b: b.left))
    missing = BinInfo(float(cpos[-1]), float(cneg[-1]), float(wpos[-1]), float(wneg[-1]))
    return bins, missing


def dynamic_rebin(categorical: bool, boundaries_or_cats, cpos, cneg, wpos, wneg, expected_bins: int,
                  iv_keep_ratio: float = 1.0, min_inst_cnt: float = 0) -> tuple[list[BinInfo], BinInfo]:
    bins, missing = column_bin_infos(categorical, boundaries_or_cats, cpos, cneg, wpos, wneg)
    if expected_bins and expected_bins > 0:
        bins = auto_dynamic_merge(bins, expected_bins)
    if min_inst_cnt and min_inst_cnt > 0:
        bins = merge_small_bins(bins, min_inst_cnt)
    max_iv = _iv(bins, missing)
    while True:
        nxt = auto_dynamic_merge([b.clone() for b in bins], len(bins) - 1)
        if len(nxt) == len(bins) or _iv(nxt, missing) < max_iv * iv_keep_ratio:
            break
        bins = nxt
    return bins, missing
