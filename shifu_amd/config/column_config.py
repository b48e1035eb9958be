"""ColumnConfig.json (C2): per-column type/flag/stats/binning.

Mirrors ``J/container/obj/ColumnConfig.java:38-99``, ``ColumnStats.java:37-142`` and
``ColumnBinning.java:40-96``.  Dict-backed so unknown keys and key order round-trip.
"""
from __future__ import annotations

import math
from collections import OrderedDict

from . import jsonio

STATS_KEYS = ("max", "min", "mean", "median", "totalCount", "distinctCount", "missingCount", "validNumCount",
              "stdDev", "missingPercentage", "woe", "ks", "iv", "weightedKs", "weightedIv", "weightedWoe",
              "skewness", "kurtosis", "psi", "unitStats", "25th", "75th")
BINNING_KEYS = ("length", "binBoundary", "binCategory", "binCountNeg", "binCountPos", "binPosRate",
                "binAvgScore", "binWeightedNeg", "binWeightedPos", "binCountWoe", "binWeightedWoe")


class ColumnConfig:
    def __init__(self, d=None):
        d = OrderedDict(d or {})
        d.setdefault("columnNum", 0)
        d.setdefault("columnName", "")
        d.setdefault("version", "0.13.0")
        d.setdefault("columnType", "N")
        d.setdefault("columnFlag", None)
        d.setdefault("finalSelect", False)
        cs = d.get("columnStats") or OrderedDict()
        for k in ("max", "min", "mean", "median", "totalCount", "distinctCount", "missingCount", "validNumCount",
                  "stdDev", "missingPercentage", "woe", "ks", "iv", "weightedKs", "weightedIv", "weightedWoe",
                  "skewness", "kurtosis", "psi", "unitStats"):
            cs.setdefault(k, None)
        d["columnStats"] = cs
        cb = d.get("columnBinning") or OrderedDict()
        cb.setdefault("length", 0)
        for k in BINNING_KEYS[1:]:
            cb.setdefault(k, None)
        d["columnBinning"] = cb
        self.d = d

    # ---- core ---------------------------------------------------------------------------
    @property
    def num(self) -> int:
        return int(self.d["columnNum"])

    @num.setter
    def num(self, v):
        self.d["columnNum"] = int(v)

    @property
    def name(self) -> str:
        return self.d["columnName"]

    @name.setter
    def name(self, v):
        self.d["columnName"] = v

    @property
    def type(self):
        return self.d.get("columnType")

    @type.setter
    def type(self, v):
        self.d["columnType"] = v

    @property
    def flag(self):
        return self.d.get("columnFlag")

    @flag.setter
    def flag(self, v):
        self.d["columnFlag"] = v

    @property
    def final_select(self) -> bool:
        return bool(self.d.get("finalSelect"))

    @final_select.setter
    def final_select(self, v):
        self.d["finalSelect"] = bool(v)

    @property
    def stats(self) -> OrderedDict:
        return self.d["columnStats"]

    @property
    def binning(self) -> OrderedDict:
        return self.d["columnBinning"]

    # ---- predicates (ColumnConfig.java isXxx) -------------------------------------------------
    def is_target(self):
        return self.flag == "Target"

    def is_meta(self):
        return self.flag == "Meta"

    def is_weight(self):
        return self.flag == "Weight"

    def is_force_select(self):
        return self.flag == "ForceSelect"

    def is_force_remove(self):
        return self.flag == "ForceRemove"

    def is_candidate_flag(self):
        return self.flag == "Candidate"

    def is_categorical(self):
        return self.type == "C"

    def is_hybrid(self):
        return self.type == "H"

    def is_numerical(self):
        return self.type in ("N", "H") or self.type is None and not self.is_target() and not self.is_meta()

    def is_candidate(self, has_candidates: bool = False) -> bool:
        """CommonUtils.isGoodCandidate semantics: not target/meta/weight/forceRemove and has stats."""
        if self.is_target() or self.is_meta() or self.is_weight() or self.is_force_remove():
            return False
        if has_candidates and not (self.is_candidate_flag() or self.is_force_select()):
            return False
        return True

    def is_good_candidate(self, has_candidates: bool = False, is_binary: bool = True) -> bool:
        if not self.is_candidate(has_candidates):
            return False
        if self.is_categorical():
            cats = self.bin_category
            return bool(cats) and len(cats) > 0
        bb = self.bin_boundary
        if not bb or len(bb) <= 1:
            return False
        if is_binary:
            ks, iv = self.stats.get("ks"), self.stats.get("iv")
            if ks is None and iv is None:
                return True
            return (ks or 0) > 0 or (iv or 0) > 0
        return True

    # ---- binning -------------------------------------------------------------------------
    @property
    def bin_boundary(self):
        bb = self.binning.get("binBoundary")
        return None if bb is None else [jsonio.to_double(x) for x in bb]

    @bin_boundary.setter
    def bin_boundary(self, v):
        self.binning["binBoundary"] = None if v is None else [float(x) for x in v]

    @property
    def bin_category(self):
        return self.binning.get("binCategory")

    @bin_category.setter
    def bin_category(self, v):
        self.binning["binCategory"] = None if v is None else [str(x) for x in v]

    def n_bins(self) -> int:
        """Bins incl. the missing bin (numerical: len(boundary)+1; categorical: len(cats)+1)."""
        if self.is_categorical():
            return len(self.bin_category or []) + 1
        return len(self.bin_boundary or []) + 1

    def _dl(self, k):
        v = self.binning.get(k)
        return None if v is None else [jsonio.to_double(x) for x in v]

    @property
    def bin_pos_rate(self):
        return self._dl("binPosRate")

    @property
    def bin_count_woe(self):
        return self._dl("binCountWoe")

    @property
    def bin_weighted_woe(self):
        return self._dl("binWeightedWoe")

    @property
    def bin_count_pos(self):
        return self.binning.get("binCountPos")

    @property
    def bin_count_neg(self):
        return self.binning.get("binCountNeg")

    @property
    def bin_weighted_pos(self):
        return self._dl("binWeightedPos")

    @property
    def bin_weighted_neg(self):
        return self._dl("binWeightedNeg")

    @property
    def bin_avg_score(self):
        return self.binning.get("binAvgScore")

    # ---- stats ---------------------------------------------------------------------------
    def stat(self, k, default=None):
        v = self.stats.get(k)
        return default if v is None else jsonio.to_double(v) if isinstance(v, str) else v

    @property
    def mean(self):
        return self.stat("mean")

    @property
    def std_dev(self):
        return self.stat("stdDev")

    @property
    def ks(self):
        return self.stat("ks")

    @property
    def iv(self):
        return self.stat("iv")

    @property
    def missing_pct(self):
        return self.stat("missingPercentage")

    @property
    def woe(self):
        return self.stat("woe")

    def to_dict(self):
        return self.d

    def __repr__(self):
        return f"ColumnConfig({self.num}, {self.name!r}, type={self.type}, flag={self.flag}, sel={self.final_select})"


def _clean(v):
    if isinstance(v, float) and (math.isnan(v) or math.isinf(v)):
        return v   # jsonio writes non-finite doubles as strings
    return v


def load_column_configs(path: str):
    return [ColumnConfig(d) for d in jsonio.load(path)]


def save_column_configs(ccs, path: str):
    jsonio.dump([c.to_dict() for c in ccs], path)


def has_candidates(ccs) -> bool:
    return any(c.is_candidate_flag() for c in ccs)


def selected_columns(ccs):
    """Final-selected model inputs in column order (DTrainUtils.getNumericAndCategoricalInputAndOutputCounts)."""
    out = [c for c in ccs if c.final_select and not c.is_target() and not c.is_meta()]
    return out


def target_column(ccs):
    for c in ccs:
        if c.is_target():
            return c
    return None


def weight_column(ccs):
    for c in ccs:
        if c.is_weight():
            return c
    return None


def model_input_columns(ccs, is_binary: bool = True):
    """Model inputs: the final-selected columns, or — before any variable selection — every good
    candidate plus force-selected columns (``DTrainUtils.getNumericAndCategoricalInputAndOutputCounts``
    falls back to candidates when nothing is finalSelect)."""
    sel = selected_columns(ccs)
    if sel:
        return sel
    hc = has_candidates(ccs)
    return [c for c in ccs if (c.is_good_candidate(hc, is_binary) or c.is_force_select())
            and not c.is_target() and not c.is_meta()]
