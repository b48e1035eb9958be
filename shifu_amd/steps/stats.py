"""``stats`` step (B4): binning + column statistics, ``-c`` correlation, ``-p`` PSI, ``-rebin``.

``StatsModelProcessor.run`` (J/core/processor/StatsModelProcessor.java:116-251): one pass over the
purified (``stats.sampleRate``) data computes every column's bins and stats
(:func:`shifu_amd.algos.stats.compute_column_stats`); ``-c`` (``runCorrMapReduceJob`` :300,
``computeCorrValue`` :490) writes ``correlation.csv`` over the normalized candidate columns;
``-p`` runs PSI by ``stats.psiColumnName``; ``-rebin`` (``doReBin`` :670,
``ColumnConfigDynamicBinning`` J/core/binning/ColumnConfigDynamicBinning.java:27-180) merges
adjacent bins with the smallest IV loss down to ``-n`` bins (``-ivr`` keeps >= ratio of IV).
"""
from __future__ import annotations

import numpy as np

from ..algos import normalize as N
from ..algos import stats as S
from ..algos.binning import rebin_categorical
from ..utils.log import get_logger
from .base import ModelSet

_log = get_logger("steps.stats")


def run_stats(root: str = ".", correlation: bool = False, psi: bool = False, rebin: bool = False,
              expected_bins: int | None = None, iv_keep_ratio: float = 1.0, bin_avg_score_only: bool = False,
              device=None) -> int:
    ms = ModelSet(root).setup("STATS")
    mc = ms.mc
    cols = ms.stats_columns()
    if rebin:
        do_rebin(ms, expected_bins or int(mc.stats.get("maxNumBin", 10)), iv_keep_ratio)
        ms.save_cc(backup=True)
        return 0
    if correlation:                     # `stats -c` only computes correlation (stats must exist)
        run_correlation(ms, device)
        return 0
    if not psi:
        md = ms.load_raw(cols, sample_rate=float(mc.stats.get("sampleRate", 1.0)),
                         sample_neg_only=bool(mc.stats.get("sampleNegOnly", False)))
        _log.info("stats: %d valid rows (%s)", md.n, md.counters.as_dict())
        S.compute_column_stats(mc, ms.ccs, md, device=device, columns={c.name for c in cols})
        ms.save_cc(backup=True)
    if psi or mc.stats.get("psiColumnName"):
        unit = mc.stats.get("psiColumnName")
        if unit:
            cc_unit = [c for c in ms.ccs if c.name == unit]
            md = ms.load_raw(cols + cc_unit)
            S.compute_psi(mc, ms.ccs, md, unit)
            ms.save_cc()
        else:
            _log.warning("stats -p: stats.psiColumnName is empty")
    return 0


def run_correlation(ms: ModelSet, device=None):
    """Pairwise-complete Pearson over numeric raw values (categoricals via their pos-rate encoding),
    written as ``correlation.csv`` (header row + one row per column, ``ColumnConfig`` order)."""
    mc = ms.mc
    cols = [c for c in ms.stats_columns() if c.bin_boundary or c.bin_category]
    md = ms.load_raw(cols)
    mats = []
    for c in cols:
        col = md.table[c.name]
        if c.is_categorical():
            mats.append(N.normalize_column(c, col, "OLD_ZSCALE", None)[:, 0])
        else:
            v = col.numeric().astype(np.float64)
            mats.append(v)
    X = np.stack(mats, 1) if mats else np.zeros((md.n, 0))
    C = S.pearson_correlation(X, device)
    path = ms.pf.correlation_csv
    with open(path, "w") as f:
        f.write("," + ",".join(c.name for c in cols) + "\n")
        for i, c in enumerate(cols):
            f.write(c.name + "," + ",".join(repr(float(v)) for v in C[i]) + "\n")
    _log.info("correlation: %d columns -> %s", len(cols), path)
    return C, [c.num for c in cols]


def read_correlation(path: str):
    with open(path) as f:
        names = f.readline().rstrip("\n").split(",")[1:]
        rows = [list(map(float, l.rstrip("\n").split(",")[1:])) for l in f if l.strip()]
    return names, np.array(rows)


def _iv(pos, neg):
    m = S.column_metrics(neg, pos)
    return m[1] if m else 0.0


def rebin_numeric(bounds, cpos, cneg, wpos, wneg, target_bins: int, iv_keep_ratio: float = 1.0):
    """Greedy adjacent merge minimizing IV loss (missing bin last, never merged)."""
    b = list(bounds)
    cp, cn = list(cpos[:-1]), list(cneg[:-1])
    wp, wn = list(wpos[:-1]), list(wneg[:-1])
    miss = (cpos[-1], cneg[-1], wpos[-1], wneg[-1])
    full_iv = _iv(np.array(cp + [miss[0]]), np.array(cn + [miss[1]]))
    while len(b) > max(1, target_bins):
        best, best_iv = None, -np.inf
        for i in range(len(b) - 1):
            p2 = cp[:i] + [cp[i] + cp[i + 1]] + cp[i + 2:] + [miss[0]]
            n2 = cn[:i] + [cn[i] + cn[i + 1]] + cn[i + 2:] + [miss[1]]
            v = _iv(np.array(p2), np.array(n2))
            if v > best_iv:
                best, best_iv = i, v
        if iv_keep_ratio < 1.0 and full_iv > 0 and best_iv < iv_keep_ratio * full_iv:
            break
        i = best
        cp[i:i + 2] = [cp[i] + cp[i + 1]]
        cn[i:i + 2] = [cn[i] + cn[i + 1]]
        wp[i:i + 2] = [wp[i] + wp[i + 1]]
        wn[i:i + 2] = [wn[i] + wn[i + 1]]
        del b[i + 1]
    return b, cp + [miss[0]], cn + [miss[1]], wp + [miss[2]], wn + [miss[3]]


def do_rebin(ms: ModelSet, target_bins: int, iv_keep_ratio: float = 1.0):
    binary = ms.mc.is_binary()
    for c in ms.stats_columns():
        if c.bin_count_pos is None:
            continue
        cp, cn = np.asarray(c.bin_count_pos), np.asarray(c.bin_count_neg)
        wp, wn = np.asarray(c.bin_weighted_pos), np.asarray(c.bin_weighted_neg)
        if c.is_categorical():
            cats = c.bin_category or []
            if len(cats) <= target_bins:
                continue
            cats2, cp2, cn2, wp2, wn2 = rebin_categorical(cats, list(cp), list(cn), list(wp), list(wn), target_bins)
            c.bin_category = cats2
        else:
            bb = c.bin_boundary or []
            if len(bb) <= target_bins:
                continue
            bb2, cp2, cn2, wp2, wn2 = rebin_numeric(bb, cp, cn, wp, wn, target_bins, iv_keep_ratio)
            c.bin_boundary = bb2
        cb = c.binning
        cb["binCountPos"], cb["binCountNeg"] = [int(x) for x in cp2], [int(x) for x in cn2]
        cb["binWeightedPos"], cb["binWeightedNeg"] = [float(x) for x in wp2], [float(x) for x in wn2]
        cb["length"] = len(cp2) - 1
        cp2, cn2 = np.array(cp2, float), np.array(cn2, float)
        cb["binPosRate"] = [float(x) for x in np.where(cp2 + cn2 > 0, cp2 / np.maximum(cp2 + cn2, 1), 0.0)]
        if binary:
            m, mw = S.column_metrics(cn2, cp2), S.column_metrics(np.array(wn2), np.array(wp2))
            if m:
                c.stats["ks"], c.stats["iv"], c.stats["woe"] = m[0], m[1], m[2]
                cb["binCountWoe"] = m[3]
            if mw:
                c.stats["weightedKs"], c.stats["weightedIv"], c.stats["weightedWoe"] = mw[0], mw[1], mw[2]
                cb["binWeightedWoe"] = mw[3]
