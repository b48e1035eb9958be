"""Binning (H1).

Numerical boundaries are left-inclusive ``[b_i, b_{i+1})`` with ``b_0 = -inf`` and an extra
missing bin (``DTWorker.getBinIndex`` J/core/dtrain/dt/DTWorker.java:1001-1034, BinUtils).
Which rows feed the boundary computation follows ``FilterBinningDataUDF.isValidRecord``
(J/udf/FilterBinningDataUDF.java:59-85): EqualPositive -> positive rows only, EqualNegtive ->
negative rows, EqualTotal / EqualInterval / DynamicBinning -> all rows; ``Weight*`` variants
weight each value by its significance.

Deviation (documented): the reference's SPDT/SPDTI streaming histogram
(``EqualPopulationBinning`` J/core/binning/EqualPopulationBinning.java) is an approximation;
we compute *exact* weighted equal-population cuts from the sorted values (GPU sort / numpy).
When a column has <= maxNumBin distinct values every value is its own bin with boundaries at
mid-points (``convertHistogramUnitIntoBin`` semantics).
"""
from __future__ import annotations

import math

import numpy as np
import torch


def equal_population_boundaries(values: np.ndarray, n_bins: int, weights: np.ndarray | None = None) -> list:
    v = np.asarray(values, dtype=np.float64)
    ok = np.isfinite(v)
    v = v[ok]
    w = None if weights is None else np.asarray(weights, dtype=np.float64)[ok]
    if v.size == 0:
        return [float("-inf")]
    if v.size > 4_000_000 and torch.cuda.is_available():
        tv = torch.from_numpy(v).cuda()
        order = torch.argsort(tv)
        vs = tv[order].cpu().numpy()
        ws = None if w is None else w[order.cpu().numpy()]
    else:
        order = np.argsort(v, kind="stable")
        vs = v[order]
        ws = None if w is None else w[order]
    uniq, first = np.unique(vs, return_index=True)
    cnt = np.diff(np.append(first, vs.size)).astype(np.float64) if ws is None else \
        np.add.reduceat(ws, first)
    bounds = [float("-inf")]
    if uniq.size <= n_bins:
        for i in range(1, uniq.size):
            bounds.append(float((uniq[i - 1] + uniq[i]) / 2.0))
        return bounds
    cum = np.cumsum(cnt)
    total = cum[-1]
    for j in range(1, n_bins):
        s = j * total / n_bins
        k = int(np.searchsorted(cum, s, side="left"))
        if k >= uniq.size - 1:
            continue
        b = float((uniq[k] + uniq[k + 1]) / 2.0)
        if b > bounds[-1]:
            bounds.append(b)
    return bounds


def sketch_boundaries(values: np.ndarray, n_bins: int, algorithm: str, weights=None) -> list:
    """Reference-parity cuts from the streaming sketches of ``stats.binningAlgorithm``
    (runtime/csrc/binning_stream.cpp): SPDT / SPDTI -> ``EqualPopulationBinning``,
    MunroPat / MunroPatI -> ``MunroPatBinning``; values in row order, NaN = missing."""
    from ..ops import _native
    lib = _native.rt()
    if lib is None:
        raise RuntimeError("binning parity mode needs the native runtime library (g++)")
    v = np.ascontiguousarray(values, dtype=np.float64)
    cap = max(4 * n_bins + 8, 64)
    out = np.empty(cap, np.float64)
    algo = algorithm.upper()
    if algo.startswith("SPDT"):
        w = None if weights is None else np.ascontiguousarray(weights, dtype=np.float64)
        n = lib.shifu_spdt_bins(v.ctypes.data, None if w is None else w.ctypes.data, v.size, int(n_bins),
                                out.ctypes.data, cap)
    elif algo.startswith("MUNROPAT"):
        n = lib.shifu_munropat_bins(v.ctypes.data, v.size, int(n_bins), out.ctypes.data, cap)
    else:
        raise ValueError(f"no streaming sketch for binning algorithm {algorithm!r}")
    if n < 0:
        raise ValueError(f"sketch binning failed ({algorithm}, bins={n_bins})")
    if n > cap:
        out = np.empty(n, np.float64)
        n = lib.shifu_spdt_bins(v.ctypes.data, None, v.size, int(n_bins), out.ctypes.data, n) \
            if algo.startswith("SPDT") else lib.shifu_munropat_bins(v.ctypes.data, v.size, int(n_bins),
                                                                      out.ctypes.data, n)
    return [float(x) for x in out[:n]]


def equal_interval_boundaries(values: np.ndarray, n_bins: int) -> list:
    v = np.asarray(values, dtype=np.float64)
    v = v[np.isfinite(v)]
    if v.size == 0:
        return [float("-inf")]
    lo, hi = float(v.min()), float(v.max())
    if hi <= lo:
        return [float("-inf")]
    step = (hi - lo) / n_bins
    return [float("-inf")] + [lo + i * step for i in range(1, n_bins)]


def bin_index_numeric(values: np.ndarray, boundaries) -> np.ndarray:
    """Left-inclusive bin index; NaN/missing -> len(boundaries) (the missing bin)."""
    b = np.asarray(boundaries, dtype=np.float64)
    v = np.asarray(values, dtype=np.float64)
    idx = np.searchsorted(b, v, side="right") - 1
    idx = np.clip(idx, 0, len(b) - 1)
    idx[~np.isfinite(v) & ~np.isinf(v)] = len(b)
    # +inf -> last bin, -inf -> first bin (getBinIndex)
    return idx.astype(np.int32)


def bin_index_torch(values: torch.Tensor, boundaries: torch.Tensor) -> torch.Tensor:
    idx = torch.bucketize(values, boundaries, right=True) - 1
    idx = idx.clamp(0, boundaries.numel() - 1)
    idx = torch.where(torch.isnan(values), torch.full_like(idx, boundaries.numel()), idx)
    return idx.to(torch.int32)


def categorical_bins(codes: np.ndarray, dictionary: list, y: np.ndarray, is_binary: bool,
                     max_cate: int = 10000):
    """Categories ordered by first appearance (CategoricalBinning keeps insertion order)."""
    present = np.unique(codes[codes >= 0])
    cats = [dictionary[i] for i in sorted(present)]
    return cats[:max_cate] if len(cats) > max_cate else cats


def category_index(codes: np.ndarray, dictionary: list, categories: list) -> np.ndarray:
    """Row category code -> bin index in ``categories``; missing/unknown -> len(categories)."""
    pos = {c: i for i, c in enumerate(categories)}
    lut = np.array([pos.get(s, len(categories)) for s in dictionary] + [len(categories)], dtype=np.int32)
    return lut[np.where(codes >= 0, codes, len(dictionary))]


def rebin_categorical(cats, cpos, cneg, wpos, wneg, max_bins: int):
    """``UpdateBinningInfoReducer.rebinCategoricalValues``: merge categories with similar
    positive rate (sorted by rate, adjacent merge minimizing IV loss) down to ``max_bins``;
    merged categories are joined with '^' (CalculateStatsUDF.CATEGORY_VAL_SEPARATOR)."""
    n = len(cats)
    if n <= max_bins:
        return cats, cpos, cneg, wpos, wneg
    rate = [(cpos[i] / (cpos[i] + cneg[i]) if cpos[i] + cneg[i] > 0 else 0.0, i) for i in range(n)]
    rate.sort()
    groups = [[i] for _, i in rate]
    tp, tn = sum(cpos[:n]) or 1, sum(cneg[:n]) or 1

    def iv(g):
        p = sum(cpos[i] for i in g) / tp
        q = sum(cneg[i] for i in g) / tn
        return (q - p) * math.log((q + 1e-10) / (p + 1e-10))
    while len(groups) > max_bins:
        best, bi = None, 0
        for k in range(len(groups) - 1):
            loss = iv(groups[k]) + iv(groups[k + 1]) - iv(groups[k] + groups[k + 1])
            if best is None or loss < best:
                best, bi = loss, k
        groups[bi] = groups[bi] + groups.pop(bi + 1)
    ncats = ["^".join(cats[i] for i in g) for g in groups]
    agg = lambda arr: [sum(arr[i] for i in g) for g in groups] + [arr[n]]  # noqa: E731
    return ncats, agg(cpos), agg(cneg), agg(wpos), agg(wneg)
