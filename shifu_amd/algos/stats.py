"""Column statistics (H2) + KS/IV/WOE (K3) + PSI (H4).

Per column, over purified rows (``UpdateBinningInfoMapper.populateStats``
J/core/binning/UpdateBinningInfoMapper.java:427-598 and ``UpdateBinningInfoReducer.reduce``
J/core/binning/UpdateBinningInfoReducer.java:125-433):
  * bins (+ missing bin) with pos/neg counts and weighted sums
  * count / missing / sum / sum^2 / sum^3 / sum^4 / min / max of valid numeric values
  * mean, stdDev (sample, with the reference's +EPS), skewness, kurtosis (population sigma)
  * p25 / median / p75 interpolated inside bins
  * KS x100, IV, WOE and per-bin WOE ``ln((n+eps)/(p+eps))`` (``ColumnStatsCalculator`` long[]/double[]
    variants, J/core/ColumnStatsCalculator.java:76-165) for binary targets
  * categorical: pos-rate per bin, stats recomputed over bin pos-rates
  * distinct count (exact; the reference uses HyperLogLog++)

The per-column histogram + moments run through torch on the device the data lives on (GPU
when available), the KS/IV scan is O(bins).
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

from ..utils.log import get_logger
from . import binning as B

_log = get_logger("algos.stats")
EPS = 1e-10


def column_metrics(neg, pos):
    """ColumnStatsCalculator.calculateColumnMetrics: (ks*100, iv, woe, bin_woe) or None."""
    neg = np.asarray(neg, dtype=np.float64)
    pos = np.asarray(pos, dtype=np.float64)
    sn, sp = neg.sum(), pos.sum()
    if sn == 0 or sp == 0:
        return None
    woe = math.log((sn + EPS) / (sp + EPS))
    p = pos / sp
    n = neg / sn
    bw = np.log((n + EPS) / (p + EPS))
    iv = float(((n - p) * bw).sum())
    ks = float(np.abs(np.cumsum(p) - np.cumsum(n)).max())
    return ks * 100.0, iv, woe, [float(x) for x in bw]


def _hist(bin_idx: np.ndarray, y: np.ndarray, w: np.ndarray, nb: int, binary: bool, dev):
    b = torch.as_tensor(bin_idx, device=dev, dtype=torch.int64)
    yy = torch.as_tensor(y, device=dev, dtype=torch.float32)
    ww = torch.as_tensor(w, device=dev, dtype=torch.float64)
    if binary:
        pos = yy > 0.5
        cpos = torch.bincount(b[pos], minlength=nb)[:nb]
        cneg = torch.bincount(b[~pos], minlength=nb)[:nb]
        wpos = torch.bincount(b[pos], weights=ww[pos], minlength=nb)[:nb]
        wneg = torch.bincount(b[~pos], weights=ww[~pos], minlength=nb)[:nb]
    else:
        cpos = torch.bincount(b, minlength=nb)[:nb]
        cneg = torch.zeros_like(cpos)
        wpos = torch.bincount(b, weights=ww, minlength=nb)[:nb]
        wneg = torch.zeros_like(wpos)
    return (cpos.cpu().numpy().astype(np.int64), cneg.cpu().numpy().astype(np.int64),
            wpos.cpu().numpy(), wneg.cpu().numpy())


def _moments(v: np.ndarray, dev):
    t = torch.as_tensor(v, device=dev, dtype=torch.float64)
    ok = torch.isfinite(t)
    x = t[ok]
    n = int(x.numel())
    if n == 0:
        return n, 0.0, 0.0, 0.0, 0.0, float("nan"), float("nan")
    x2 = x * x
    return (n, float(x.sum()), float(x2.sum()), float((x2 * x).sum()), float((x2 * x2).sum()),
            float(x.min()), float(x.max()))


def _finish_moments(cc, count, s1, s2, s3, s4, mn, mx, total, missing):
    real = count
    if real > 0:
        mean = s1 / real
        std = math.sqrt(abs((s2 - s1 * s1 / real + EPS) / (real - 1))) if real > 1 else 0.0
        astd = math.sqrt(abs((s2 - s1 * s1 / real + EPS) / real))
        skew = (s3 - 3 * s2 * mean + 3 * mean * mean * s1 - real * mean ** 3) / (real * astd ** 3) \
            if astd > 0 else 0.0
        kurt = (s4 - 4 * s3 * mean + 6 * s2 * mean * mean - 4 * s1 * mean ** 3 + real * mean ** 4) / \
            (real * astd ** 4) if astd > 0 else 0.0
    else:
        mean = std = skew = kurt = 0.0
    st = cc.stats
    st["max"] = float(mx) if mx == mx else None
    st["min"] = float(mn) if mn == mn else None
    st["mean"] = float(mean)
    st["stdDev"] = float(std)
    st["skewness"] = float(skew)
    st["kurtosis"] = float(kurt)
    st["totalCount"] = int(total)
    st["missingCount"] = int(missing)
    st["missingPercentage"] = float(missing) / total if total else 0.0


def _percentiles(bounds, counts, mn, mx, count):
    """Interpolated p25/median/p75 inside bins (UpdateBinningInfoReducer.reduce :229-262)."""
    p25c = count // 4
    medc = p25c * 2
    p75c = p25c * 3
    p25 = med = p75 = mn
    cur = 0

    def cut(b):
        return mx if b > mx else (mn if b < mn else b)
    for i in range(len(bounds)):
        left = cut(bounds[i])
        right = mx if i == len(bounds) - 1 else cut(bounds[i + 1])
        c = counts[i]
        if c > 0:
            if cur <= p25c < cur + c:
                p25 = (p25c - cur) / c * (right - left) + left
            if cur <= medc < cur + c:
                med = (medc - cur) / c * (right - left) + left
            if cur <= p75c < cur + c:
                p75 = (p75c - cur) / c * (right - left) + left
                break
        cur += c
    return p25, med, p75


_DEFER = None      # list while a deferred_metrics block is open (K3 batched on the device)


class deferred_metrics:
    """K3 on the device: inside the block ``_finish_binning`` queues each column's (neg, pos)
    bins; on exit ONE ``column_metrics_kernel`` launch computes KS / IV / WOE / per-bin WOE of the
    counts and weighted bins of every queued column.  A no-op on the CPU (the host oracle
    ``column_metrics`` runs per column)."""

    def __init__(self, dev):
        self.on = torch.device(dev).type == "cuda" if dev is not None else False
        self.dev = dev

    def __enter__(self):
        global _DEFER
        self.prev = _DEFER
        if self.on:
            _DEFER = []
        return self

    def __exit__(self, exc_type, *exc):
        global _DEFER
        q = _DEFER if self.on else None
        _DEFER = self.prev
        if exc_type is None and q:
            from ..ops.stats_ops import column_metrics_batch
            res = column_metrics_batch([(c[2], c[4]) for c in q], [(c[1], c[3]) for c in q], self.dev)
            for (cc, *_), (m, mw) in zip(q, res):
                _apply_metrics(cc, len(_[0]), m, mw)
        return False


def _apply_metrics(cc, nb, m, mw):
    zero = [0.0] * nb
    cc.stats["ks"], cc.stats["iv"], cc.stats["woe"] = (m[0], m[1], m[2]) if m else (None, None, None)
    cc.stats["weightedKs"], cc.stats["weightedIv"], cc.stats["weightedWoe"] = \
        (mw[0], mw[1], mw[2]) if mw else (None, None, None)
    cc.binning["binCountWoe"] = m[3] if m else zero
    cc.binning["binWeightedWoe"] = mw[3] if mw else zero


def _finish_binning(cc, binary, nb, cpos, cneg, wpos, wneg, total):
    """Write binning arrays + KS/IV/WOE for one column (shared by the CPU and HIP paths)."""
    if binary:
        rate = np.where(cpos + cneg > 0, cpos / np.maximum(cpos + cneg, 1), 0.0)
    else:
        tot = cpos.sum()
        rate = cpos / tot if tot else np.zeros(nb)
    cc.stats["validNumCount"] = int(total - cc.stats.get("missingCount", 0))
    cb = cc.binning
    cb["length"] = int(nb - 1)
    cb["binCountPos"] = [int(x) for x in cpos]
    cb["binCountNeg"] = [int(x) for x in cneg]
    cb["binWeightedPos"] = [float(x) for x in wpos]
    cb["binWeightedNeg"] = [float(x) for x in wneg]
    cb["binPosRate"] = [float(x) for x in rate]
    if binary:
        if _DEFER is not None:         # K3 batched on the device at the end of the pass
            _DEFER.append((cc, np.asarray(cpos, np.float64), np.asarray(cneg, np.float64),
                           np.asarray(wpos, np.float64), np.asarray(wneg, np.float64)))
            return
        _apply_metrics(cc, nb, column_metrics(cneg, cpos), column_metrics(wneg, wpos))
    else:
        cb["binCountWoe"] = [0.0] * nb
        cb["binWeightedWoe"] = [0.0] * nb


# columns up to this many rows get an exact distinct count (one batched device sort); larger
# ones keep the K4 histogram count (exact for low-cardinality columns) or the HLL estimate -- the
# reference itself reports HyperLogLogPlus estimates for every column
EXACT_DISTINCT_ROWS = 1 << 22


_STAGE = {}


def upload_columns(cols, dev) -> torch.Tensor:
    """Host numeric columns -> one column-major [C, n] float64 device tensor.  GPU: the columns are
    packed into one of two pinned staging buffers and sent with ONE async H2D copy (per-column
    pageable copies cost a synchronous round trip each: ~1600 per chunk for a 1600-column table);
    an event per buffer keeps a refill from overtaking its previous copy."""
    n = len(cols[0]) if cols else 0
    C = len(cols)
    out = torch.empty((C, n), dtype=torch.float64, device=dev)
    if dev.type != "cuda" or C * n == 0 or C * n * 8 > (256 << 20):
        # (large columns: each copy is big enough to amortise its round trip; no pinned staging)
        for k, v in enumerate(cols):
            out[k].copy_(torch.from_numpy(np.ascontiguousarray(v, dtype=np.float64)))
        return out
    import threading
    key = (str(dev), threading.get_ident())       # per thread: stats lanes upload concurrently
    st = _STAGE.setdefault(key, {"bufs": [None, None], "ev": [None, None], "i": 0})
    i = st["i"]
    st["i"] ^= 1
    buf = st["bufs"][i]
    if buf is None or buf.numel() < C * n:
        buf = torch.empty(max(C * n, 1 << 20), dtype=torch.float64, pin_memory=True)
        st["bufs"][i], st["ev"][i] = buf, None
    if st["ev"][i] is not None:
        st["ev"][i].synchronize()                 # the copy that last read this buffer is done
    host = buf[: C * n].numpy().reshape(C, n)
    from ..data.reader import numeric_rows
    hit = numeric_rows(cols)
    if hit is not None and np.array_equal(hit[1], np.arange(hit[1][0], hit[1][0] + C)):
        host[:] = hit[0][hit[1][0]: hit[1][0] + C]     # a run of the parser's block rows: one memcpy
    else:
        for k, v in enumerate(cols):
            host[k] = v
    out.copy_(buf[: C * n].view(C, n), non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(dev))
    st["ev"][i] = ev
    return out


def exact_distinct(vals: torch.Tensor, num_thr: float) -> list:
    """Distinct finite values per row of ``vals`` [C, n] (threshold -> invalid, -0.0 == 0.0)."""
    v = torch.where(vals > num_thr, torch.full_like(vals, float("nan")), vals) + 0.0
    v = torch.where(torch.isfinite(v), v, torch.full_like(v, float("inf")))
    s, _ = torch.sort(v, dim=1)
    fin = torch.isfinite(s)
    if s.shape[1] == 0:
        return [0] * s.shape[0]
    first = fin[:, :1].long().sum(1)
    chg = ((s[:, 1:] != s[:, :-1]) & fin[:, 1:]).long().sum(1)
    return (first + chg).cpu().tolist()


def batch_histograms(vals: torch.Tensor, y: torch.Tensor, w: torch.Tensor, bounds, binary: bool,
                     num_thr: float = 1.7976931348623157e308):
    """K1+K2 for a column batch ``vals`` [C, n]: per column (cpos, cneg, wpos, wneg, moments).
    GPU: the HIP ``column_stats`` kernel; CPU: the torch/numpy oracle with the same layout."""
    if vals.device.type == "cuda":
        from ..ops import stats_ops
        return stats_ops.column_stats(vals, y, w, bounds, binary, num_thr)
    yn = y.cpu().numpy() if torch.is_tensor(y) else np.asarray(y)
    wn = w.cpu().numpy() if torch.is_tensor(w) else np.asarray(w)
    out = []
    for c in range(vals.shape[0]):
        v = vals[c].cpu().numpy().astype(np.float64, copy=True)
        v[v > num_thr] = np.nan
        bidx = B.bin_index_numeric(v, bounds[c])
        cpos, cneg, wpos, wneg = _hist(bidx, yn, wn, len(bounds[c]) + 1, binary, torch.device("cpu"))
        mom = _moments(v, torch.device("cpu"))
        out.append((cpos, cneg, wpos, wneg, mom))
    return out


def run_lanes(fn, items, dev, lanes: int | None = None):
    """``[fn(item) for item in items]`` with ``lanes`` column batches in flight (worker threads, one
    HIP stream each): a batch's host planning between its K4 passes (~20 % of a 64-column batch at
    100M rows, profiles/r2/stats_host_vs_device_per_batch_r2r.txt) overlaps the other batch's
    kernels.  Single-process only (the data-parallel passes issue collectives, whose order must
    match across ranks); ``SHIFU_STATS_LANES`` (default 2) sets the width."""
    from ..parallel import dist
    lanes = int(os.environ.get("SHIFU_STATS_LANES", "2")) if lanes is None else lanes
    if lanes <= 1 or len(items) <= 1 or dev.type != "cuda" or dist.info().world_size > 1:
        return [fn(it) for it in items]
    import threading
    main = torch.cuda.current_stream(dev)
    streams = [torch.cuda.Stream(dev) for _ in range(lanes)]
    for st in streams:
        st.wait_stream(main)                  # inputs produced on the caller's stream
    results, errors = [None] * len(items), []
    order = iter(range(len(items)))
    lock = threading.Lock()

    dev_index = dev.index if dev.index is not None else torch.cuda.current_device()

    def worker(k):
        try:
            torch.cuda.set_device(dev_index)
            with torch.cuda.stream(streams[k]):
                while not errors:
                    with lock:
                        i = next(order, None)
                    if i is None:
                        return
                    results[i] = fn(items[i])
        except BaseException as e:            # re-raised on the caller's thread
            errors.append(e)

    threads = [threading.Thread(target=worker, args=(k,), daemon=True) for k in range(min(lanes, len(items)))]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    for st in streams:
        main.wait_stream(st)
    if errors:
        raise errors[0]
    return results


def parity_algorithm(mc):
    """``shifu.stats.binning.parity=true`` + binningAlgorithm SPDT/SPDTI/MunroPat/MunroPatI: the
    reference's streaming-sketch cuts (BinningDataUDF semantics: every valid value of the column in
    row order, unweighted, whatever the class) instead of the exact equal-population cuts."""
    from ..config import environment
    algo = str(mc.stats.get("binningAlgorithm", "SPDTI") or "SPDTI")
    if not environment.get_bool("shifu.stats.binning.parity", False):
        return None
    if mc.binning_method in ("EqualInterval", "WeightEqualInterval"):
        return None
    return algo if algo.upper().startswith(("SPDT", "MUNROPAT")) else None


def _numeric_bounds(vals, y, w, binary, method, n_bins):
    if binary and method in ("EqualPositive", "WeightEqualPositive"):
        sel = y > 0.5
    elif binary and method in ("EqualNegtive", "WeightEqualNegative"):
        sel = y <= 0.5
    else:
        sel = np.ones(len(vals), dtype=bool)
    weighted = method.startswith("Weight")
    if method in ("EqualInterval", "WeightEqualInterval"):
        bounds = B.equal_interval_boundaries(vals[sel], n_bins)
    else:
        bounds = B.equal_population_boundaries(vals[sel], n_bins, w[sel] if weighted else None)
    if len(bounds) <= 1 and sel.sum() < len(vals):
        bounds = B.equal_population_boundaries(vals, n_bins)
    return bounds


def finish_categorical(cc, cats, cpos, cneg, wpos, wneg, total, binary, cate_max, dict_size):
    """Categorical column from its per-category histograms (last bin = missing/unknown):
    ``cateMaxNumBin`` merge, pos-rate moments (UpdateBinningInfoReducer.reduce :309-333), binning."""
    nb = len(cats) + 1
    if cate_max > 0 and len(cats) > cate_max:
        cats, cpos, cneg, wpos, wneg = B.rebin_categorical(cats, list(cpos), list(cneg), list(wpos),
                                                           list(wneg), cate_max)
        cpos, cneg = np.array(cpos, np.int64), np.array(cneg, np.int64)
        wpos, wneg = np.array(wpos), np.array(wneg)
        nb = len(cats) + 1
    cc.bin_category = cats
    cc.bin_boundary = None
    missing = int(cpos[-1] + cneg[-1])
    if binary:
        rate = np.where(cpos + cneg > 0, cpos / np.maximum(cpos + cneg, 1), 0.0)
    else:
        tot = cpos.sum()
        rate = cpos / tot if tot else np.zeros_like(cpos, dtype=float)
    cnt = cpos + cneg if binary else cpos
    okr = np.isfinite(rate)
    mx = float(rate[okr].max()) if okr.any() else 0.0
    mn = float(rate[okr].min()) if okr.any() else 0.0
    _finish_moments(cc, total - missing, float((rate * cnt).sum()), float((rate ** 2 * cnt).sum()),
                    float((rate ** 3 * cnt).sum()), float((rate ** 4 * cnt).sum()), mn, mx, total, missing)
    cc.stats["distinctCount"] = int(dict_size)
    cc.stats["median"] = None
    _finish_binning(cc, binary, nb, cpos, cneg, wpos, wneg, total)


def _finish_numeric(cc, binary, bounds, cpos, cneg, wpos, wneg, mom, total, distinct):
    cc.bin_boundary = bounds
    cc.bin_category = None
    cnt, s1, s2, s3, s4, mn, mx = mom
    _finish_moments(cc, cnt, s1, s2, s3, s4, mn, mx, total, total - cnt)
    p25, med, p75 = _percentiles(bounds, (cpos + cneg) if binary else cpos, mn, mx, total)
    cc.stats["median"] = float(med)
    cc.stats["25th"] = float(p25)
    cc.stats["75th"] = float(p75)
    cc.stats["distinctCount"] = int(distinct)
    _finish_binning(cc, binary, len(bounds) + 1, cpos, cneg, wpos, wneg, total)


def compute_column_stats(mc, ccs, md, device=None, columns=None, gpu_batch: int = 64):
    """Fill ``columnBinning``/``columnStats`` of every candidate column from ModelData ``md``.

    Numeric columns on the GPU go through the fused HIP kernel (K1+K2: bin search + pos/neg
    histograms + fp64 moments for a batch of columns in one launch); the CPU path is the
    oracle with identical semantics."""
    from ..utils.device import is_gpu_available
    dev = torch.device(device or ("cuda" if is_gpu_available() else "cpu"))
    binary = mc.is_binary()
    method = mc.binning_method
    n_bins = int(mc.stats.get("maxNumBin", 10))
    cate_max = int(mc.stats.get("cateMaxNumBin", 0) or 0)
    num_thr = float(mc.stats.get("numericalValueThreshold", 1.7976931348623157e308))
    y, w = md.y, md.w
    total = md.n
    parity = parity_algorithm(mc)
    numeric = []
    for cc in ccs:
        if columns is not None and cc.name not in columns:
            continue
        if cc.is_target() or cc.is_meta() or cc.name not in md.table:
            continue
        col = md.table[cc.name]
        if not cc.is_categorical():
            numeric.append(cc)
            continue
        codes = col.values if col.kind == "str" else None
        if codes is None:   # numeric-parsed categorical: categories = formatted values
            s = col.strings()
            uniq = {}
            codes = np.array([uniq.setdefault(v, len(uniq)) if v != "" else -1 for v in s], dtype=np.int32)
            dictionary = list(uniq.keys())
        else:
            dictionary = col.dictionary
        cats = B.categorical_bins(codes, dictionary, y, binary)
        bidx = B.category_index(codes, dictionary, cats)
        cpos, cneg, wpos, wneg = _hist(bidx, y, w, len(cats) + 1, binary, dev)
        finish_categorical(cc, cats, cpos, cneg, wpos, wneg, total, binary, cate_max, len(dictionary))
    if not numeric:
        return ccs
    if dev.type == "cuda":
        # K4 on the device: exact cuts from the qprep/qhist/qgather passes (algos/quantile.py),
        # then K1+K2 (column_stats) with those cuts -- no host sort, no per-column loop
        from ..ops import stats_ops
        from . import quantile as Q
        yt = torch.as_tensor(np.asarray(y, np.float32), device=dev)
        wt = torch.as_tensor(np.asarray(w, np.float64), device=dev)

        def one_batch(batch):
            vals = upload_columns([md.table[c.name].numeric() for c in batch], dev)
            bounds, distinct = Q.column_cuts(vals, yt, wt, n_bins, method, binary, num_thr)
            if parity:
                bounds = [B.sketch_boundaries(md.table[c.name].numeric(), n_bins, parity) for c in batch]
            if total <= EXACT_DISTINCT_ROWS:
                distinct = exact_distinct(vals, num_thr)
            return bounds, distinct, stats_ops.column_stats(vals, yt, wt, bounds, binary, num_thr)

        batches = [numeric[b0: b0 + gpu_batch] for b0 in range(0, len(numeric), gpu_batch)]
        for batch, (bounds, distinct, res) in zip(batches, run_lanes(one_batch, batches, dev)):
            for c, bnd, (cpos, cneg, wpos, wneg, mom), dc in zip(batch, bounds, res, distinct):
                _finish_numeric(c, binary, bnd, cpos, cneg, wpos, wneg, mom, total, dc)
        return ccs
    for cc in numeric:
        vals = md.table[cc.name].numeric().astype(np.float64).copy()
        vals[vals > num_thr] = np.nan          # numericalValueThreshold -> invalid
        bounds = B.sketch_boundaries(md.table[cc.name].numeric(), n_bins, parity) if parity else \
            _numeric_bounds(vals, y, w, binary, method, n_bins)
        bidx = B.bin_index_numeric(vals, bounds)
        cpos, cneg, wpos, wneg = _hist(bidx, y, w, len(bounds) + 1, binary, dev)
        fin = vals[np.isfinite(vals)]
        _finish_numeric(cc, binary, bounds, cpos, cneg, wpos, wneg, _moments(vals, dev), total,
                        np.unique(fin).size)
    return ccs


def compute_psi(mc, ccs, md, unit_column: str, unit_stats_path: str | None = None):
    """Population stability per column across the units of ``psiColumnName`` (P/PSI.pig:19-46).

    Reference parity:
      * per (unit, column) counters = ``PopulationCounterUDF`` with ``NumericCounter`` /
        ``CategoryCounter`` (J/udf/stats/*Counter.java): one count per bin + a missing bin, the
        unit mean (sum of valid numeric values, or of the category's ``binPosRate`` for
        categoricals, over ALL the unit's records incl. missing; NaN when every record is
        missing), the missing rate and the record count;
      * the EXPECTED distribution comes from the ColumnConfig stats pass:
        ``(binCountNeg[i] + binCountPos[i]) / totalCount`` (``PSICalculatorUDF.exec`` :55-65),
        not from the PSI pass's own rows;
      * PSI = sum over units of sum_i (a_i - e_i) ln(a_i / e_i), accumulated with the UDF's
        exact loop -- its bin index only advances on the terms it adds (a zero actual or
        expected share, or an empty unit, skips the term WITHOUT advancing), reproduced as is;
      * unit statistics ``unit^mean^missingRate^count`` (Java ``Double.toString``), sorted as
        strings, joined by ``\u0001`` and written per column as ``columnNum|stats`` lines to
        ``tmp/columnconfig.unitstats`` (MapReducerStatsWorker.runPSI :624-651); like the
        reference, ColumnConfig gets ``psi`` only.
    Data parallel: the unit set is the union over ranks and the (unit, bin) counts + unit value
    sums of every column are all-reduced in one bucket (the PopulationCounter shuffle)."""
    from ..config.jsonio import java_double_str
    from ..parallel import dist
    if unit_column not in md.table:
        _log.warning("psiColumnName %s not in data", unit_column)
        return ccs
    units_s = md.table[unit_column].strings()
    units = sorted(set(units_s))
    if dist.info().world_size > 1:
        units = sorted(set().union(*dist.all_gather_objects(units)))
    U = len(units)
    uidx = {u: i for i, u in enumerate(units)}
    ucode = np.array([uidx[u] for u in units_s], dtype=np.int64) if len(units_s) else np.zeros(0, np.int64)
    from ..utils.device import default_device
    dev = default_device()
    if dev.type == "cuda":                     # K17 on the device: keyed_hist (scoring_kernels.hip)
        from ..ops.stats_ops import keyed_hist
        ucode_d = torch.as_tensor(ucode).to(dev)
    cols, counts = [], []
    for cc in ccs:
        if cc.is_target() or cc.is_meta() or cc.name not in md.table:
            continue
        col = md.table[cc.name]
        if cc.is_categorical():
            cats = cc.bin_category or []
            codes = col.values if col.kind == "str" else None
            if codes is None or not cats:
                continue
            bidx = B.category_index(codes, col.dictionary, cats)
            nb = len(cats) + 1
            rate = np.asarray(list(cc.bin_pos_rate or [0.0] * len(cats)) + [0.0], dtype=np.float64)
            contrib = rate[np.clip(bidx, 0, nb - 1)]
            contrib[bidx >= nb - 1] = 0.0
        else:
            bb = cc.bin_boundary
            if not bb:
                continue
            v = col.numeric()
            nb = len(bb) + 1
            if dev.type == "cuda":
                bidx = B.bin_index_torch(torch.as_tensor(np.asarray(v, np.float64)).to(dev),
                                         torch.as_tensor(np.asarray(bb, np.float64)).to(dev))
            else:
                bidx = B.bin_index_numeric(v, bb)
            contrib = np.where(np.isnan(v), 0.0, v)
        if dev.type == "cuda":                 # exact integer (unit, bin) counts on the device
            cnt = keyed_hist(ucode_d * nb + torch.as_tensor(bidx).to(dev), U * nb)[0][0].cpu().numpy()
        else:
            cnt = np.bincount(ucode * nb + bidx, minlength=U * nb).astype(np.float64)
        # unit value sums stay an in-order fp64 host sum: they are printed at full double
        # precision in the unit stats (Double.toString), so no fixed-point rounding here
        vsum = np.bincount(ucode, weights=contrib, minlength=U).astype(np.float64)
        cols.append((cc, nb))
        counts.append(np.concatenate([cnt, vsum]))
    if counts and dist.info().world_size > 1:
        flat = dist.all_reduce_np(np.concatenate(counts))
        off = 0
        for i, c in enumerate(counts):
            counts[i] = flat[off:off + c.size]
            off += c.size
    lines = []
    for (cc, nb), buf in zip(cols, counts):
        per_unit = buf[:U * nb].reshape(U, nb)
        vsum = buf[U * nb:]
        neg = list(cc.bin_count_neg or [])
        pos = list(cc.bin_count_pos or [])
        total_cnt = float(cc.stat("totalCount", 0) or 0)
        expected = [0.0 if total_cnt == 0 else (float(neg[i]) + float(pos[i])) / total_cnt
                    for i in range(min(len(neg), len(pos)))]
        psi = 0.0
        unit_stats = []
        for ui, u in enumerate(units):
            sub = per_unit[ui]
            total = float(sub.sum())
            i = 0
            for sv in sub:                       # PSICalculatorUDF.exec :75-95, index quirk kept
                if total == 0 or i >= len(expected) or expected[i] == 0:
                    continue
                log_num = (sv / total) / expected[i]
                if log_num <= 0:
                    continue
                psi += (sv / total - expected[i]) * math.log(log_num)
                i += 1
            miss = float(sub[nb - 1])
            mean = float("nan") if (total == 0 or total == miss) else float(vsum[ui]) / total
            mrate = miss / total if total != 0 else 0.0
            unit_stats.append(f"{u}^{java_double_str(mean)}^{java_double_str(mrate)}^{int(total)}")
        unit_stats.sort()
        cc.stats["psi"] = psi
        lines.append(f"{cc.num}|" + "\u0001".join(unit_stats))
    if unit_stats_path and dist.info().rank == 0:
        os.makedirs(os.path.dirname(unit_stats_path) or ".", exist_ok=True)
        with open(unit_stats_path, "w", encoding="utf-8") as f:
            f.write("".join(line + "\n" for line in lines))
    return ccs


CORR_CHUNK = 65536      # rows per int8-digit GEMM launch (int32 bound: 7 pairs x 64^2 x 2^16 < 2^31)


def corr_job_list(S: int) -> list:
    """The K15 GEMM jobs for S digits: (name, [(A plane, B plane), ...], A scale row, B scale row,
    digit weight exponent, symmetric).  Planes: 0 mask, 1..S digits of u / 2^ex, S+1..2S digits of
    u^2 / 2^ey; scale rows 0 (ones), 1 (2^ex), 2 (2^ey).  A job's pairs share the weight
    2^-wexp, so they sum in one int32 accumulator: sxy_d is the digit diagonal s + t = d."""
    X, Y = (lambda s: 1 + s), (lambda s: 1 + S + s)
    jobs = [("n", [(0, 0)], 0, 0, 0, True)]
    jobs += [(f"sx{s}", [(X(s), 0)], 1, 0, 7 * (s + 1), False) for s in range(S)]
    jobs += [(f"sxx{s}", [(Y(s), 0)], 2, 0, 7 * (s + 1), False) for s in range(S)]
    jobs += [(f"sxy{d}", [(X(s), X(d - s)) for s in range(d + 1)], 1, 1, 7 * (d + 2), True) for d in range(S)]
    return jobs


class CorrAccumulator:
    """Pairwise-complete Pearson sums (H3, FastCorrelationMapper J/core/correlation/
    FastCorrelationMapper.java:171-278: rows where either value is missing are skipped per pair),
    accumulated over row chunks on the device, of the shifted values u = x - c (``shift`` c per
    column -- e.g. the stats step's means; Pearson is shift invariant and the shift keeps the
    final ``sxy - sx*sy/n`` free of cancellation), zero-filled where missing, and the mask M:
        n = M'M,  sx = U'M (sum of u_i where j valid; sy = sx'),  sxx = (U*U)'M (syy = sxx'),
        sxy = U'U
    so the table never has to sit on the device (or in fp64 on the host) whole.

    ``method="i8"`` (default on the GPU, K15): every sum is an EXACT integer GEMM on the int8 MFMA
    (ops/csrc/corr_kernels.hip digit planes + gemm_kernels.hip corr_i8_kernel): u / 2^ex and
    u^2 / 2^ey are split into ``slices`` S balanced base-128 digits (S x 7 bits of each value,
    relative to its column's chunk maximum), products of digit planes are summed in int32 and
    flushed per 64K-row chunk into fp64 with their exact power-of-two weights; the symmetric n and
    sxy run their upper tiles only.  ~2S + S(S+1)/4 int8 GEMMs at 2x the bf16 MFMA rate replace
    four fp64 GEMMs at 1/32 of it.  ``method="fp64"``: four torch fp64 ``addmm`` per chunk (CPU,
    and the oracle of the GPU tests)."""

    def __init__(self, n_cols: int, device=None, shift=None, method: str | None = None, slices: int | None = None):
        from ..config import environment
        self.F = int(n_cols)
        self.dev = torch.device(device) if device is not None else \
            (torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
        self.shift = None if shift is None else \
            torch.as_tensor(np.asarray(shift, dtype=np.float64), device=self.dev).reshape(self.F).contiguous()
        method = method or environment.get("shifu.stats.corr.method", "auto")
        if method == "auto":
            method = "i8" if self.dev.type == "cuda" and self.F > 0 else "fp64"
        if method not in ("i8", "fp64"):
            raise ValueError(f"unknown correlation method {method!r}")
        if method == "i8" and self.dev.type != "cuda":
            raise ValueError("correlation method i8 needs a GPU")
        self.method = method
        if method == "fp64":
            self.sums = torch.zeros(4, self.F, self.F, dtype=torch.float64, device=self.dev)
            return
        from ..ops import _native as nat
        nat.require_gpu_native()
        self.S = int(slices or environment.get_int("shifu.stats.corr.slices", 6))
        if not 4 <= self.S <= 7:
            raise ValueError("shifu.stats.corr.slices must be in 4..7")
        self._build_jobs(nat)
        self.J = torch.zeros(len(self.job_names), self.F, self.F, dtype=torch.float64, device=self.dev)
        self._planes = None
        self._scale = torch.empty(3, self.F, dtype=torch.float64, device=self.dev)
        self._maxbits = torch.empty(self.F, dtype=torch.int64, device=self.dev)

    # -- i8 path -----------------------------------------------------------------------------
    def _build_jobs(self, nat):
        """Job table (gemm_kernels.hip CorrJob) and the (job, tile m, tile n) launch order."""
        jobs = corr_job_list(self.S)
        self.job_names = [j[0] for j in jobs]
        self.job_sym = [j[5] for j in jobs]
        rec = np.zeros((len(jobs), 4 + 14), dtype=np.int32)
        for k, (_, pairs, ka, kb, wexp, _) in enumerate(jobs):
            rec[k, :4] = (len(pairs), ka, kb, wexp)
            for q, (a, b) in enumerate(pairs):
                rec[k, 4 + q], rec[k, 11 + q] = a, b
        assert rec.shape[1] * 4 == nat.hip().shifu_corr_job_bytes()
        self._jobs = torch.from_numpy(rec).to(self.dev)
        T = -(-self.F // 256)
        items = []
        for k, (_, pairs, _, _, _, sym) in enumerate(jobs):
            for tm in range(T):
                for tn in range(tm if sym else 0, T):
                    items.append((len(pairs), k, tm, tn))
        # heaviest first (longest K), then job / tile order so consecutive blocks share operand rows
        items.sort(key=lambda t: (-t[0], t[1], t[2], t[3]))
        self._items = torch.tensor([(k, tm, tn, 0) for _, k, tm, tn in items], dtype=torch.int32, device=self.dev)
        self.n_items = len(items)

    def _update_i8(self, X: torch.Tensor) -> None:
        from ..ops import _native as nat
        n, F = X.shape
        if n == 0:
            return
        kpad = max(128, 1 << (n - 1).bit_length())
        P = 1 + 2 * self.S
        if self._planes is None or self._planes.numel() < P * F * kpad:
            self._planes = torch.empty(P * F * kpad, dtype=torch.int8, device=self.dev)
        st = nat.stream_of(X)
        nat.call_hip("shifu_corr_planes", X, X.stride(0), n, F, self.shift, self.S, kpad, self._planes, F * kpad,
                     self._scale, self._maxbits, st)
        nat.call_hip("shifu_corr_gemm", self._planes, F * kpad, kpad, F, self._jobs, self._items, self.n_items,
                     self._scale, self.J, F * F, st)

    def _fold(self) -> torch.Tensor:
        """[4, F, F] fp64 sums (n, sx, sxx, sxy) from the per-job buffers."""
        T = torch.arange(self.F, device=self.dev) // 256
        lower = T[:, None] > T[None, :]

        def mirror(U):
            return torch.where(lower, U.t(), U)
        J, names = self.J, self.job_names
        pick = lambda pre: [J[k] for k, nm in enumerate(names) if nm.rstrip("0123456789") == pre]
        n = mirror(J[names.index("n")])
        sx = torch.stack(pick("sx")).sum(0)
        sxx = torch.stack(pick("sxx")).sum(0)
        sxy = mirror(torch.stack(pick("sxy")).sum(0))
        return torch.stack([n, sx, sxx, sxy])

    # -- common ------------------------------------------------------------------------------
    def update(self, X) -> None:
        if not torch.is_tensor(X):
            X = torch.from_numpy(np.ascontiguousarray(X, dtype=np.float64))
        if self.method == "i8":
            for r0 in range(0, X.shape[0], CORR_CHUNK):
                xs = X[r0:r0 + CORR_CHUNK].to(self.dev, torch.float64, non_blocking=True)
                self._update_i8(xs if xs.stride(1) == 1 else xs.contiguous())
            return
        X = X.to(self.dev, torch.float64)
        M = torch.isfinite(X)
        U = torch.where(M, X - self.shift if self.shift is not None else X, torch.zeros((), dtype=X.dtype, device=X.device))
        M = M.to(torch.float64)
        self.sums[0].addmm_(M.t(), M)
        self.sums[1].addmm_(U.t(), M)
        self.sums[2].addmm_((U * U).t(), M)
        self.sums[3].addmm_(U.t(), U)

    def raw_sums(self) -> torch.Tensor:
        """This rank's [4, F, F] fp64 (n, sx, sxx, sxy) of the shifted values."""
        return self._fold() if self.method == "i8" else self.sums

    @staticmethod
    def _corr_rows(n, sx, sy, sxx, syy, sxy):
        num = sxy - sx * sy / n.clamp(min=1)
        den = torch.sqrt((sxx - sx * sx / n.clamp(min=1)).clamp(min=0) * (syy - sy * sy / n.clamp(min=1)).clamp(min=0))
        return torch.where(den > 0, num / den, torch.zeros_like(num))

    def finalize(self, dst: int = 0):
        """Global correlation matrix on rank ``dst`` (numpy), None elsewhere.  Data parallel: the
        six F x F sums (the four + the transposes that supply sy/syy), laid out row-major as
        [F][6][F] so that a rank's row block is one contiguous slab, are REDUCE-SCATTERED -- each
        rank gets 1/R of the bytes an all-reduce would leave on every rank --, every rank computes
        its block of correlation rows, and the blocks are gathered to ``dst``."""
        from ..parallel import dist
        F = self.F
        n, sx, sxx, sxy = self.raw_sums().unbind(0)
        six = torch.stack([n, sx, sx.t(), sxx, sxx.t(), sxy], dim=1)      # [F, 6, F]
        if self.method == "i8":
            self.J = None                                                  # free the job sums
        blk = dist.reduce_scatter_rows(six, dim0=True)                     # [b - a, 6, F]
        a, b = dist.row_block(F)
        rows = self._corr_rows(*blk.unbind(1))
        idx = torch.arange(a, b, device=rows.device)
        rows[idx - a, idx] = 1.0
        full = dist.gather_rows_to(rows, F, dst)
        return None if full is None else full.cpu().numpy()


def pearson_correlation(mats, device=None, chunk_rows: int = 1 << 18, dst: int = 0, method: str | None = None):
    """Pairwise-complete Pearson of the columns of ``mats`` ([N, F] array, NaN = missing, or an
    iterable of such row chunks) -> [F, F] on rank ``dst`` (every rank when not distributed)."""
    from ..parallel import dist
    acc = None
    chunks = [mats] if isinstance(mats, np.ndarray) or torch.is_tensor(mats) else mats
    for X in chunks:
        X = np.asarray(X) if not torch.is_tensor(X) else X
        if acc is None:
            shift = None
            if not dist._active() and len(X):       # single process: center on the first chunk's means
                Xt = torch.as_tensor(X[:CORR_CHUNK], dtype=torch.float64)
                shift = torch.nan_to_num(torch.nanmean(torch.where(torch.isfinite(Xt), Xt, torch.nan), 0)).cpu().numpy()
            acc = CorrAccumulator(X.shape[1], device, shift=shift, method=method)
        for r0 in range(0, X.shape[0], chunk_rows):
            acc.update(X[r0:r0 + chunk_rows])
    if acc is None:
        return np.zeros((0, 0))
    return acc.finalize(dst)


