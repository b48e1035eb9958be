"""Streamed ``shifu stats``: every column's bins and statistics from a stream of row chunks, with
host memory bounded by one chunk (out-of-core data sets, and the per-rank byte-range path of a
data-parallel run).

The reference runs stats as MapReduce jobs over input splits - mappers build per-column streaming
histograms / counts, reducers merge them (``UpdateBinningInfoMapper``
J/core/binning/UpdateBinningInfoMapper.java:349-599, ``UpdateBinningInfoReducer`` :125-433,
``MapReducerStatsWorker`` J/core/processor/stats/MapReducerStatsWorker.java:105-176).  Here the
chunks come from :func:`data.stream.iter_model_data` and every pass is mergeable:

1. A  (one stream pass) K4 ``qprep`` per numeric column batch; categorical per-category
      histograms in first-appearance order; row totals;
2. B  K4 ``qhist`` once per refinement level (usually one), C ``qgather`` when a cut target sits
      in a multi-valued bucket -- the exact cuts of ``algos/quantile.py``;
3. D  K1+K2 (``column_stats`` kernel) bin histograms + moments with those cuts.

Each numeric batch is uploaded to the device once per chunk; when the whole stream's numeric
columns fit the device budget (``SHIFU_STATS_CACHE_GB``, default half the free HBM) the uploaded
chunks are kept resident and the data is parsed exactly once.  ``reduce`` / ``allgather`` /
``gather_objects`` merge the partials across ranks (identity for one process).

Results equal :func:`algos.stats.compute_column_stats` over the same rows (cuts, histograms,
moments up to fp64 summation order, categories) and ``distinctCount`` up to one exception: on
data sets of at most ``stats.EXACT_DISTINCT_ROWS`` rows the in-memory pass counts exactly, the
stream counts exactly only columns with at most ``DISTINCT_SET_CAP`` distinct values (bounded
memory) and reports the K4 bucket count / HyperLogLog estimate for the others -- as both paths do
on larger data sets (the reference reports HyperLogLogPlus estimates for every column).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ..utils.trace import trace_range
from ..utils.log import get_logger
from . import binning as B
from . import quantile as Q
from . import stats as S

_log = get_logger("algos.stats_stream")

DISTINCT_SET_CAP = 1 << 16


class _Batch:
    def __init__(self, cols, eng):
        self.cols = cols                  # ColumnConfig list
        self.eng = eng
        self.distinct_sets = [None] * len(cols)   # exact value sets while rows <= EXACT_DISTINCT_ROWS
        self.rows_seen = 0
        self.overflow = [False] * len(cols)
        self.bounds = None
        self.distinct = None
        self.hist = None
        self.mom = None


def _cache_budget(dev) -> int:
    env = os.environ.get("SHIFU_STATS_CACHE_GB")
    if env is not None:
        return int(float(env) * (1 << 30))
    if dev.type == "cuda":
        from ..utils.device import free_hbm
        free = free_hbm(dev)
        # everything but ~40 GiB of working room (parse pipeline blocks, per-batch kernels): at
        # 20M x 1600 the whole 256-GB rank share stays resident and the later passes stop
        # re-parsing an uncached tail (stats 17.5-19.4 -> 13.0 s; 70 % of free HBM cached 214 GB)
        return int(max(0.5 * free, min(0.9 * free, free - (40 << 30))))
    return 0


def compute_column_stats_streamed(mc, ccs, chunks_fn, device=None, columns=None, batch: int = 64,
                                  reduce=None, allgather=None, gather_objects=None):
    """``chunks_fn(resume=None, with_keys=False)`` -> a fresh iterator of ModelData chunks (this
    rank's rows; ``with_keys``: (key, chunk) pairs, ``resume``: start at a key's block).  Fills the same
    ColumnConfig fields as ``compute_column_stats``; returns the merged row count."""
    from ..utils.device import is_gpu_available
    dev = torch.device(device or ("cuda" if is_gpu_available() else "cpu"))
    binary = mc.is_binary()
    method = mc.binning_method
    n_bins = int(mc.stats.get("maxNumBin", 10))
    cate_max = int(mc.stats.get("cateMaxNumBin", 0) or 0)
    num_thr = float(mc.stats.get("numericalValueThreshold", 1.7976931348623157e308))
    sm = Q.sel_mode_for(method, binary)
    weighted = method.startswith("Weight")
    interval = method in ("EqualInterval", "WeightEqualInterval")
    numeric, categorical = [], []
    for cc in ccs:
        if columns is not None and cc.name not in columns:
            continue
        if cc.is_target() or cc.is_meta():
            continue
        (categorical if cc.is_categorical() else numeric).append(cc)
    batches = [_Batch(numeric[b0:b0 + batch],
                      Q.QuantileEngine(len(numeric[b0:b0 + batch]), n_bins, sm, weighted, interval, num_thr, dev,
                                       reduce, allgather))
               for b0 in range(0, len(numeric), batch)]
    budget = _cache_budget(dev)
    cache, cached_bytes, cache_ok = [], 0, True

    def upload(md, bt):
        from ..data.gpu_parse import device_rows
        if dev.type == "cuda":          # GPU-parsed columns (K0): already in HBM
            v = device_rows([md.table.columns.get(c.name) for c in bt.cols], dev)
            if v is not None:
                return v
        vals = S.upload_columns([md.table[c.name].numeric() if c.name in md.table
                                 else np.full(md.n, np.nan) for c in bt.cols], dev)
        return vals

    def yw(md):
        return (torch.as_tensor(np.asarray(md.y, np.float32), device=dev),
                torch.as_tensor(np.asarray(md.w, np.float64), device=dev))

    resume = [None]          # key of the first chunk that did not fit the device cache

    def stream():
        """(y, w, [vals per batch]) per chunk: the chunks that fit the HBM budget come from the
        device cache, the rest is re-read and re-parsed from the first uncached block on."""
        yield from cache
        if resume[0] is None:
            return
        for md in chunks_fn(resume=resume[0]):
            y, w = yw(md)
            yield y, w, [upload(md, bt) for bt in batches]

    # ---- pass A (+ categorical histograms, totals, exact distinct sets while small) ----------
    total, unselected = 0, 0
    cat_state = {cc.name: ({}, []) for cc in categorical}     # name -> (cat -> idx, [counts rows])
    cat_missing = {cc.name: np.zeros(4) for cc in categorical}
    first = True
    for key, md in chunks_fn(with_keys=True):
        total += md.n
        y, w = yw(md)
        if sm:
            unselected += int((~Q._selmask(y, sm, md.n, y.device)).sum())
        vals_all = []
        for bi, bt in enumerate(batches):
            with trace_range(f"stats.passA.batch{bi}"):
                v = upload(md, bt)
                bt.eng.pass_a(v, y, w)
                _track_distinct(bt, v, num_thr)
            vals_all.append(v)
        for cc in categorical:
            _cat_update(cc, md, binary, cat_state[cc.name], cat_missing[cc.name])
        if cache_ok:
            nbytes = sum(v.numel() * 8 for v in vals_all) + md.n * 12
            if cached_bytes + nbytes <= budget:
                cache.append((y, w, vals_all))
                cached_bytes += nbytes
            else:                  # keep the cached prefix; later passes resume at this block
                cache_ok = False
                resume[0] = key
        del vals_all
        first = False
    if first:
        _log.warning("stats: empty data stream")
    t = torch.tensor([float(total), float(unselected)], dtype=torch.float64, device=dev if reduce else "cpu")
    if reduce is not None:
        reduce(t, "sum")
    total, unselected = int(t[0].item()), int(t[1].item())
    _log.info("stats stream: %d rows, %d numeric batches, device cache %d chunks (%.1f GB)%s", total,
              len(batches), len(cache), cached_bytes / 1e9,
              "" if resume[0] is None else ", later passes re-parse from block %s" % (resume[0][:2],))
    for bt in batches:
        bt.eng.finish_a()

    # ---- passes B (one per refinement level) and C --------------------------------------------
    with trace_range("stats.cut_passes"):
        _run_cut_passes([bt.eng for bt in batches], stream)
    for bt in batches:
        bt.bounds, bt.distinct = bt.eng.finish()
    # class-restricted cuts that degenerate are redone over all rows, unweighted (reference rule)
    if sm and unselected > 0:
        redo = [(bt, [k for k, b in enumerate(bt.bounds) if len(b) <= 1]) for bt in batches]
        redo = [(bt, ks) for bt, ks in redo if ks]
        if redo:
            engs = [Q.QuantileEngine(len(ks), n_bins, 0, False, False, num_thr, dev, reduce, allgather)
                    for bt, ks in redo]

            def sub_stream():
                for y, w, vl in stream():
                    yield y, w, [vl[batches.index(bt)][ks] for bt, ks in redo]
            for y, w, vl in sub_stream():
                for e, v in zip(engs, vl):
                    e.pass_a(v, y, w)
            for e in engs:
                e.finish_a()
            _run_cut_passes(engs, sub_stream)
            for e, (bt, ks) in zip(engs, redo):
                b2, _ = e.finish()
                for k, b in zip(ks, b2):
                    bt.bounds[k] = b

    # ---- pass D: bin histograms + moments ------------------------------------------------------
    bcache = {}
    acc = [None] * len(batches)      # GPU: per batch [counts, weight sums, moments] arrays
    for y, w, vl in stream():
        if dev.type == "cuda":       # every batch of the chunk: one weight scan, two D2H copies
            from ..ops import stats_ops
            multi = stats_ops.column_stats_multi(vl, y, w, [bt.bounds for bt in batches], binary, num_thr, bcache)
            for i, (cnt, wsum, mom, boff) in enumerate(multi):
                acc[i] = _acc_chunk(acc[i], cnt, wsum, mom, boff)
            continue
        for bt, v in zip(batches, vl):
            res = S.batch_histograms(v, y, w, bt.bounds, binary, num_thr)
            if bt.hist is None:
                bt.hist = [[r[0].astype(np.int64), r[1].astype(np.int64), r[2].astype(np.float64),
                            r[3].astype(np.float64)] for r in res]
                bt.mom = [list(r[4]) for r in res]
            else:
                for h, m, r in zip(bt.hist, bt.mom, res):
                    for i in range(4):
                        h[i] = h[i] + r[i]
                    _merge_moments(m, r[4])
    for bt, a in zip(batches, acc):
        if a is not None:
            bt.hist, bt.mom = _acc_lists(a)
    for bt in batches:
        if bt.hist is None:     # no rows on this rank: zero partials shaped by the (global) cuts, so
            # every rank sends same-sized buffers to the merging collectives
            bt.hist = [[np.zeros(len(b) + 1, np.int64), np.zeros(len(b) + 1, np.int64),
                        np.zeros(len(b) + 1, np.float64), np.zeros(len(b) + 1, np.float64)] for b in bt.bounds]
            bt.mom = [[0, 0.0, 0.0, 0.0, 0.0, float("nan"), float("nan")] for _ in bt.bounds]
        _finish_batch(bt, binary, total, reduce, gather_objects, dev, n_bins)
    for cc in categorical:
        _finish_cat(cc, cat_state[cc.name], cat_missing[cc.name], binary, total, cate_max, gather_objects,
                    reduce, dev)
    return total


def _run_cut_passes(engs, stream):
    state = {id(e): "B" for e in engs}
    while any(s == "B" for s in state.values()):
        for y, w, vl in stream():
            for e, v in zip(engs, vl):
                if state[id(e)] == "B":
                    e.pass_b(v, y, w)
        for e in engs:
            if state[id(e)] == "B":
                state[id(e)] = e.finish_b()
    if any(s == "C" for s in state.values()):
        for y, w, vl in stream():
            for e, v in zip(engs, vl):
                if state[id(e)] == "C":
                    e.pass_c(v, y, w)


def _acc_chunk(a, cnt, wsum, mom, boff):
    """Vectorized form of the per-column merge below for one chunk's batch arrays (the same
    elementwise float adds in chunk order, so the totals are bit-identical)."""
    if a is None:
        return [cnt.copy(), wsum.copy(), mom.copy(), boff]
    a[0] += cnt
    a[1] += wsum
    m = a[2]
    take = mom[:, 0] != 0
    new = take & (m[:, 0] == 0)
    upd = take & ~new
    m[new] = mom[new]
    m[upd, :5] += mom[upd, :5]
    m[upd, 5] = np.minimum(m[upd, 5], mom[upd, 5])
    m[upd, 6] = np.maximum(m[upd, 6], mom[upd, 6])
    return a


def _acc_lists(a):
    """Accumulated batch arrays -> the per-column hist / moment lists of the host path."""
    cnt, wsum, mom, boff = a
    hist, moms = [], []
    for f in range(cnt.shape[0]):
        k = int(boff[f + 1] - boff[f]) + 1
        hist.append([cnt[f, :k, 0].copy(), cnt[f, :k, 1].copy(), wsum[f, :k, 0].copy(), wsum[f, :k, 1].copy()])
        moms.append([int(mom[f, 0])] + [float(x) for x in mom[f, 1:]])
    return hist, moms


def _merge_moments(m, r):
    if r[0] == 0:
        return
    if m[0] == 0:
        m[:] = list(r)
        return
    m[0] += r[0]
    for i in range(1, 5):
        m[i] += r[i]
    m[5] = min(m[5], r[5])
    m[6] = max(m[6], r[6])


def _track_distinct(bt, vals, num_thr):
    """Exact value sets while the data set is small enough for the in-memory rule
    (<= stats.EXACT_DISTINCT_ROWS rows) and the set itself stays <= DISTINCT_SET_CAP values (so the
    sets never outgrow a few chunks); a column that overflows falls back to the K4 estimate.
    GPU: batched over the batch's columns -- the current sets ([C, K] sorted, +inf padded) and the chunk
    ([C, n], non-finite -> +inf) are sorted together per row, duplicates become +inf and a second
    sort compacts the new sets -- two sorts per chunk and batch instead of a unique per column."""
    bt.rows_seen += vals.shape[1]
    C = vals.shape[0]
    if bt.rows_seen > S.EXACT_DISTINCT_ROWS:
        bt.distinct_sets = [None] * len(bt.cols)
        bt.overflow = [True] * len(bt.cols)
        bt._dset = None
        return
    if all(bt.overflow):
        return
    if vals.device.type != "cuda":                 # host: per-column sets (no padded [C, K] copies)
        for k in range(C):
            if bt.overflow[k]:
                continue
            v = vals[k]
            v = torch.where(v > num_thr, torch.full_like(v, float("nan")), v) + 0.0
            u = torch.unique(v[torch.isfinite(v)])
            cur = bt.distinct_sets[k]
            u = u if cur is None else torch.unique(torch.cat([cur, u]))
            if u.numel() > DISTINCT_SET_CAP:
                bt.overflow[k] = True
                u = None
            bt.distinct_sets[k] = u
        return
    inf = float("inf")
    v = torch.where(vals > num_thr, torch.full_like(vals, float("nan")), vals) + 0.0
    v = torch.where(torch.isfinite(v), v, torch.full_like(v, inf))
    ovf = torch.tensor(bt.overflow, dtype=torch.bool, device=v.device)
    v = torch.where(ovf[:, None], torch.full_like(v, inf), v)
    cur = getattr(bt, "_dset", None)
    comb = v if cur is None else torch.cat([cur, v], 1)
    srt, _ = torch.sort(comb, dim=1)
    dup = torch.zeros_like(srt, dtype=torch.bool)
    dup[:, 1:] = srt[:, 1:] == srt[:, :-1]
    srt = torch.where(dup, torch.full_like(srt, inf), srt)
    srt, _ = torch.sort(srt, dim=1)
    cnt = torch.isfinite(srt).sum(1)
    new_ovf = (cnt > DISTINCT_SET_CAP).cpu().numpy()
    cnt_h = cnt.cpu().numpy()
    for k in range(C):
        if new_ovf[k]:
            bt.overflow[k] = True
    keep = [int(cnt_h[k]) for k in range(C) if not bt.overflow[k]]
    width = max(keep) if keep else 0
    bt._dset = srt[:, :max(width, 1)].contiguous()
    bt._dcnt = cnt_h
    bt.distinct_sets = [None if bt.overflow[k] else bt._dset[k, : int(cnt_h[k])] for k in range(C)]


def _finish_batch(bt, binary, total, reduce, gather_objects, dev, n_bins):
    # merge histograms / moments over ranks
    if reduce is not None:
        flat = np.concatenate([np.concatenate([h[0], h[1], h[2], h[3]]).astype(np.float64) for h in bt.hist])
        t = torch.as_tensor(flat, device=dev)
        reduce(t, "sum")
        flat = t.cpu().numpy()
        off = 0
        for h in bt.hist:
            for i in range(4):
                n = h[i].size
                h[i] = flat[off:off + n].astype(np.int64 if i < 2 else np.float64)
                off += n
        sums = torch.tensor([m[:5] for m in bt.mom], dtype=torch.float64, device=dev)
        mn = torch.tensor([m[5] if m[0] else np.inf for m in bt.mom], dtype=torch.float64, device=dev)
        mx = torch.tensor([m[6] if m[0] else -np.inf for m in bt.mom], dtype=torch.float64, device=dev)
        reduce(sums, "sum")
        reduce(mn, "min")
        reduce(mx, "max")
        sums, mn, mx = sums.cpu().numpy(), mn.cpu().numpy(), mx.cpu().numpy()
        bt.mom = [[int(s[0]), s[1], s[2], s[3], s[4], a if s[0] else float("nan"), b if s[0] else float("nan")]
                  for s, a, b in zip(sums, mn, mx)]
    # exact distinct counts while every rank's set stayed small (small data sets: the in-memory rule)
    if total <= S.EXACT_DISTINCT_ROWS:
        mine = [None if o else (np.zeros(0) if s is None else s.cpu().numpy())
                for o, s in zip(bt.overflow, bt.distinct_sets)]
        parts = gather_objects(mine) if gather_objects is not None else [mine]
        for k in range(len(bt.cols)):
            if all(p[k] is not None for p in parts):
                bt.distinct[k] = int(np.unique(np.concatenate([p[k] for p in parts])).size)
    for k, cc in enumerate(bt.cols):
        h, m = bt.hist[k], bt.mom[k]
        mom = (int(m[0]), float(m[1]), float(m[2]), float(m[3]), float(m[4]), float(m[5]), float(m[6]))
        if mom[0] == 0:
            mom = (0, 0.0, 0.0, 0.0, 0.0, float("nan"), float("nan"))
        S._finish_numeric(cc, binary, bt.bounds[k], h[0], h[1], h[2], h[3], mom, total, bt.distinct[k])


def _cat_update(cc, md, binary, state, missing_acc):
    """Accumulate per-category (cpos, cneg, wpos, wneg) in global first-appearance order."""
    index, rows = state
    if cc.name not in md.table:
        return
    col = md.table[cc.name]
    if col.kind == "str":
        codes, dictionary = col.values, col.dictionary
    else:
        s = col.strings()
        uniq = {}
        codes = np.array([uniq.setdefault(v, len(uniq)) if v != "" else -1 for v in s], dtype=np.int32)
        dictionary = list(uniq.keys())
    y = np.asarray(md.y)
    w = np.asarray(md.w, np.float64)
    nd = len(dictionary)
    # one counted and one weighted bincount over (category, positive) keys: no masked copies
    key = np.where(codes >= 0, codes, nd).astype(np.intp) * 2
    if binary:
        key += (y > 0.5)
    else:
        key += 1
    c = np.bincount(key, minlength=2 * (nd + 1)).reshape(nd + 1, 2)
    ws = np.bincount(key, weights=w, minlength=2 * (nd + 1)).reshape(nd + 1, 2)
    cp, cn, wp, wn = c[:, 1], c[:, 0], ws[:, 1], ws[:, 0]
    present = np.flatnonzero(c[:nd].sum(1) > 0)
    for d in present:
        name = dictionary[d]
        g = index.get(name)
        if g is None:
            g = index[name] = len(rows)
            rows.append(np.zeros(4))
        rows[g] += (cp[d], cn[d], wp[d], wn[d])
    missing_acc += (cp[nd], cn[nd], wp[nd], wn[nd])


def _finish_cat(cc, state, missing_acc, binary, total, cate_max, gather_objects, reduce, dev):
    index, rows = state
    names = list(index.keys())
    mat = np.array(rows) if rows else np.zeros((0, 4))
    if gather_objects is not None:        # rank order = row order: first appearance over ranks
        parts = gather_objects((names, mat, missing_acc))
        gidx, grows = {}, []
        miss = np.zeros(4)
        for nm, mt, ms in parts:
            miss += ms
            for k, n in enumerate(nm):
                g = gidx.get(n)
                if g is None:
                    g = gidx[n] = len(grows)
                    grows.append(np.zeros(4))
                grows[g] += mt[k]
        names, mat, missing_acc = list(gidx.keys()), (np.array(grows) if grows else np.zeros((0, 4))), miss
    cats = names[:10000]
    extra = mat[10000:].sum(0) if len(names) > 10000 else np.zeros(4)
    body = mat[:10000]
    last = missing_acc + extra
    cpos = np.append(body[:, 0], last[0]).astype(np.int64)
    cneg = np.append(body[:, 1], last[1]).astype(np.int64)
    wpos = np.append(body[:, 2], last[2])
    wneg = np.append(body[:, 3], last[3])
    if not binary:
        cpos, cneg = cpos + cneg, np.zeros_like(cneg)
        wpos, wneg = wpos + wneg, np.zeros_like(wneg)
    S.finish_categorical(cc, cats, cpos, cneg, wpos, wneg, total, binary, cate_max, len(names))
