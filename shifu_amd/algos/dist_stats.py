"""Data-parallel ``shifu stats`` over row shards (F7 / G3): every rank holds a contiguous row
range, and the per-column partials are merged with collectives instead of the reference's
MapReduce shuffle (``UpdateBinningInfoMapper`` -> ``UpdateBinningInfoReducer``,
J/core/binning/UpdateBinningInfoMapper.java:349-599, UpdateBinningInfoReducer.java:125-433).

The result is the single-process result (``algos.stats.compute_column_stats``), not an
approximation of it, with ONE exception (the distinct count of high-cardinality columns, last
bullet):

* numeric bin boundaries are the EXACT equal-population cuts over all ranks: the single-process
  rule (first distinct value whose cumulative count reaches j * total / bins, cut halfway to the
  next distinct value) is evaluated by a 64-step bisection in the order-preserving integer image of
  the float64 values - each step one all_reduce(SUM) of [columns x bins] counts from a
  ``searchsorted`` over each rank's sorted shard - then one all_reduce(MIN) finds the next distinct
  value.  Columns with at most ``bins`` distinct values gather their (tiny) value sets;
* categories keep the global first-appearance order (rank order = row order), gathered once;
* histograms (count/weight x pos/neg) and moments are all_reduce(SUM); min/max all_reduce(MIN/MAX);
* distinct counts: exact when the per-rank distinct sets are small enough to gather
  (<= ``DISTINCT_GATHER_CAP`` values each), otherwise a HyperLogLog (p = 14) merged with
  all_reduce(MAX) of its registers.  So for a column with more than ``DISTINCT_GATHER_CAP``
  distinct values on some rank, ``distinctCount`` is an estimate (relative error ~0.8 %) and can
  differ from the single-process exact count; the reference itself reports HyperLogLogPlus(8)
  estimates for every column.
"""
from __future__ import annotations

import numpy as np
import torch

from ..parallel import dist
from ..utils.log import get_logger
from . import binning as B
from . import stats as S

_log = get_logger("algos.dist_stats")

DISTINCT_GATHER_CAP = 1 << 16
HLL_P = 14


def _dev():
    return dist.coll_device()


def _allreduce(t: torch.Tensor, op="sum") -> torch.Tensor:
    d = _dev()
    x = t.to(d)
    dist.all_reduce_(x, op)
    return x.to(t.device)


def _gather_objects(obj):
    return dist.all_gather_objects(obj)


# ---- order-preserving float64 <-> int64 keys ----------------------------------------------------
_MAG = 0x7FFFFFFFFFFFFFFF


def _key(x: torch.Tensor) -> torch.Tensor:
    b = x.contiguous().view(torch.int64)
    return torch.where(b < 0, b ^ _MAG, b)


def _unkey(k: torch.Tensor) -> torch.Tensor:
    return torch.where(k < 0, k ^ _MAG, k).view(torch.float64)


def exact_equal_population(cols_vals, cols_w, n_bins: int, dev) -> list:
    """cols_vals: per column a 1-D float64 tensor of this rank's finite selected values;
    cols_w: per column None or the matching weights.  Returns the global boundary list per
    column, identical to ``binning.equal_population_boundaries`` over the union of all ranks."""
    C = len(cols_vals)
    out = [None] * C
    # sorted shards (+ weight prefix sums) padded into [C, L] with +inf
    L = max([int(v.numel()) for v in cols_vals] + [1])
    vs = torch.full((C, L), float("inf"), dtype=torch.float64, device=dev)
    cw = torch.zeros((C, L + 1), dtype=torch.float64, device=dev)
    weighted = any(w is not None for w in cols_w)
    local_n = torch.zeros(C, dtype=torch.float64, device=dev)
    for c, (v, w) in enumerate(zip(cols_vals, cols_w)):
        n = int(v.numel())
        if n == 0:
            continue
        order = torch.argsort(v)
        vs[c, :n] = v[order]
        ww = (w[order] if w is not None else torch.ones(n, dtype=torch.float64, device=dev))
        cw[c, 1:n + 1] = torch.cumsum(ww, 0)
        cw[c, n + 1:] = cw[c, n]
        local_n[c] = n
    total = _allreduce(cw[:, -1].clone())
    # small distinct sets: gather them (the midpoint rule over <= n_bins distinct values)
    small = torch.zeros(C, dtype=torch.float64, device=dev)
    local_uniq = []
    for c in range(C):
        n = int(local_n[c])
        u = torch.unique_consecutive(vs[c, :n]) if n else vs[c, :0]
        local_uniq.append(u)
        small[c] = 1.0 if u.numel() <= n_bins else 0.0
    small = _allreduce(small, "min")
    small_cols = [c for c in range(C) if small[c] > 0]
    if small_cols:
        gathered = _gather_objects([local_uniq[c].cpu().numpy() for c in small_cols]) \
            if dist.info().world_size > 1 else [[local_uniq[c].cpu().numpy() for c in small_cols]]
        for i, c in enumerate(small_cols):
            u = np.unique(np.concatenate([g[i] for g in gathered]))
            if u.size == 0:
                out[c] = [float("-inf")]
            elif u.size <= n_bins:
                out[c] = [float("-inf")] + [float((u[k - 1] + u[k]) / 2.0) for k in range(1, u.size)]
    todo = [c for c in range(C) if out[c] is None]
    if not todo:
        return out
    idx = torch.tensor(todo, device=dev)
    T = total[idx]
    js = torch.arange(1, n_bins, dtype=torch.float64, device=dev)
    targets = T[:, None] * js[None, :] / n_bins                     # [c, j]
    mn = torch.where(local_n[idx] > 0, vs[idx, 0], torch.full_like(T, float("inf")))
    mx = torch.where(local_n[idx] > 0, vs[idx].gather(1, (local_n[idx].long() - 1).clamp(min=0)[:, None])[:, 0],
                     torch.full_like(T, float("-inf")))
    mn, mx = _allreduce(mn, "min"), _allreduce(mx, "max")
    lo = _key(mn)[:, None].expand(-1, n_bins - 1).clone()
    hi = _key(mx)[:, None].expand(-1, n_bins - 1).clone()
    sub_vs, sub_cw = vs[idx], cw[idx]
    # minimal key with C(key) >= target (C monotone; C(max) = total >= target)
    for _ in range(64):
        mid = (lo >> 1) + (hi >> 1) + (lo & hi & 1)
        x = _unkey(mid)
        pos = torch.searchsorted(sub_vs, x.contiguous(), right=True)       # [c, j] values <= x
        cnt = _allreduce(sub_cw.gather(1, pos))
        ge = cnt >= targets
        hi = torch.where(ge, mid, hi)
        lo = torch.where(ge, lo, mid + 1)
        if bool((lo >= hi).all()):
            break
    vk = _unkey(hi)
    # next distinct value above v_k (global MIN over ranks)
    pos = torch.searchsorted(sub_vs, vk.contiguous(), right=True)
    nxt = sub_vs.gather(1, pos.clamp(max=sub_vs.shape[1] - 1))
    nxt = torch.where(pos < local_n[idx].long()[:, None], nxt, torch.full_like(nxt, float("inf")))
    nxt = _allreduce(nxt, "min")
    vk_np, nx_np = vk.cpu().numpy(), nxt.cpu().numpy()
    for r, c in enumerate(todo):
        bounds = [float("-inf")]
        for j in range(n_bins - 1):
            if not np.isfinite(nx_np[r, j]):           # v_k is the last distinct value
                continue
            b = float((vk_np[r, j] + nx_np[r, j]) / 2.0)
            if b > bounds[-1]:
                bounds.append(b)
        out[c] = bounds
    return out


# ---- HyperLogLog (distinct counts of large columns across ranks) ------------------------------
def _splitmix64(x: torch.Tensor) -> torch.Tensor:
    x = x + (-7046029254386353131)                    # 0x9E3779B97F4A7C15 as int64
    x = (x ^ ((x >> 30) & 0x3FFFFFFFF)) * (-4658895280553007687)    # 0xBF58476D1CE4E5B9
    x = (x ^ ((x >> 27) & 0x1FFFFFFFFF)) * (-7723592293110705685)   # 0x94D049BB133111EB
    return x ^ ((x >> 31) & 0x1FFFFFFFF)


def hll_registers(vals: torch.Tensor, p: int = HLL_P) -> torch.Tensor:
    m = 1 << p
    if vals.numel() == 0:
        return torch.zeros(m, dtype=torch.int64, device=vals.device)
    h = _splitmix64(vals.contiguous().view(torch.int64))
    bucket = (h >> (64 - p)) & (m - 1)
    rest = (h << p) | (1 << (p - 1))                  # guard bit bounds the rank
    # rank = leading zeros of the 64-bit pattern + 1; for rest > 0 the top set bit is b:
    # floor(log2) through float64, corrected for the round-up near powers of two
    pos_ = rest.clamp(min=1)
    b = torch.floor(torch.log2(pos_.double())).long().clamp(max=62)
    b = torch.where(torch.bitwise_left_shift(torch.ones_like(b), b) > pos_, b - 1, b)
    rank = torch.where(rest < 0, torch.ones_like(rest), 63 - b + 1)
    reg = torch.zeros(m, dtype=torch.int64, device=vals.device)
    return reg.scatter_reduce(0, bucket, rank, reduce="amax")


def hll_estimate(reg: torch.Tensor, p: int = HLL_P) -> float:
    m = 1 << p
    r = reg.double()
    alpha = 0.7213 / (1 + 1.079 / m)
    e = alpha * m * m / float(torch.sum(torch.pow(2.0, -r)))
    zeros = int((reg == 0).sum())
    if e <= 2.5 * m and zeros:
        e = m * np.log(m / zeros)
    return float(e)


def global_distinct(vals: torch.Tensor) -> int:
    """Exact global distinct count when every rank's distinct set is small, else HyperLogLog."""
    u = torch.unique(vals)
    small = _allreduce(torch.tensor([1.0 if u.numel() <= DISTINCT_GATHER_CAP else 0.0], dtype=torch.float64,
                                    device=vals.device), "min")
    if small.item() > 0:
        if dist.info().world_size == 1:
            return int(u.numel())
        g = _gather_objects(u.cpu().numpy())
        return int(np.unique(np.concatenate(g)).size)
    reg = _allreduce(hll_registers(vals), "max")
    return int(round(hll_estimate(reg)))


# ---- the data-parallel stats pass -------------------------------------------------------------
def compute_column_stats_dp(mc, ccs, md, device=None, columns=None, batch: int = 64):
    """``compute_column_stats`` over this rank's rows ``md`` with every partial merged across
    ranks; fills the same ColumnConfig fields on every rank."""
    dev = torch.device(device) if device is not None else _dev()
    binary = mc.is_binary()
    method = mc.binning_method
    n_bins = int(mc.stats.get("maxNumBin", 10))
    cate_max = int(mc.stats.get("cateMaxNumBin", 0) or 0)
    num_thr = float(mc.stats.get("numericalValueThreshold", 1.7976931348623157e308))
    y = np.asarray(md.y)
    w = np.asarray(md.w, dtype=np.float64)
    total = int(_allreduce(torch.tensor([float(md.n)], dtype=torch.float64)).item())
    numeric, categorical = [], []
    for cc in ccs:
        if columns is not None and cc.name not in columns:
            continue
        if cc.is_target() or cc.is_meta() or cc.name not in md.table:
            continue
        (categorical if cc.is_categorical() else numeric).append(cc)

    # categorical: global first-appearance category order, merged histograms
    if categorical:
        local = []
        for cc in categorical:
            col = md.table[cc.name]
            if col.kind == "str":
                codes, dictionary = col.values, col.dictionary
            else:
                s = col.strings()
                uniq = {}
                codes = np.array([uniq.setdefault(v, len(uniq)) if v != "" else -1 for v in s], dtype=np.int32)
                dictionary = list(uniq.keys())
            local.append((codes, dictionary, B.categorical_bins(codes, dictionary, y, binary),
                          list(dictionary)))
        gathered = _gather_objects([(l[2], l[3]) for l in local]) if dist.info().world_size > 1 \
            else [[(l[2], l[3]) for l in local]]
        for k, cc in enumerate(categorical):
            codes, dictionary = local[k][0], local[k][1]
            cats, all_vals = [], []
            seen, seen_all = set(), set()
            for g in gathered:
                for c in g[k][0]:
                    if c not in seen:
                        seen.add(c)
                        cats.append(c)
                for c in g[k][1]:
                    if c not in seen_all:
                        seen_all.add(c)
                        all_vals.append(c)
            cats = cats[:10000]
            bidx = B.category_index(codes, dictionary, cats)
            nb = len(cats) + 1
            h = S._hist(bidx, y, w, nb, binary, dev)
            cpos = _allreduce(torch.as_tensor(h[0])).numpy()
            cneg = _allreduce(torch.as_tensor(h[1])).numpy()
            wpos = _allreduce(torch.as_tensor(h[2])).numpy()
            wneg = _allreduce(torch.as_tensor(h[3])).numpy()
            if cate_max > 0 and len(cats) > cate_max:
                cats, cpos, cneg, wpos, wneg = B.rebin_categorical(cats, list(cpos), list(cneg), list(wpos),
                                                                   list(wneg), cate_max)
                cpos, cneg = np.array(cpos, np.int64), np.array(cneg, np.int64)
                wpos, wneg = np.array(wpos), np.array(wneg)
                nb = len(cats) + 1
            cc.bin_category = cats
            cc.bin_boundary = None
            missing = int(cpos[-1] + cneg[-1]) if binary else int(cpos[-1])
            if cate_max <= 0:
                miss_local = int((bidx == len(cats)).sum())
                missing = int(_allreduce(torch.tensor([float(miss_local)], dtype=torch.float64)).item())
            if binary:
                rate = np.where(cpos + cneg > 0, cpos / np.maximum(cpos + cneg, 1), 0.0)
            else:
                tot = cpos.sum()
                rate = cpos / tot if tot else np.zeros_like(cpos, dtype=float)
            cnt = cpos + cneg if binary else cpos
            okr = np.isfinite(rate)
            mx = float(rate[okr].max()) if okr.any() else 0.0
            mn = float(rate[okr].min()) if okr.any() else 0.0
            S._finish_moments(cc, total - missing, float((rate * cnt).sum()), float((rate ** 2 * cnt).sum()),
                              float((rate ** 3 * cnt).sum()), float((rate ** 4 * cnt).sum()), mn, mx, total, missing)
            cc.stats["distinctCount"] = int(len(all_vals))
            cc.stats["median"] = None
            S._finish_binning(cc, binary, nb, cpos, cneg, wpos, wneg, total)

    # numeric: exact global boundaries, then merged histograms + moments
    for b0 in range(0, len(numeric), batch):
        cols = numeric[b0:b0 + batch]
        host = []
        for cc in cols:
            v = md.table[cc.name].numeric().astype(np.float64).copy()
            v[v > num_thr] = np.nan
            host.append(v)
        eqp, eqi = [], []
        for k, v in enumerate(host):
            if method in ("EqualInterval", "WeightEqualInterval"):
                eqi.append(k)
            else:
                eqp.append(k)
        bounds = [None] * len(cols)
        sel_masks = []
        if binary and method in ("EqualPositive", "WeightEqualPositive"):
            msel = y > 0.5
        elif binary and method in ("EqualNegtive", "WeightEqualNegative"):
            msel = y <= 0.5
        else:
            msel = np.ones(len(y), dtype=bool)
        # the reference re-cuts over all rows when a class-restricted cut degenerates (global flag)
        partial_sel = _allreduce(torch.tensor([float((~msel).sum())], dtype=torch.float64)).item() > 0
        for v in host:
            sel_masks.append(msel & np.isfinite(v))
        if eqp:
            weighted = method.startswith("Weight")
            vals = [torch.as_tensor(host[k][sel_masks[k]], device=dev) for k in eqp]
            ws = [torch.as_tensor(w[sel_masks[k]], device=dev) if weighted else None for k in eqp]
            res = exact_equal_population(vals, ws, n_bins, dev)
            # reference fallback: a class-restricted cut with < 2 boundaries re-cuts over all rows
            redo = [i for i, k in enumerate(eqp) if len(res[i]) <= 1 and partial_sel]
            if redo:
                vals2 = [torch.as_tensor(host[eqp[i]][np.isfinite(host[eqp[i]])], device=dev) for i in redo]
                res2 = exact_equal_population(vals2, [None] * len(redo), n_bins, dev)
                for i, r in zip(redo, res2):
                    res[i] = r
            for i, k in enumerate(eqp):
                bounds[k] = res[i]
        for k in eqi:
            fin = host[k][np.isfinite(host[k])]
            t = torch.tensor([fin.min() if fin.size else np.inf, -(fin.max() if fin.size else -np.inf)],
                             dtype=torch.float64)
            t = _allreduce(t, "min")
            lo, hi = float(t[0]), -float(t[1])
            if not np.isfinite(lo) or hi <= lo:
                bounds[k] = [float("-inf")]
            else:
                step = (hi - lo) / n_bins
                bounds[k] = [float("-inf")] + [lo + i * step for i in range(1, n_bins)]
        for k, cc in enumerate(cols):
            v = host[k]
            bidx = B.bin_index_numeric(v, bounds[k])
            h = S._hist(bidx, y, w, len(bounds[k]) + 1, binary, dev)
            cpos = _allreduce(torch.as_tensor(h[0])).numpy()
            cneg = _allreduce(torch.as_tensor(h[1])).numpy()
            wpos = _allreduce(torch.as_tensor(h[2])).numpy()
            wneg = _allreduce(torch.as_tensor(h[3])).numpy()
            mom = S._moments(v, dev)
            sums = _allreduce(torch.tensor(mom[:5], dtype=torch.float64)).tolist()
            mn = _allreduce(torch.tensor([mom[5] if mom[0] else np.inf], dtype=torch.float64), "min").item()
            mx = _allreduce(torch.tensor([mom[6] if mom[0] else -np.inf], dtype=torch.float64), "max").item()
            if sums[0] == 0:
                mn = mx = float("nan")
            fin = torch.as_tensor(v[np.isfinite(v)], device=dev)
            distinct = global_distinct(fin)
            S._finish_numeric(cc, binary, bounds[k], cpos, cneg, wpos, wneg,
                              (int(sums[0]), sums[1], sums[2], sums[3], sums[4], mn, mx), total, distinct)
    return ccs
