"""Exact EvalPerformance over row-sharded scores (K16, multi-rank), without gathering the rows.

The reference sorts every scored record globally (Pig ``ORDER BY score DESC``, P/Eval.pig:38-39)
and streams the sorted rows through ``ConfusionMatrix.bufferedComputeConfusionMatrixAndPerformance``
(J/core/ConfusionMatrix.java:276-507).  Every quantity that stream produces is a function of a
GLOBAL PREFIX of the sorted order (descending score, ties in row order = rank-major order here),
so each rank only sorts its own rows (radix sort on the device) and keeps prefix sums of count,
tp, fp, weighted tp / fp and weight.  A global prefix is then located by bisection over the
64-bit order-preserving score keys -- one all-reduce of the candidate prefixes' sums per step --
and the tie group at the found key is split across ranks in rank order (one all-gather):

  round 1  curve buckets: the first prefix whose fpr / recall / action rate / weighted variants
           reaches k / B (the same floating predicate as the single-process sweep);
  round 2  the confusion values and the score at every emitted position (position predicates).

Score buckets need only the global count of scores above each bucket threshold.  Counts are exact
integers, so the unweighted curves and every emitted position equal the single-process result;
weighted sums differ from a sequential cumsum only by summation order.  ``performance`` on one
rank is the single-process function itself.
"""
from __future__ import annotations

import math
import struct
from collections import OrderedDict

import numpy as np
import torch

from ..parallel import dist
from . import evaluation as E

_I64MAX = 0x7FFFFFFFFFFFFFFF
_LO, _HI = -(1 << 63), (1 << 63) - 1
Q_CNT, Q_TP, Q_FP, Q_WTP, Q_WFP, Q_W = range(6)


def _keys(s: torch.Tensor) -> torch.Tensor:
    """fp64 scores -> int64 keys with the same order (NaN ranks as -inf; -0.0 == 0.0)."""
    s = torch.where(torch.isnan(s), torch.full_like(s, -math.inf), s) + 0.0
    b = s.view(torch.int64)
    return torch.where(b >= 0, b, b ^ _I64MAX)


def _unkey(k: int) -> float:
    b = k if k >= 0 else k ^ _I64MAX
    return struct.unpack("<d", struct.pack("<q", b))[0]


def _key_of(x: float) -> int:
    x = float(x) + 0.0
    b = struct.unpack("<q", struct.pack("<d", x))[0]
    return b if b >= 0 else b ^ _I64MAX


class _Local:
    """One rank's rows sorted descending + prefix sums [6, n + 1] (count, tp, fp, wtp, wfp, w)."""

    def __init__(self, score, is_pos, weight, dev):
        s = E._as_dev(score, dev)
        p = E._as_dev(is_pos, dev)
        w = torch.ones_like(s) if weight is None else E._as_dev(weight, dev)
        order = E.order_desc(s)
        key = _keys(s)[order]
        self.nk = (~key).contiguous()                 # ascending
        self.s = s[order]                             # the scores themselves (NaN vs -inf kept)
        p, w = p[order], w[order]
        self.n = s.numel()
        z = torch.zeros(1, dtype=torch.float64, device=dev)
        c = lambda v: torch.cat([z, torch.cumsum(v, 0)])
        self.cum = torch.stack([torch.arange(self.n + 1, dtype=torch.float64, device=dev), c(p), c(1 - p),
                                c(p * w), c((1 - p) * w), c(w)])
        self.dev = dev

    def count_ge(self, v: list) -> torch.Tensor:
        """#local rows with key >= v[t] (int64 [T])."""
        vt = torch.tensor(v, dtype=torch.int64, device=self.dev)
        return torch.searchsorted(self.nk, ~vt, right=True)


def _gather(t: torch.Tensor) -> np.ndarray:
    """[R, *t.shape] of every rank's ``t`` (host numpy, rank order)."""
    R = dist.info().world_size
    if R == 1:
        return t.detach().cpu().numpy()[None]
    out = [torch.empty_like(t) for _ in range(R)]
    torch.distributed.all_gather(out, t.contiguous())
    return torch.stack(out).cpu().numpy()


def _rsum(a: np.ndarray) -> np.ndarray:
    """Sum over the leading (rank) axis strictly in rank order: a global prefix in which ranks
    0..r-1 are complete then sums their totals exactly as the global totals are summed, so e.g. a
    weighted recall reaches 1.0 exactly at the last positive, as the sequential sweep does."""
    out = a[0].copy()
    for r in range(1, len(a)):
        out = out + a[r]
    return out


def _cross(loc: _Local, coef: np.ndarray, den: np.ndarray, thr: np.ndarray):
    """For targets t: the smallest global prefix whose Q_t = coef[t] . sums satisfies
    Q_t / den[t] >= thr[t].  Returns (found [T] bool, per-rank prefix lengths [T, R] int64, key of
    the prefix's last row [T]).  Global sums are rank-order sums of the ranks' prefix values."""
    T = len(thr)
    R = dist.info().world_size
    dev = loc.dev
    C = torch.as_tensor(coef, dtype=torch.float64, device=dev)           # [T, 6]
    Cn = np.asarray(coef, dtype=np.float64)
    D = np.asarray(den, dtype=np.float64)
    c = np.asarray(thr, dtype=np.float64)

    def pred(q):                                      # q: [T] global prefix values (host)
        with np.errstate(divide="ignore", invalid="ignore"):
            return np.where(D != 0, q / np.where(D != 0, D, 1.0), np.nan) >= c

    def q_at(counts):                                 # local prefix values at per-target lengths
        return (C * loc.cum[:, counts].t()).sum(1)

    def q_global(v):
        return _rsum(_gather(q_at(loc.count_ge(v))))

    lo, hi = [_LO] * T, [_HI] * T
    found = pred(q_global(lo))
    for _ in range(64):
        if all(h - l <= 1 for l, h in zip(lo, hi)):
            break
        mid = [l + (h - l) // 2 for l, h in zip(lo, hi)]
        ok = pred(q_global(mid))
        lo = [m if o else l for m, o, l in zip(mid, ok, lo)]
        hi = [h if o else m for m, o, h in zip(mid, ok, hi)]
    vstar = lo
    # tie group key == v*: rows [a_r, b_r) on every rank, taken in rank order
    a = loc.count_ge([v + 1 if v < _HI else v for v in vstar])
    b = loc.count_ge(vstar)
    allinfo = _gather(torch.stack([q_at(a), q_at(b), a.double(), b.double()], 1))    # [R, T, 4]
    me = dist.info().rank
    m_out = np.zeros((T, R), dtype=np.int64)
    rst = np.full(T, -1, dtype=np.int64)
    mine = torch.zeros(T, dtype=torch.float64, device=dev)
    for t in range(T):
        if not found[t]:
            continue
        qa, qb = allinfo[:, t, 0], allinfo[:, t, 1]
        rstar = None
        for r in range(R):                            # rank r's whole tie group taken
            q = _rsum(np.concatenate([qb[: r + 1], qa[r + 1:]])[:, None])[0]
            if D[t] != 0 and q / D[t] >= c[t]:
                rstar = r
                break
        if rstar is None:                             # rounding: the whole group
            rstar = R - 1
        rst[t] = rstar
        for r in range(R):
            m_out[t, r] = int(allinfo[r, t, 3]) if r <= rstar else int(allinfo[r, t, 2])
        if me == rstar:
            ai, bi = int(a[t]), int(b[t])
            part = (C[t] @ loc.cum[:, ai + 1: bi + 1]).cpu().numpy()      # Q_r*(m), m = a+1..b
            left = _rsum(qb[:rstar, None])[0] if rstar > 0 else None
            vals = part if left is None else left + part
            for r in range(rstar + 1, R):
                vals = vals + qa[r]
            hit = np.nonzero(pred_vec(vals, D[t], c[t]))[0]
            mine[t] = ai + 1 + (int(hit[0]) if len(hit) else bi - ai - 1)
    mh = _rsum(_gather(mine))
    for t in range(T):
        if found[t]:
            m_out[t, rst[t]] = int(mh[t])
    return found, m_out, vstar, rst


def pred_vec(q, d, c):
    if d == 0:
        return np.zeros(len(q), dtype=bool)
    return q / d >= c


def performance(score, is_pos, weight=None, num_bucket: int = 10, max_score: float = 1000.0,
                min_score: float = 0.0, device=None, version: str = "0.13.0"):
    """EvalPerformance.json of the union of every rank's rows (rank-major row order), on every
    rank; single process: ``evaluation.performance``."""
    info = dist.info()
    if info.world_size == 1:
        return E.performance(score, is_pos, weight, num_bucket, max_score, min_score, device, version)
    dev = device or (score.device if torch.is_tensor(score) else
                     (torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")))
    loc = _Local(score, is_pos, weight, dev)
    tot = _rsum(_gather(loc.cum[:, -1].clone()))
    n, P, Nn, WP, WN = (float(tot[q]) for q in (Q_CNT, Q_TP, Q_FP, Q_WTP, Q_WFP))
    N = int(n)
    nb, cap = num_bucket, 1.0 / num_bucket
    e = np.eye(6)
    curves = (("roc", e[Q_FP], Nn), ("pr", e[Q_TP], P), ("gains", e[Q_CNT], float(max(N, 1))),
              ("weightedRoc", e[Q_WFP], WN), ("weightedPr", e[Q_WTP], WP),
              ("weightedGains", e[Q_WTP] + e[Q_WFP], WP + WN))
    coef, den, thr, tag = [], [], [], []
    for key, cf, d in curves:
        for k in range(1, nb + 2):
            coef.append(cf)
            den.append(d)
            thr.append(k * cap)
            tag.append((key, k))
    found, m, _, _ = _cross(loc, np.array(coef), np.array(den), np.array(thr))
    u = {t: (int(m[i].sum()) if found[i] else None) for i, t in enumerate(tag)}
    marks = OrderedDict()
    for key, _, _ in curves:
        out, prev = [], 0
        for k in range(1, nb + 2):
            uk = u[(key, k)]
            if uk is None:
                break
            j = max(uk, prev + 1)
            if j >= N + 1:
                break
            out.append((k, j))
            prev = j
        marks[key] = out
    # score buckets: bucket k closes at 1 + #(score > max_score - k * bin_score) (or last + 1)
    bin_score = (max_score - min_score) / nb
    emits, k, last = [], 1, 0
    while last < N:
        ks = list(range(k, k + 16))
        v = [(_key_of(max_score - kk * bin_score) + 1) for kk in ks]
        cnt = _rsum(_gather(loc.count_ge([min(x, _HI) for x in v]).double()))
        stop = False
        for kk, cg in zip(ks, cnt):
            j = max(int(cg) + 1, last + 1)
            if j > N:
                stop = True
                break
            emits.append((kk, j, last))
            last = j
            if last >= N:
                stop = True
                break
        if stop:
            break
        k = ks[-1] + 1
    # round 2: confusion values + score at every emitted position
    pos = sorted({j for v_ in marks.values() for _, j in v_} | {j for _, j, _ in emits} |
                 {l for _, _, l in emits if l > 0})
    vals = {0: np.zeros(6)}
    score_at = {0: float(max_score)}
    if pos:
        T = len(pos)
        found2, m2, vst, own = _cross(loc, np.tile(e[Q_CNT], (T, 1)), np.ones(T), np.array(pos, dtype=np.float64))
        me = dist.info().rank
        cnts = torch.as_tensor(m2[:, me], device=dev)
        qh = _rsum(_gather(loc.cum[:, cnts].t().contiguous()))        # [T, 6]
        # the j-th row's own score, from the rank that holds it (a tie group keyed -inf mixes -inf
        # and NaN scores)
        mine = torch.zeros(T, dtype=torch.float64, device=dev)
        for i in range(T):
            if own[i] == me and m2[i, me] > 0:
                mine[i] = loc.s[int(m2[i, me]) - 1]
        sc = _gather(mine)
        for i, j in enumerate(pos):
            vals[j] = qh[i]
            score_at[j] = float(sc[own[i], i]) if own[i] >= 0 else _unkey(vst[i])
    keys = ("tp", "fp", "fn", "tn", "wtp", "wfp", "wfn", "wtn", "score")
    idx = sorted(vals)
    rowpos = {j: q_ for q_, j in enumerate(idx)}
    V = np.stack([vals[j] for j in idx])
    tp, fp, wtp, wfp = V[:, Q_TP], V[:, Q_FP], V[:, Q_WTP], V[:, Q_WFP]
    hcm = dict(tp=tp, fp=fp, fn=P - tp, tn=Nn - fp, wtp=wtp, wfp=wfp, wfn=WP - wtp, wtn=WN - wfp,
               score=np.array([score_at[j] for j in idx]))
    hw = V[:, Q_W]
    first = E._po(0, hcm, first=True)
    lists = OrderedDict()
    for key in ("roc", "pr", "gains", "weightedRoc", "weightedPr", "weightedGains"):
        lists[key] = [first] + [E._po(rowpos[j], hcm, kk) for kk, j in marks[key]]
    ms = [first] + [E._po(rowpos[j], hcm, kk, float(j - l), float(hw[rowpos[j]] - hw[rowpos[l]]))
                    for kk, j, l in emits]
    res = OrderedDict(version=version)
    res["areaUnderRoc"] = E.auc(lists["roc"], "fpr", "recall")
    res["weightedAreaUnderRoc"] = E.auc(lists["weightedRoc"], "weightedFpr", "weightedRecall")
    res["areaUnderPr"] = E.auc(lists["pr"], "recall", "precision")
    res["weightedAreaUnderPr"] = E.auc(lists["weightedPr"], "weightedRecall", "weightedPrecision")
    for key in ("pr", "weightedPr", "roc", "weightedRoc", "gains", "weightedGains"):
        res[key] = lists[key]
    res["modelScoreList"] = ms
    return res
