"""K4: exact equal-population binning on the device, as three mergeable passes (+ K19 HLL).

The reference cuts numeric columns from per-mapper streaming histograms merged in a reducer
(``EqualPopulationBinning`` J/core/binning/EqualPopulationBinning.java:491,
``UpdateBinningInfoMapper`` J/core/binning/UpdateBinningInfoMapper.java:349-599,
``MapReducerStatsWorker`` J/core/processor/stats/MapReducerStatsWorker.java:105-176).  Here the
cut is EXACT - the same boundaries as :func:`binning.equal_population_boundaries` (first distinct
value whose cumulative count reaches ``j * total / bins``, cut halfway to the next distinct value;
columns with at most ``bins`` distinct values cut between every pair) - and costs three streaming
passes over the column batch (``ops/csrc/quantile_kernels.hip``):

A  ``qprep``   min/max keys of the selected and of all finite values, selected count, HLL(p=14);
B  ``qhist``   2048 linear buckets over [lo, hi]: count, fixed-point weight, min/max key per
               bucket (+ min/max keys per bucket of all finite values for exact distinct counts);
C  ``qgather`` the values of the few buckets that hold a cut target AND more than one distinct
               value (each ~N/2048 rows), sorted on the device and searched.

Every pass accumulates, so the engine is fed either one resident column batch, a stream of row
chunks (host RSS bounded by the chunk), or one row shard per rank with ``reduce`` = an
all-reduce between passes and ``allgather`` for the gathered values.  CPU runs use a torch
implementation of the same three passes (the oracle for the HIP kernels).

Ranks are integers (counts, or weights in fixed point with ``wscale``), so the cumulative-rank
comparisons are exact; for the Weight* methods a weight with more fractional bits than the fixed
point carries can in rare ties move a cut relative to the float64 host rule.  Negative weights
count as 0.
"""
from __future__ import annotations

import math

import numpy as np
import torch

NB = 2048
HLL_P = 14
HLL_M = 1 << HLL_P
_I64_MIN = -(1 << 63)
_I64_MAX = (1 << 63) - 1
_MAG = 0x7FFFFFFFFFFFFFFF

EMPTY, SMALL, EQPOP, AMBIG, INTERVAL = range(5)


def skey(x: torch.Tensor) -> torch.Tensor:
    """float64 -> signed-comparable int64 key (order preserving)."""
    b = x.contiguous().view(torch.int64)
    return torch.where(b < 0, b ^ _MAG, b)


def unskey(k: torch.Tensor) -> torch.Tensor:
    return torch.where(k < 0, k ^ _MAG, k).view(torch.float64)


def _unskey_np(k: np.ndarray) -> np.ndarray:
    k = np.asarray(k, np.int64)
    return np.where(k < 0, k ^ _MAG, k).view(np.float64)


def _splitmix64(x: torch.Tensor) -> torch.Tensor:
    x = x + (-7046029254386353131)                    # 0x9E3779B97F4A7C15
    x = (x ^ ((x >> 30) & 0x3FFFFFFFF)) * (-4658895280553007687)
    x = (x ^ ((x >> 27) & 0x1FFFFFFFFF)) * (-7723592293110705685)
    return x ^ ((x >> 31) & 0x1FFFFFFFF)


def hll_update(reg: torch.Tensor, vals: torch.Tensor) -> None:
    """reg [HLL_M] int64 in place; vals: canonical finite float64 (same hash/rank as qprep)."""
    if vals.numel() == 0:
        return
    h = _splitmix64(vals.contiguous().view(torch.int64))
    bucket = (h >> (64 - HLL_P)) & (HLL_M - 1)
    rest = (h << HLL_P) | (1 << (HLL_P - 1))
    pos = rest.clamp(min=1)
    b = torch.floor(torch.log2(pos.double())).long().clamp(max=62)
    b = torch.where(torch.bitwise_left_shift(torch.ones_like(b), b) > pos, b - 1, b)
    rank = torch.where(rest < 0, torch.ones_like(rest), 64 - b)
    reg.scatter_reduce_(0, bucket, rank, reduce="amax")


def hll_estimate(reg) -> float:
    r = np.asarray(reg, np.float64)
    m = r.size
    alpha = 0.7213 / (1 + 1.079 / m)
    e = alpha * m * m / float(np.sum(np.power(2.0, -r)))
    zeros = int((r == 0).sum())
    if e <= 2.5 * m and zeros:
        e = m * math.log(m / zeros)
    return float(e)


def sel_mode_for(method: str, binary: bool) -> int:
    if binary and method in ("EqualPositive", "WeightEqualPositive"):
        return 1
    if binary and method in ("EqualNegtive", "WeightEqualNegative"):
        return 2
    return 0


def _clean(vals: torch.Tensor, thr: float) -> torch.Tensor:
    v = torch.where(vals > thr, torch.full_like(vals, float("nan")), vals)
    return v + 0.0


def _selmask(y: torch.Tensor | None, mode: int, n: int, dev) -> torch.Tensor:
    if mode == 0 or y is None:
        return torch.ones(n, dtype=torch.bool, device=dev)
    return (y > 0.5) if mode == 1 else ~(y > 0.5)


def _bucket(v: torch.Tensor, lo: torch.Tensor, sc: torch.Tensor) -> torch.Tensor:
    f = (v - lo[:, None]) * sc[:, None]
    f = torch.nan_to_num(f, nan=0.0, posinf=float(NB), neginf=0.0)
    b = torch.where(f <= 0, torch.zeros_like(f), torch.where(f >= NB - 1, torch.full_like(f, NB - 1), f))
    return b.long()


class QuantileEngine:
    """Exact cuts for a batch of ``C`` numeric columns; see the module docstring.

    ``reduce(t, op)`` (op in sum/min/max) merges state across ranks in place; ``allgather(t)``
    returns the concatenation of a 1-D tensor over ranks (both identity for one process)."""

    def __init__(self, C: int, n_bins: int, sel_mode: int = 0, weighted: bool = False, interval: bool = False,
                 num_thr: float = 1.7976931348623157e308, device=None, reduce=None, allgather=None):
        self.C, self.nb = int(C), int(n_bins)
        self.sel_mode, self.weighted, self.interval = int(sel_mode), bool(weighted), bool(interval)
        self.thr = float(num_thr)
        self.dev = torch.device(device or "cpu")
        self.hip = self.dev.type == "cuda"
        self.reduce = reduce
        self.allgather = allgather
        self.with_all = self.sel_mode != 0
        C, dev, i64 = self.C, self.dev, torch.int64
        if self.hip:
            from ..ops import _native as nat
            nat.require_gpu_native()
            self._nat = nat
            # unsigned key patterns: min slots start at ~0 (= -1), max slots at 0
            self.mm = torch.tensor([-1, 0, -1, 0] * C, dtype=i64, device=dev).view(C, 4)
        else:
            self.mm = torch.tensor([_I64_MAX, _I64_MIN, _I64_MAX, _I64_MIN] * C, dtype=i64, device=dev).view(C, 4)
        self.scnt = torch.zeros(C, dtype=i64, device=dev)
        self.hll = torch.zeros(C, HLL_M, dtype=torch.int32 if self.hip else i64, device=dev)
        self.wmax = 0.0
        self.stage = "a"

    # ---- helpers -----------------------------------------------------------------------------
    def _red(self, t, op):
        if self.reduce is not None:
            self.reduce(t, op)
        return t

    def _check(self, vals, y, w):
        if vals.dim() != 2 or vals.shape[0] != self.C or vals.dtype != torch.float64 or vals.stride(1) != 1:
            raise ValueError("QuantileEngine: vals must be [C, n] float64 with unit row stride")
        n = vals.shape[1]
        if self.sel_mode and (y is None or y.numel() < n):
            raise ValueError("QuantileEngine: y required for class-restricted methods")
        if self.weighted and (w is None or w.numel() < n):
            raise ValueError("QuantileEngine: weights required for Weight* methods")
        return n

    def _stream(self):
        return self._nat.stream_of(self.mm)

    # ---- pass A ------------------------------------------------------------------------------
    def pass_a(self, vals: torch.Tensor, y=None, w=None) -> None:
        n = self._check(vals, y, w)
        if n == 0:
            return
        if self.weighted:
            sm = _selmask(y, self.sel_mode, n, vals.device)
            if bool(sm.any()):
                self.wmax = max(self.wmax, float(w[:n][sm].clamp(min=0).max()))
        if self.hip:
            self._nat.call_hip("shifu_qprep", vals, vals.stride(0), n, self.C, y if self.sel_mode else None,
                               self.sel_mode, self.thr, self.mm, self.scnt, self.hll, self._stream())
            return
        v = _clean(vals, self.thr)
        fin = torch.isfinite(v)
        sel = fin & _selmask(y, self.sel_mode, n, v.device)[None, :]
        k = skey(torch.where(fin, v, torch.zeros_like(v)))
        mx, mn = torch.full_like(k, _I64_MAX), torch.full_like(k, _I64_MIN)
        self.mm[:, 0] = torch.minimum(self.mm[:, 0], torch.where(sel, k, mx).amin(1))
        self.mm[:, 1] = torch.maximum(self.mm[:, 1], torch.where(sel, k, mn).amax(1))
        self.mm[:, 2] = torch.minimum(self.mm[:, 2], torch.where(fin, k, mx).amin(1))
        self.mm[:, 3] = torch.maximum(self.mm[:, 3], torch.where(fin, k, mn).amax(1))
        self.scnt += sel.sum(1)
        for c in range(self.C):
            hll_update(self.hll[c], v[c][fin[c]])

    def finish_a(self) -> None:
        if self.hip:
            self.mm ^= _I64_MIN                                   # unsigned -> signed-comparable
            self.hll = self.hll.long()
        mn = self.mm[:, [0, 2]].contiguous()
        mx = self.mm[:, [1, 3]].contiguous()
        self._red(mn, "min")
        self._red(mx, "max")
        self.mm[:, 0], self.mm[:, 2] = mn[:, 0], mn[:, 1]
        self.mm[:, 1], self.mm[:, 3] = mx[:, 0], mx[:, 1]
        self._red(self.scnt, "sum")
        self._red(self.hll, "max")
        if self.weighted:
            t = torch.tensor([self.wmax], dtype=torch.float64, device=self.dev)
            self._red(t, "max")
            self.wmax = float(t.item())
        mm = self.mm.cpu().numpy()
        self.scnt_np = self.scnt.cpu().numpy()
        self.lo, self.hi = _unskey_np(mm[:, 0]), _unskey_np(mm[:, 1])
        alo, ahi = _unskey_np(mm[:, 2]), _unskey_np(mm[:, 3])
        self.any_fin = mm[:, 2] <= mm[:, 3]
        self.prm_np = np.zeros((self.C, 4), np.float64)
        for c in range(self.C):
            if self.scnt_np[c] > 0:
                self.prm_np[c, :2] = _mapping(self.lo[c], self.hi[c])
            if self.any_fin[c]:
                self.prm_np[c, 2:] = _mapping(alo[c], ahi[c])
        self.win_np = np.tile(np.array([_I64_MIN, _I64_MAX], np.int64), (self.C, 1))
        nmax = max(int(self.scnt_np.max()) if self.C else 1, 1)
        if self.weighted:
            lim = 2.0 ** 61 / (max(self.wmax, 1e-300) * nmax * max(self.nb, 1))
            self.wscale = 2.0 ** max(-60, min(40, math.floor(math.log2(lim))))
        else:
            self.wscale = 1.0
        C, dev, i64 = self.C, self.dev, torch.int64
        self.cnt = torch.zeros(C, NB, dtype=i64, device=dev)
        self.wq = torch.zeros(C, NB, dtype=i64, device=dev) if self.weighted else None
        self._init_mn, self._init_mx = (-1, 0) if self.hip else (_I64_MAX, _I64_MIN)
        self.kmn = torch.full((C, NB), self._init_mn, dtype=i64, device=dev)
        self.kmx = torch.full((C, NB), self._init_mx, dtype=i64, device=dev)
        self.akmn = torch.full((C, NB), self._init_mn, dtype=i64, device=dev) if self.with_all else None
        self.akmx = torch.full((C, NB), self._init_mx, dtype=i64, device=dev) if self.with_all else None
        self.level = 1
        self.cols = [_Col() for _ in range(C)]
        self.active = [c for c in range(C) if self.any_fin[c]]
        self.slots = []                       # (column, bucket) gathered in pass C
        self._upload_level()
        self.stage = "b"

    def _upload_level(self):
        self.prm = torch.as_tensor(self.prm_np, device=self.dev)
        w = self.win_np ^ _I64_MIN if self.hip else self.win_np      # unsigned patterns for HIP
        self.win = torch.as_tensor(np.ascontiguousarray(w), device=self.dev)
        self.colmap = torch.as_tensor(np.asarray(self.active or [0], np.int32), device=self.dev)

    # ---- pass B ------------------------------------------------------------------------------
    def pass_b(self, vals: torch.Tensor, y=None, w=None) -> None:
        n = self._check(vals, y, w)
        if n == 0 or not self.active:
            return
        with_all = self.with_all and self.level == 1
        if self.hip:
            self._nat.call_hip("shifu_qhist", vals, vals.stride(0), n, self.C, y if self.sel_mode else None,
                               w if self.weighted else None, self.sel_mode, self.thr, self.colmap, len(self.active),
                               self.win, self.prm, self.wscale, int(with_all), self.cnt, self.wq, self.kmn, self.kmx,
                               self.akmn, self.akmx, self._stream())
            return
        act = torch.as_tensor(self.active, device=vals.device)
        v = _clean(vals[act], self.thr)
        fin = torch.isfinite(v)
        vz = torch.where(fin, v, torch.zeros_like(v))
        k = skey(vz)
        win = self.win[act]
        sel = fin & _selmask(y, self.sel_mode, n, v.device)[None, :] & (k >= win[:, :1]) & (k <= win[:, 1:])
        base = (act * NB)[:, None]
        b = _bucket(vz, self.prm[act, 0], self.prm[act, 1]) + base
        bs, ks = b[sel], k[sel]
        self.cnt.view(-1).scatter_add_(0, bs, torch.ones_like(bs))
        self.kmn.view(-1).scatter_reduce_(0, bs, ks, reduce="amin")
        self.kmx.view(-1).scatter_reduce_(0, bs, ks, reduce="amax")
        if self.weighted:
            q = torch.round(w[:n].clamp(min=0) * self.wscale).long()[None, :].expand(len(self.active), n)[sel]
            self.wq.view(-1).scatter_add_(0, bs, q)
        if with_all:
            ab = _bucket(vz, self.prm[act, 2], self.prm[act, 3]) + base
            self.akmn.view(-1).scatter_reduce_(0, ab[fin], k[fin], reduce="amin")
            self.akmx.view(-1).scatter_reduce_(0, ab[fin], k[fin], reduce="amax")

    def finish_b(self) -> str:
        """Merge this level's histograms and plan every active column: returns "B" when some
        column refines into a narrower window (another pass B), "C" when values must be gathered,
        "done" otherwise."""
        if self.hip:
            for t in (self.kmn, self.kmx) + ((self.akmn, self.akmx) if self.with_all and self.level == 1 else ()):
                t ^= _I64_MIN
        if self.level == 1:
            self.local_cnt = self.cnt.clone()
        else:
            self.local_cnt[self.active_t()] = self.cnt[self.active_t()]
        if self.reduce is not None:       # merge only this level's rows (finished rows are merged)
            idx = self.active_t()
            for t, op in ((self.cnt, "sum"), (self.wq, "sum"), (self.kmn, "min"), (self.kmx, "max")):
                if t is None:
                    continue
                sub = t[idx].contiguous()
                self._red(sub, op)
                t[idx] = sub
        if self.with_all and self.level == 1:
            self._red(self.akmn, "min")
            self._red(self.akmx, "max")
            self.akmn_np, self.akmx_np = self.akmn.cpu().numpy(), self.akmx.cpu().numpy()
        act = self.active
        cnt = self.cnt.cpu().numpy()
        rank = self.wq.cpu().numpy() if self.weighted else cnt
        kmn, kmx = self.kmn.cpu().numpy(), self.kmx.cpu().numpy()
        if self.level == 1:
            self.h1 = (cnt.copy(), kmn.copy(), kmx.copy())
        refine = []
        for c in act:
            if self._plan(c, cnt[c], rank[c], kmn[c], kmx[c]):
                refine.append(c)
        if refine:
            self.level += 1
            self.active = refine
            idx = torch.as_tensor(refine, device=self.dev)
            self.cnt[idx] = 0
            if self.weighted:
                self.wq[idx] = 0
            if self.hip:      # kernels keep unsigned patterns; planned columns keep signed state
                self.kmn[idx] = self._init_mn
                self.kmx[idx] = self._init_mx
            else:
                self.kmn[idx] = _I64_MAX
                self.kmx[idx] = _I64_MIN
            if self.hip:      # the next finish_b flips every row: pre-flip the finished ones
                keep = torch.ones(self.C, dtype=torch.bool, device=self.dev)
                keep[idx] = False
                self.kmn[keep] ^= _I64_MIN
                self.kmx[keep] ^= _I64_MIN
            self._upload_level()
            return "B"
        self.active = []
        return self._plan_gather()

    def active_t(self):
        return torch.as_tensor(self.active, device=self.dev)

    def _plan(self, c, cnt, rank, kmn, kmx) -> bool:
        """One level of column ``c``; True when it refines into a narrower window."""
        st, nb = self.cols[c], self.nb
        ne_mask = cnt > 0
        multi = ne_mask & (kmn != kmx)
        ne, mu = int(ne_mask.sum()), int(multi.sum())
        if self.level == 1:
            if self.scnt_np[c] == 0 or ne == 0:
                st.mode = EMPTY
                return False
            if self.interval:
                st.mode = INTERVAL
                return False
            T = int(rank.sum())
            st.pending = [(j, -((-j * T) // nb)) for j in range(1, nb)]      # ceil(j*T/nb), exact
            if mu == 0 and ne <= nb:
                st.mode, st.small = SMALL, _unskey_np(kmn[ne_mask])
                return False
            st.mode = EQPOP if ne + mu > nb else AMBIG
        # AMBIG: decide small vs equal-population once the distinct count is known
        if st.mode == AMBIG:
            if len(st.outside) + ne + mu > nb:
                st.mode = EQPOP
            elif mu == 0:
                st.small = np.sort(np.concatenate([np.asarray(st.outside, np.float64),
                                                   _unskey_np(kmn[ne_mask])]))
                st.distinct = int(st.small.size)
                if st.small.size <= nb:
                    st.mode = SMALL
                    return False
                st.mode = EQPOP
        # targets: single-valued buckets resolve here, the rest stay pending
        cum = st.off + np.cumsum(rank)
        nxt_ne = _next_nonempty(ne_mask)
        pend = []
        for j, s in st.pending:
            b = int(np.searchsorted(cum, s, side="left"))
            b = min(b, NB - 1)
            if not ne_mask[b]:
                b = int(nxt_ne[b])
                if b < 0:                       # beyond the window (cannot happen for valid ranks)
                    continue
            if not multi[b]:
                st.res[j] = (float(_unskey_np(kmn[b])), self._after_bucket(st, b, ne_mask, kmn, nxt_ne))
            else:
                before = int(cum[b - 1]) if b > 0 else st.off
                pend.append((j, s, b, s - before))
        st.pending = [(j, s) for j, s, _, _ in pend]
        need = sorted({b for _, _, b, _ in pend})
        if st.mode == AMBIG:
            need = [int(b) for b in np.nonzero(multi)[0]]
        if not need:
            st.done = True
            return False
        if self.level < MAX_LEVEL and int(cnt[need].max()) > GATHER_CAP:
            f, l = need[0], need[-1]
            if st.mode == AMBIG:          # single values outside the new window stay known
                outside = ne_mask & ~multi
                outside[f:l + 1] = False
                st.outside += list(_unskey_np(kmn[outside]))
            st.off = int(cum[f - 1]) if f > 0 else st.off
            st.after = self._after_bucket(st, l, ne_mask, kmn, nxt_ne)
            self.win_np[c] = (kmn[f], kmx[l])
            self.prm_np[c, :2] = _mapping(float(_unskey_np(kmn[f])), float(_unskey_np(kmx[l])))
            return True
        # final level: gather the pending buckets (AMBIG: every multi bucket)
        st.gather = [(b, [(j, nd) for j, _, bb, nd in pend if bb == b],
                      self._after_bucket(st, b, ne_mask, kmn, nxt_ne)) for b in need]
        st.singles = _unskey_np(kmn[ne_mask & ~multi])
        self.slots += [(c, b) for b in need]
        return False

    @staticmethod
    def _after_bucket(st, b, ne_mask, kmn, nxt_ne):
        """first value above bucket ``b`` (next non-empty bucket of the window, else above it)."""
        n = int(nxt_ne[b + 1]) if b + 1 < NB else -1
        return float(_unskey_np(kmn[n])) if n >= 0 else st.after

    def _plan_gather(self) -> str:
        slots = sorted(self.slots)
        self.slots = slots
        self.slot_of = {cb: i for i, cb in enumerate(slots)}
        slot_arr = np.full((self.C, NB), -1, np.int32)
        for i, (c, b) in enumerate(slots):
            slot_arr[c, b] = i
        self.slot_t = torch.as_tensor(slot_arr, device=self.dev)
        lcnt = self.local_cnt.cpu().numpy()
        lens = np.array([lcnt[c, b] for c, b in slots], np.int64)
        self.local_lens = lens
        base = np.concatenate([[0], np.cumsum(lens)[:-1]]) if len(lens) else np.zeros(0, np.int64)
        self.sbase = torch.as_tensor(base.astype(np.int64), device=self.dev)
        M = int(lens.sum())
        self.gv = torch.empty(max(M, 1), dtype=torch.float64, device=self.dev)
        self.gq = torch.empty(max(M, 1), dtype=torch.int64, device=self.dev) if self.weighted else None
        self.scur = torch.zeros(max(len(slots), 1), dtype=torch.int32 if self.hip else torch.int64, device=self.dev)
        self.gcols = sorted({c for c, _ in slots})
        self.gcolmap = torch.as_tensor(np.asarray(self.gcols or [0], np.int32), device=self.dev)
        self.win = torch.as_tensor(np.ascontiguousarray(self.win_np ^ _I64_MIN if self.hip else self.win_np),
                                   device=self.dev)
        self.prm = torch.as_tensor(self.prm_np, device=self.dev)
        self.stage = "c"
        return "C" if slots else "done"

    # ---- pass C ------------------------------------------------------------------------------
    def pass_c(self, vals: torch.Tensor, y=None, w=None) -> None:
        n = self._check(vals, y, w)
        if n == 0 or not self.slots:
            return
        if self.hip:
            self._nat.call_hip("shifu_qgather", vals, vals.stride(0), n, self.C, y if self.sel_mode else None,
                               w if self.weighted else None, self.sel_mode, self.thr, self.gcolmap, len(self.gcols),
                               self.win, self.prm, self.wscale, self.slot_t, self.sbase, self.scur, self.gv, self.gq,
                               self._stream())
            return
        act = torch.as_tensor(self.gcols, device=vals.device)
        v = _clean(vals[act], self.thr)
        fin = torch.isfinite(v)
        vz = torch.where(fin, v, torch.zeros_like(v))
        k = skey(vz)
        win = self.win[act]
        sel = fin & _selmask(y, self.sel_mode, n, v.device)[None, :] & (k >= win[:, :1]) & (k <= win[:, 1:])
        b = _bucket(vz, self.prm[act, 0], self.prm[act, 1])
        s = torch.gather(self.slot_t[act].long(), 1, b)
        take = sel & (s >= 0)
        ss, vv = s[take], v[take]
        if ss.numel() == 0:
            return
        order = torch.argsort(ss, stable=True)
        ss, vv = ss[order], vv[order]
        cnts = torch.bincount(ss, minlength=len(self.slots))
        first = torch.cumsum(cnts, 0) - cnts
        pos = torch.arange(ss.numel(), device=v.device) - first[ss]
        at = self.sbase[ss] + self.scur[ss] + pos
        self.gv[at] = vv
        if self.weighted:
            q = torch.round(w[:n].clamp(min=0) * self.wscale).long()[None, :].expand(len(self.gcols), n)[take][order]
            self.gq[at] = q
        self.scur += cnts

    # ---- resolution --------------------------------------------------------------------------
    def finish(self):
        """-> (bounds list per column, distinct count of all finite values per column)."""
        dev = self.dev
        if self.slots:
            M = int(self.local_lens.sum())
            gv = self.gv[:M]
            seg = torch.repeat_interleave(torch.arange(len(self.slots), device=dev),
                                          torch.as_tensor(self.local_lens, device=dev))
            gq = self.gq[:M] if self.weighted else None
            if self.allgather is not None:
                gv, seg = self.allgather(gv), self.allgather(seg)
                gq = self.allgather(gq) if self.weighted else None
            o1 = torch.argsort(gv, stable=True)
            o2 = torch.argsort(seg[o1], stable=True)
            perm = o1[o2]
            V, SEG = gv[perm], seg[perm]
            P = torch.cumsum(gq[perm], 0) if self.weighted else None
            ar = torch.arange(len(self.slots), device=dev)
            seg_lo = torch.searchsorted(SEG, ar, right=False)
            seg_hi = torch.searchsorted(SEG, ar, right=True)
            is_start = torch.ones_like(SEG, dtype=torch.bool)
            if SEG.numel() > 1:
                is_start[1:] = (V[1:] != V[:-1]) | (SEG[1:] != SEG[:-1])
            slot_distinct = torch.bincount(SEG[is_start], minlength=len(self.slots)).cpu().numpy()
            q = []                                  # gathered targets: (c, j, slot, need, after)
            for c, st in enumerate(self.cols):
                if not st.gather:
                    continue
                if st.mode == AMBIG:
                    ids = [self.slot_of[(c, b)] for b, _, _ in st.gather]
                    d = len(st.outside) + st.singles.size + int(sum(slot_distinct[i] for i in ids))
                    st.distinct = d
                    if d <= self.nb:
                        vals = list(st.outside) + list(st.singles)
                        for i in ids:
                            vals += torch.unique_consecutive(V[int(seg_lo[i]):int(seg_hi[i])]).cpu().tolist()
                        st.mode, st.small = SMALL, np.sort(np.asarray(vals, np.float64))
                        continue
                    st.mode = EQPOP
                for b, tl, after in st.gather:
                    for j, nd in tl:
                        q.append((c, j, self.slot_of[(c, b)], nd, after))
            if q:
                sidx = torch.as_tensor([t[2] for t in q], device=dev)
                a, e = seg_lo[sidx], seg_hi[sidx]
                nd = torch.as_tensor([t[3] for t in q], dtype=torch.int64, device=dev)
                if self.weighted:
                    base = torch.where(a > 0, P[(a - 1).clamp(min=0)], torch.zeros_like(a))
                    i = _first_ge(P, base + nd, a, e)
                else:
                    i = torch.minimum(a + nd.clamp(min=1) - 1, e - 1)
                vi = V[i]
                jn = _first_gt(V, vi, i + 1, e)
                has = (jn < e).cpu().numpy()
                vin = vi.cpu().numpy()
                nv = V[jn.clamp(max=V.numel() - 1)].cpu().numpy()
                for t, (c, j, _, _, after) in enumerate(q):
                    self.cols[c].res[j] = (float(vin[t]), float(nv[t]) if has[t] else after)
        bounds, distinct = [], []
        for c, st in enumerate(self.cols):
            if self.interval or st.mode == INTERVAL:
                bounds.append(self._interval(c))
            elif st.mode == EMPTY:
                bounds.append([float("-inf")])
            elif st.mode == SMALL:
                u = st.small
                bounds.append([float("-inf")] + [float((u[i - 1] + u[i]) / 2.0) for i in range(1, u.size)])
            else:
                bl = [float("-inf")]
                for j in sorted(st.res):
                    v, nx = st.res[j]
                    if nx is None:
                        continue
                    bb = float((v + nx) / 2.0)
                    if bb > bl[-1]:
                        bl.append(bb)
                bounds.append(bl)
            distinct.append(self._distinct(c))
        return bounds, distinct

    def _interval(self, c):
        if self.scnt_np[c] == 0:
            return [float("-inf")]
        lo, hi = float(self.lo[c]), float(self.hi[c])
        if hi <= lo:
            return [float("-inf")]
        step = (hi - lo) / self.nb
        return [float("-inf")] + [lo + i * step for i in range(1, self.nb)]

    def _distinct(self, c) -> int:
        """Exact when every non-empty level-1 bucket holds one value (or the value set was
        resolved exactly); otherwise the HLL estimate, never below the bucket lower bound."""
        if not self.any_fin[c]:
            return 0
        if self.with_all:
            mn, mx = self.akmn_np[c], self.akmx_np[c]
            ne = mn <= mx
        else:
            st = self.cols[c]
            if st.distinct is not None:
                return int(st.distinct)
            if st.mode == SMALL:
                return int(st.small.size)
            cnt, mn, mx = self.h1
            mn, mx, ne = mn[c], mx[c], cnt[c] > 0
        multi = ne & (mn != mx)
        if not multi.any():
            return int(ne.sum())
        return max(int(ne.sum() + multi.sum()), int(round(hll_estimate(self.hll[c].cpu().numpy()))))


MAX_LEVEL = 4
GATHER_CAP = 1 << 18          # values per gathered bucket before a column refines instead


class _Col:
    """Per-column plan: mode, rank offset / first value above the current window, pending and
    resolved targets, known values outside the window (AMBIG), gathered buckets."""

    def __init__(self):
        self.mode = None
        self.off = 0
        self.after = None
        self.pending = []
        self.res = {}
        self.outside = []
        self.gather = []
        self.singles = np.zeros(0)
        self.small = None
        self.distinct = None
        self.done = False


def _mapping(lo: float, hi: float):
    """(lo, scale) of the 2048-bucket linear map; scale 0 puts everything in bucket 0."""
    if not (hi > lo):
        return lo, 0.0
    with np.errstate(all="ignore"):
        return lo, (NB / 2) / (hi / 2 - lo / 2)


def _next_nonempty(ne_mask: np.ndarray) -> np.ndarray:
    """index of the first non-empty bucket >= i (or -1)."""
    idx = np.where(ne_mask, np.arange(ne_mask.size), ne_mask.size)
    nxt = np.minimum.accumulate(idx[::-1])[::-1]
    return np.where(nxt >= ne_mask.size, -1, nxt)


def _first_ge(P: torch.Tensor, tgt: torch.Tensor, lo: torch.Tensor, hi: torch.Tensor) -> torch.Tensor:
    """per query: first i in [lo, hi) with P[i] >= tgt (P non-decreasing); hi - 1 if none."""
    lo, hi = lo.clone(), hi.clone()
    top = hi - 1
    for _ in range(64):
        act = lo < hi
        if not bool(act.any()):
            break
        mid = (lo + hi) // 2
        ge = P[mid.clamp(max=P.numel() - 1)] >= tgt
        hi = torch.where(act & ge, mid, hi)
        lo = torch.where(act & ~ge, mid + 1, lo)
    return torch.minimum(lo, top)


def _first_gt(V: torch.Tensor, v: torch.Tensor, lo: torch.Tensor, hi: torch.Tensor) -> torch.Tensor:
    """per query: first i in [lo, hi) with V[i] > v (V sorted in the range); hi if none."""
    lo, hi = lo.clone(), hi.clone()
    for _ in range(64):
        act = lo < hi
        if not bool(act.any()):
            break
        mid = (lo + hi) // 2
        gt = V[mid.clamp(max=V.numel() - 1)] > v
        hi = torch.where(act & gt, mid, hi)
        lo = torch.where(act & ~gt, mid + 1, lo)
    return lo


def column_cuts(vals: torch.Tensor, y, w, n_bins: int, method: str, binary: bool,
                num_thr: float = 1.7976931348623157e308, reduce=None, allgather=None):
    """One resident batch ``vals [C, n]`` -> (bounds, distinct), the reference rule including the
    class-restricted fallback (a cut with < 2 boundaries over the selected rows is redone over all
    rows, unweighted, when any row is unselected)."""
    sm = sel_mode_for(method, binary)
    eng = QuantileEngine(vals.shape[0], n_bins, sm, method.startswith("Weight"),
                         method in ("EqualInterval", "WeightEqualInterval"), num_thr, vals.device, reduce, allgather)
    run_passes(eng, [(vals, y, w)])
    bounds, distinct = eng.finish()
    if sm:
        nsel = _selmask(y, sm, vals.shape[1], vals.device).sum()
        partial = torch.tensor([float(vals.shape[1] - nsel)], dtype=torch.float64, device=vals.device)
        if reduce is not None:
            reduce(partial, "sum")
        redo = [c for c in range(vals.shape[0]) if len(bounds[c]) <= 1] if partial.item() > 0 else []
        if redo:
            sub = vals[redo]
            e2 = QuantileEngine(len(redo), n_bins, 0, False, False, num_thr, vals.device, reduce, allgather)
            run_passes(e2, [(sub, y, w)])
            b2, _ = e2.finish()
            for c, b in zip(redo, b2):
                bounds[c] = b
    return bounds, distinct


def run_passes(eng: QuantileEngine, chunks) -> None:
    """Drive the passes over a re-iterable sequence of (vals, y, w) chunks: A, then B once per
    refinement level, then C when values must be gathered."""
    for v, y, w in chunks:
        eng.pass_a(v, y, w)
    eng.finish_a()
    while True:
        for v, y, w in chunks:
            eng.pass_b(v, y, w)
        nxt = eng.finish_b()
        if nxt == "B":
            continue
        if nxt == "C":
            for v, y, w in chunks:
                eng.pass_c(v, y, w)
        return
