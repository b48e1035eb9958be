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
import weakref

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
        self.smom = torch.zeros(C, 2, dtype=torch.float64, device=dev)      # selected sum, sum of squares
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

    def _sel(self, y, n):
        """Packed selection bitmask of this chunk's rows for the kernels (None = every row)."""
        if not self.sel_mode:
            return None
        ref = getattr(self, "_sel_ref", None)
        if ref is None or ref[0]() is not y or ref[1] != n:       # weakref: no address aliasing
            from ..ops.stats_ops import pack_sel
            self._sel_bits = pack_sel(y[:n], self.sel_mode)
            self._sel_ref = (weakref.ref(y), n)
        return self._sel_bits

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
            self._nat.call_hip("shifu_qprep", vals, vals.stride(0), n, self.C, self._sel(y, n),
                               self.sel_mode, self.thr, self.mm, self.scnt, self.hll, self.smom, self._stream())
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
        vs = torch.where(sel, v, torch.zeros_like(v))
        self.smom[:, 0] += vs.sum(1)
        self.smom[:, 1] += (vs * vs).sum(1)
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
        self._red(self.smom, "sum")
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
        aprm = np.zeros((self.C, 2), np.float64)
        smom = self.smom.cpu().numpy()
        self.cols = [_Col() for _ in range(self.C)]
        for c in range(self.C):
            if self.any_fin[c]:
                aprm[c] = _lin_map(alo[c], ahi[c], NB)
            if self.scnt_np[c] > 0:
                n = float(self.scnt_np[c])
                with np.errstate(all="ignore"):
                    var = smom[c, 1] / n - (smom[c, 0] / n) ** 2
                    span = self.hi[c] - self.lo[c]
                    heavy = bool(np.isfinite(var) and np.isfinite(span) and span > HEAVY_RATIO * math.sqrt(max(var, 0.0)))
                self.cols[c].windows = [_Win(int(mm[c, 0]), int(mm[c, 1]), 0, NB, key=heavy)]
        self.aprm = torch.as_tensor(aprm, device=self.dev)
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
        self.active = [c for c in range(C) if self.any_fin[c]]
        self.slots = []                       # (column, bucket) gathered in pass C
        self._upload_windows()
        self.stage = "b"

    def _upload_windows(self):
        wptr = np.zeros(self.C + 1, np.int32)
        rows = []
        for c in range(self.C):
            ws = self.cols[c].windows
            wptr[c + 1] = wptr[c] + len(ws)
            rows += [w.record() for w in ws]
        self.wptr_np = wptr
        self.wins_np = rows
        if self.hip:
            arr = np.zeros(max(len(rows), 1), dtype=_QWIN)
            for i, r in enumerate(rows):
                arr[i] = (r[0] + (1 << 63), r[1] + (1 << 63), r[2], r[3], r[4], (r[5] + (1 << 63)) & ((1 << 64) - 1),
                          r[6], r[7])
            self.wins = torch.as_tensor(np.frombuffer(arr.tobytes(), np.uint8).copy(), device=self.dev)
            self.wptr = torch.as_tensor(wptr, device=self.dev)
        self.colmap = torch.as_tensor(np.asarray(self.active or [0], np.int32), device=self.dev)

    # ---- pass B ------------------------------------------------------------------------------
    def pass_b(self, vals: torch.Tensor, y=None, w=None) -> None:
        n = self._check(vals, y, w)
        if n == 0 or not self.active:
            return
        with_all = self.with_all and self.level == 1
        if self.hip:
            self._nat.call_hip("shifu_qhist", vals, vals.stride(0), n, self.C, self._sel(y, n),
                               w if self.weighted else None, self.sel_mode, self.thr, self.colmap, len(self.active),
                               self.wptr, self.wins, self.aprm, self.wscale, int(with_all), self.cnt, self.wq,
                               self.kmn, self.kmx, self.akmn, self.akmx, self._stream())
            return
        sm = _selmask(y, self.sel_mode, n, vals.device)
        q_all = torch.round(w[:n].clamp(min=0) * self.wscale).long() if self.weighted else None
        for c in self.active:
            v = _clean(vals[c], self.thr)
            fin = torch.isfinite(v)
            vz = torch.where(fin, v, torch.zeros_like(v))
            k = skey(vz)
            sel = fin & sm
            b = self._win_buckets(c, vz, k, sel)
            take = b >= 0
            bs, ks = b[take] + c * NB, k[take]
            self.cnt.view(-1).scatter_add_(0, bs, torch.ones_like(bs))
            self.kmn.view(-1).scatter_reduce_(0, bs, ks, reduce="amin")
            self.kmx.view(-1).scatter_reduce_(0, bs, ks, reduce="amax")
            if self.weighted:
                self.wq.view(-1).scatter_add_(0, bs, q_all[take])
            if with_all:
                ab = _bucket(vz[None, :], self.aprm[c:c + 1, 0], self.aprm[c:c + 1, 1])[0] + c * NB
                self.akmn.view(-1).scatter_reduce_(0, ab[fin], k[fin], reduce="amin")
                self.akmx.view(-1).scatter_reduce_(0, ab[fin], k[fin], reduce="amax")

    def _win_buckets(self, c, vz, k, sel):
        """torch twin of the kernels' win_bucket: bucket index per row (-1 outside every window)."""
        out = torch.full_like(k, -1)
        for w in self.cols[c].windows:
            m = sel & (k >= w.lo_key) & (k <= w.hi_key)
            if not bool(m.any()):
                continue
            if w.msh < 0:
                f = (vz[m] - w.mlo) * w.msc
                f = torch.nan_to_num(f, nan=0.0, posinf=float(w.size), neginf=0.0)
                b = torch.where(f <= 0, torch.zeros_like(f),
                                torch.where(f >= w.size - 1, torch.full_like(f, w.size - 1), f)).long()
            else:
                d = k[m] - w.mklo
                q = torch.bitwise_right_shift(d, w.msh)
                if w.msh > 0:
                    q = q & ((1 << (64 - w.msh)) - 1)
                b = torch.where((q < 0) | (q > w.size - 1), torch.full_like(q, w.size - 1), q)
            out[m] = w.base + b
        return out

    def finish_b(self) -> str:
        """Merge this level's histograms and plan every active column: returns "B" when some
        column refines into narrower windows (another pass B), "C" when values must be gathered,
        "done" otherwise."""
        if self.hip:
            for t in (self.kmn, self.kmx) + ((self.akmn, self.akmx) if self.with_all and self.level == 1 else ()):
                t ^= _I64_MIN
        idx = self.active_t()
        if self.level == 1:
            self.local_cnt = self.cnt.clone()
        else:
            self.local_cnt[idx] = self.cnt[idx]
        if self.reduce is not None:       # merge only this level's rows (finished rows are merged)
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
        cnt = self.cnt.cpu().numpy()
        rank = self.wq.cpu().numpy() if self.weighted else cnt
        kmn, kmx = self.kmn.cpu().numpy(), self.kmx.cpu().numpy()
        if self.level == 1:
            self.h1 = (cnt.copy(), kmn.copy(), kmx.copy())
        refine = [c for c in self.active if self._plan(c, cnt[c], rank[c], kmn[c], kmx[c])]
        # keep the gather (one device sort of every gathered value) within budget: the columns
        # with the largest gathers refine instead (one more histogram pass over those columns)
        gathering = sorted((c for c in self.active if c not in refine and self.cols[c].gather
                            and self.can_refine(self.cols[c])), key=lambda c: -self.cols[c].gather_size)
        total = sum(self.cols[c].gather_size for c in self.active if self.cols[c].gather)
        for c in gathering:
            if total <= GATHER_BUDGET:
                break
            st = self.cols[c]
            total -= st.gather_size
            self.slots = [sb for sb in self.slots if sb[0] != c]
            st.gather, st.singles = [], np.zeros(0)
            self._refine(st)
            refine.append(c)
        if refine:
            refine.sort()
            self.level += 1
            self.active = refine
            ridx = torch.as_tensor(refine, device=self.dev)
            self.cnt[ridx] = 0
            if self.weighted:
                self.wq[ridx] = 0
            if self.hip:      # kernels keep unsigned patterns: reset refined rows, re-flip finished ones
                keep = torch.ones(self.C, dtype=torch.bool, device=self.dev)
                keep[ridx] = False
                self.kmn[keep] ^= _I64_MIN
                self.kmx[keep] ^= _I64_MIN
            self.kmn[ridx] = self._init_mn
            self.kmx[ridx] = self._init_mx
            self._upload_windows()
            return "B"
        self.active = []
        return self._plan_gather()

    def active_t(self):
        return torch.as_tensor(self.active, device=self.dev)

    def _plan(self, c, cnt, rank, kmn, kmx) -> bool:
        """One level of column ``c`` over its windows; True when it refines further."""
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
            st.windows[0].targets = [(j, -((-j * T) // nb)) for j in range(1, nb)]   # ceil(j*T/nb), exact
            if mu == 0 and ne <= nb:
                st.mode, st.small = SMALL, _unskey_np(kmn[ne_mask])
                return False
            st.mode = EQPOP if ne + mu > nb else AMBIG
        if st.mode == AMBIG:              # small vs equal-population once the distinct count is known
            if len(st.outside) + ne + mu > nb:
                st.mode = EQPOP
            elif mu == 0:
                st.small = np.sort(np.concatenate([np.asarray(st.outside, np.float64), _unskey_np(kmn[ne_mask])]))
                st.distinct = int(st.small.size)
                if st.small.size <= nb:
                    st.mode = SMALL
                    return False
                st.mode = EQPOP
        pend = []                         # (bucket, targets [(j, s, need)], off, after)
        singles = []
        for win in st.windows:
            lo, hi = win.base, win.base + win.size
            cum = win.off + np.cumsum(rank[lo:hi])
            nem = ne_mask[lo:hi]
            nxt = _next_nonempty(nem)
            by_b = {}
            for j, s in win.targets:
                b = min(int(np.searchsorted(cum, s, side="left")), win.size - 1)
                if not nem[b]:
                    b = int(nxt[b])
                    if b < 0:
                        continue
                if not multi[lo + b]:
                    st.res[j] = (float(_unskey_np(kmn[lo + b])), _after(nxt, b, kmn[lo:hi], win.after))
                else:
                    by_b.setdefault(b, []).append((j, s))
            bs = sorted(by_b)
            if st.mode == AMBIG:
                bs = [int(b) for b in np.nonzero(multi[lo:hi])[0]]
                singles += list(_unskey_np(kmn[lo:hi][nem & ~multi[lo:hi]]))
            for b in bs:
                off = int(cum[b - 1]) if b > 0 else win.off
                pend.append((lo + b, by_b.get(b, []), off, _after(nxt, b, kmn[lo:hi], win.after)))
        if not pend:
            return False
        st.pend, st.pend_singles = pend, singles
        st.pend_kmn, st.pend_kmx = kmn, kmx
        st.gather_size = int(sum(cnt[b] for b, _, _, _ in pend))
        big = int(max(cnt[b] for b, _, _, _ in pend)) > GATHER_CAP
        if big and self.can_refine(st):
            self._refine(st)
            return True
        # final level: gather the pending buckets
        st.gather = [(b, [(j, s - off) for j, s in tg], after) for b, tg, off, after in pend]
        st.singles = np.asarray(singles, np.float64)
        self.slots += [(c, b) for b, _, _, _ in pend]
        return False

    def can_refine(self, st) -> bool:
        return self.level < MAX_LEVEL and len(st.pend) <= MAX_WINDOWS

    def _refine(self, st) -> None:
        """Every pending bucket becomes a window of the next level (sharing the 2048 buckets)."""
        pend, kmn, kmx = st.pend, st.pend_kmn, st.pend_kmx
        size = NB // len(pend)
        if st.mode == AMBIG:
            st.outside += st.pend_singles
        st.windows = []
        for i, (b, tg, off, after) in enumerate(pend):
            wlo, whi = float(_unskey_np(kmn[b])), float(_unskey_np(kmx[b]))
            w = _Win(int(kmn[b]), int(kmx[b]), i * size, size, key=_spans_binades(wlo, whi))
            w.off, w.after, w.targets = off, after, tg
            st.windows.append(w)

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
        self.active = self.gcols
        self._upload_windows()
        self.active = []
        self.gcolmap = torch.as_tensor(np.asarray(self.gcols or [0], np.int32), device=self.dev)
        self.two_phase = M > TWO_PHASE_GATHER
        self.stage = "c"
        return "C" if slots else "done"

    # ---- pass C ------------------------------------------------------------------------------
    def pass_c(self, vals: torch.Tensor, y=None, w=None) -> None:
        n = self._check(vals, y, w)
        if n == 0 or not self.slots:
            return
        if self.hip:
            self._nat.call_hip("shifu_qgather", vals, vals.stride(0), n, self.C, self._sel(y, n),
                               w if self.weighted else None, self.sel_mode, self.thr, self.gcolmap, len(self.gcols),
                               self.wptr, self.wins, self.wscale, self.slot_t, self.sbase, self.scur, self.gv,
                               self.gq, int(self.two_phase), self._stream())
            return
        sm = _selmask(y, self.sel_mode, n, vals.device)
        q_all = torch.round(w[:n].clamp(min=0) * self.wscale).long() if self.weighted else None
        for c in self.gcols:
            v = _clean(vals[c], self.thr)
            fin = torch.isfinite(v)
            vz = torch.where(fin, v, torch.zeros_like(v))
            b = self._win_buckets(c, vz, skey(vz), fin & sm)
            s = torch.where(b >= 0, self.slot_t[c].long()[b.clamp(min=0)], torch.full_like(b, -1))
            take = s >= 0
            ss, vv = s[take], v[take]
            if ss.numel() == 0:
                continue
            order = torch.argsort(ss, stable=True)
            ss, vv = ss[order], vv[order]
            cnts = torch.bincount(ss, minlength=len(self.slots))
            first = torch.cumsum(cnts, 0) - cnts
            pos = torch.arange(ss.numel(), device=v.device) - first[ss]
            at = self.sbase[ss] + self.scur[ss] + pos
            self.gv[at] = vv
            if self.weighted:
                self.gq[at] = q_all[take][order]
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
            # segmented sort: one sort by (slot, value) through the order-preserving key
            key = skey(gv)
            o1 = torch.argsort(key)
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
            elif st.mode in (EMPTY, None):
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
MAX_WINDOWS = 128             # windows per column (MAXW in quantile_kernels.hip)
GATHER_CAP = 1 << 17          # values per gathered bucket before a column refines instead
GATHER_BUDGET = 4 << 20       # gathered values per engine (batch) before the largest refine
TWO_PHASE_GATHER = 1 << 24    # above this many gathered values qgather reserves per block
HEAVY_RATIO = 64.0            # range > 64 sigma: bucket in key space (heavy tails)

_QWIN = np.dtype([("lo", "<u8"), ("hi", "<u8"), ("mlo", "<f8"), ("msc", "<f8"), ("msh", "<i8"), ("mklo", "<u8"),
                  ("base", "<i4"), ("size", "<i4")])
assert _QWIN.itemsize == 56


class _Win:
    """A key window [lo_key, hi_key] (signed keys) of one column mapped onto ``size`` buckets at
    ``base``: linear in value, or in key space (heavy tails / windows spanning binades)."""

    def __init__(self, lo_key: int, hi_key: int, base: int, size: int, key: bool = False):
        self.lo_key, self.hi_key, self.base, self.size = int(lo_key), int(hi_key), int(base), int(size)
        lo, hi = float(_unskey_np(np.int64(lo_key))), float(_unskey_np(np.int64(hi_key)))
        if key:
            self.msh, self.mklo = ((max(hi_key - lo_key, 0) // self.size).bit_length(), self.lo_key)
            self.mlo, self.msc = 0.0, 0.0
        else:
            self.msh, self.mklo = -1, 0
            self.mlo, self.msc = _lin_map(lo, hi, self.size)
        self.off = 0
        self.after = None
        self.targets = []

    def record(self):
        return (self.lo_key, self.hi_key, self.mlo, self.msc, self.msh, self.mklo, self.base, self.size)


class _Col:
    """Per-column plan: mode, windows of the current level, resolved targets, values known
    outside the windows (AMBIG), gathered buckets."""

    def __init__(self):
        self.mode = None
        self.windows = []
        self.res = {}
        self.outside = []
        self.gather = []
        self.singles = np.zeros(0)
        self.small = None
        self.distinct = None
        self.pend = []
        self.gather_size = 0


def _lin_map(lo: float, hi: float, size: int):
    """(lo, scale) of a ``size``-bucket linear map; scale 0 puts everything in bucket 0."""
    if not (hi > lo):
        return lo, 0.0
    with np.errstate(all="ignore"):
        return lo, (size / 2) / (hi / 2 - lo / 2)


def _after(nxt, b, kmn_w, outer):
    """First value above bucket ``b`` of a window: the next non-empty bucket's min, else the
    window's own ``after`` (the first value above the window)."""
    n = int(nxt[b + 1]) if b + 1 < nxt.size else -1
    return float(_unskey_np(kmn_w[n])) if n >= 0 else outer


def _spans_binades(lo: float, hi: float) -> bool:
    """A refinement window worth bucketing in key space: one sign and > 2^10 magnitude ratio (a
    window straddling 0 stays linear: in key space the values near 0 would own most buckets)."""
    if lo < 0.0 < hi:
        return False
    a, b = sorted((abs(lo), abs(hi)))
    return b > 1024.0 * max(a, 1e-300)


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
