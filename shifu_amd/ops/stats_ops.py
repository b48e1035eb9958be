"""Python side of ``stats_kernels.hip`` (K1/K2/K5/K9/K14): packs per-column parameters,
launches the HIP kernels on the current stream and unpacks results.  Every function here
requires the native library (``_native.require_gpu_native``) — there is no silent fallback;
callers choose the CPU oracle explicitly when no GPU is present."""
from __future__ import annotations

import math

import numpy as np
import torch

from . import _native as nat

NM = {"zscore": 0, "num_table": 1, "cat_table": 2, "raw": 3, "discrete": 4, "cat_index": 5}


def _dev_tensor(a, dtype, dev):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype).to(dev)


def pack_bits(mask: torch.Tensor) -> torch.Tensor:
    """bool [n] -> int32 words, bit r of word r // 32 = mask[r] (the kernels' row bitmasks)."""
    n = mask.numel()
    m = torch.zeros(((n + 31) // 32) * 32, dtype=torch.int64, device=mask.device)
    m[:n] = mask.reshape(-1).to(torch.int64)
    words = (m.view(-1, 32) << torch.arange(32, device=mask.device, dtype=torch.int64)).sum(1)
    return torch.where(words >= (1 << 31), words - (1 << 32), words).to(torch.int32)


def pack_sel(y: torch.Tensor, mode: int) -> torch.Tensor:
    """Row bitmask of ``y > 0.5`` (mode 1) or its complement (mode 2): the HIP ballot kernel on the
    GPU, :func:`pack_bits` on the CPU."""
    n = y.numel()
    if y.device.type != "cuda":
        m = y.reshape(-1) > 0.5
        return pack_bits(m if mode == 1 else ~m)
    out = torch.empty((n + 31) // 32 + 1, dtype=torch.int32, device=y.device)
    yf = y.reshape(-1)
    if yf.dtype != torch.float32 or not yf.is_contiguous():
        yf = yf.float().contiguous()
    nat.call_hip("shifu_pack_bits", yf, n, int(mode), out, nat.stream_of(yf))
    return out


def pack_bounds(bounds_list):
    offs = [0]
    flat = []
    for b in bounds_list:
        b = list(b) if b is not None and len(b) else [float("-inf")]
        flat.extend(float(x) for x in b)
        offs.append(len(flat))
    return np.asarray(flat if flat else [0.0], np.float64), np.asarray(offs, np.int32)


def column_stats(vals: torch.Tensor, y: torch.Tensor, w: torch.Tensor, bounds_list, binary: bool,
                 num_thr: float = 1.7976931348623157e308, nchunks: int | None = None):
    """vals [F, N] fp64 (column-major) on the GPU -> per column (cpos, cneg, wpos, wneg) numpy
    arrays of length nb+1 (missing bin last) and moments (count, s1..s4, min, max)."""
    nat.require_gpu_native()
    F, N = vals.shape
    dev = vals.device
    bflat, boff = pack_bounds(bounds_list)
    max_nb = int(np.max(np.diff(boff))) if F else 1
    if max_nb > 1024:
        raise ValueError("column_stats: more than 1024 bin boundaries per column")
    hstride = max_nb + 1
    wmax = float(w.abs().max().item()) if N else 1.0
    wscale = 2.0 ** min(40, math.floor(62 - math.log2(max(wmax, 1e-30) * max(N, 1))))
    nchunks = nchunks or max(1, min(256, (N + 65535) // 65536))
    hist = torch.zeros(F * hstride * 4, dtype=torch.int64, device=dev)
    part = torch.zeros(F * nchunks * 8, dtype=torch.float64, device=dev)
    bt, ot = _dev_tensor(bflat, torch.float64, dev), _dev_tensor(boff, torch.int32, dev)
    unit_w = bool(N) and bool(torch.all(w[:N] == 1.0).item())
    posbits = pack_sel(y[:N], 1) if binary else None
    rc = nat.call_hip("shifu_column_stats", vals, vals.stride(0), y, w, N, F, bt, ot, max_nb, int(binary), wscale,
                      float(num_thr), hist, hstride, part, nchunks, int(unit_w), posbits, nat.stream_of(vals))
    if rc:
        raise RuntimeError(f"shifu_column_stats failed rc={rc}")
    h = hist.view(F, hstride, 4).cpu().numpy()
    p = part.view(F, nchunks, 8).cpu().numpy()
    out = []
    for f in range(F):
        nb = int(boff[f + 1] - boff[f])
        hh = h[f, : nb + 1]
        mom = (int(p[f, :, 0].sum()), float(p[f, :, 1].sum()), float(p[f, :, 2].sum()), float(p[f, :, 3].sum()),
               float(p[f, :, 4].sum()), float(p[f, :, 5].min()), float(p[f, :, 6].max()))
        if mom[0] == 0:
            mom = (0, 0.0, 0.0, 0.0, 0.0, float("nan"), float("nan"))
        out.append((hh[:, 0].astype(np.int64), hh[:, 1].astype(np.int64), hh[:, 2] / wscale, hh[:, 3] / wscale, mom))
    return out


def column_stats_multi(vals_list, y: torch.Tensor, w: torch.Tensor, bounds_lists, binary: bool,
                       num_thr: float = 1.7976931348623157e308, bounds_cache: dict | None = None):
    """:func:`column_stats` for several column batches of ONE row chunk (the streamed stats pass D):
    the weight scale, unit-weight test and positive-row bitmask are computed once, every batch's
    kernel is launched back to back and all histograms / moment partials come back in two D2H
    copies -- per chunk 3 host syncs instead of 4 per 64-column batch.  ``bounds_cache`` keeps the
    batches' packed boundaries on the device across chunks.  -> per batch (counts [F, hs, 2] int64
    (pos, neg), weight sums [F, hs, 2] fp64, moments [F, 7] (count, s1..s4, min, max), bin offsets):
    column_stats' values as arrays (no per-column Python work)."""
    nat.require_gpu_native()
    if not vals_list:
        return []
    N = vals_list[0].shape[1]
    dev = vals_list[0].device
    if N:
        hw = torch.stack([w[:N].abs().max().double(), torch.all(w[:N] == 1.0).double()]).cpu().numpy()
        wmax, unit_w = float(hw[0]), bool(hw[1])
    else:
        wmax, unit_w = 1.0, False
    wscale = 2.0 ** min(40, math.floor(62 - math.log2(max(wmax, 1e-30) * max(N, 1))))
    nchunks = max(1, min(256, (N + 65535) // 65536))
    posbits = pack_sel(y[:N], 1) if binary else None
    hists, parts, metas = [], [], []
    for vals, bounds_list in zip(vals_list, bounds_lists):
        F = vals.shape[0]
        hit = bounds_cache.get(id(bounds_list)) if bounds_cache is not None else None
        if hit is None or hit[0] is not bounds_list:
            bflat, boff = pack_bounds(bounds_list)
            max_nb = int(np.max(np.diff(boff))) if F else 1
            if max_nb > 1024:
                raise ValueError("column_stats: more than 1024 bin boundaries per column")
            hit = (bounds_list, boff, max_nb, _dev_tensor(bflat, torch.float64, dev), _dev_tensor(boff, torch.int32, dev))
            if bounds_cache is not None:
                bounds_cache[id(bounds_list)] = hit
        _, boff, max_nb, bt, ot = hit
        hstride = max_nb + 1
        hist = torch.zeros(F * hstride * 4, dtype=torch.int64, device=dev)
        part = torch.zeros(F * nchunks * 8, dtype=torch.float64, device=dev)
        rc = nat.call_hip("shifu_column_stats", vals, vals.stride(0), y, w, N, F, bt, ot, max_nb, int(binary), wscale,
                          float(num_thr), hist, hstride, part, nchunks, int(unit_w), posbits, nat.stream_of(vals))
        if rc:
            raise RuntimeError(f"shifu_column_stats failed rc={rc}")
        hists.append(hist)
        parts.append(part)
        metas.append((F, hstride, boff))
    H = torch.cat(hists).cpu().numpy()
    P = torch.cat(parts).cpu().numpy()
    res, ho, po = [], 0, 0
    for F, hstride, boff in metas:
        h = H[ho: ho + F * hstride * 4].reshape(F, hstride, 4)
        p = P[po: po + F * nchunks * 8].reshape(F, nchunks, 8)
        ho += F * hstride * 4
        po += F * nchunks * 8
        mom = np.empty((F, 7), np.float64)
        for k in range(5):
            mom[:, k] = p[:, :, k].sum(1)
        mom[:, 5] = p[:, :, 5].min(1)
        mom[:, 6] = p[:, :, 6].max(1)
        mom[mom[:, 0] == 0] = (0, 0.0, 0.0, 0.0, 0.0, np.nan, np.nan)
        res.append((h[:, :, :2].astype(np.int64), h[:, :, 2:4] / wscale, mom, boff))
    return res


def normalize(vals: torch.Tensor, specs: list, out: torch.Tensor):
    """vals [F, N] fp64; specs[f] = dict(mode, out_col, bounds, table, mean, std, cutoff, zflag,
    zmean, zstd); out [N, ldo] fp32 (written in place)."""
    nat.require_gpu_native()
    F, N = vals.shape
    dev = vals.device
    ip = np.zeros((F, 8), np.int32)
    dp = np.zeros((F, 8), np.float64)
    bounds, tables = [], []
    for f, s in enumerate(specs):
        b = list(s.get("bounds") or [float("-inf")])
        t = list(s.get("table") or [0.0])
        nt = int(s["ncat"]) if s["mode"] == "cat_index" else len(t)
        ip[f] = [NM[s["mode"]], s["out_col"], len(bounds), len(b), len(tables), nt, int(s.get("zflag", 0)), 0]
        bounds.extend(b)
        tables.extend(t)
        dp[f, :5] = [s.get("mean", 0.0) or 0.0, s.get("std", 0.0) or 0.0, s.get("cutoff", 6.0),
                     s.get("zmean", 0.0) or 0.0, s.get("zstd", 0.0) or 0.0]
    rc = nat.call_hip("shifu_normalize", vals, vals.stride(0), N, F, _dev_tensor(ip, torch.int32, dev),
                      _dev_tensor(dp, torch.float64, dev), _dev_tensor(np.asarray(bounds, np.float64), torch.float64, dev),
                      _dev_tensor(np.asarray(tables, np.float64), torch.float64, dev), out, out.stride(0),
                      nat.stream_of(vals))
    if rc:
        raise RuntimeError(f"shifu_normalize failed rc={rc}")
    return out


def bin_codes(vals: torch.Tensor, is_cat, bounds_list, ncat, out: torch.Tensor):
    """Tree bin codes uint8 [N, ldo] from column-major fp64 values."""
    nat.require_gpu_native()
    F, N = vals.shape
    dev = vals.device
    bflat, boff = pack_bounds(bounds_list)
    ip = np.zeros((F, 4), np.int32)
    for f in range(F):
        ip[f] = [int(is_cat[f]), boff[f], boff[f + 1] - boff[f], int(ncat[f])]
    rc = nat.call_hip("shifu_bin_codes", vals, vals.stride(0), N, F, _dev_tensor(ip, torch.int32, dev),
                      _dev_tensor(bflat, torch.float64, dev), out, out.stride(0), nat.stream_of(vals))
    if rc:
        raise RuntimeError(f"shifu_bin_codes failed rc={rc}")
    return out


def lr_grad(x: torch.Tensor, w: torch.Tensor, y: torch.Tensor, s: torch.Tensor | None, nblk: int = 1024):
    """Fused LR gradient pass -> (grad [F+1] fp32 (ascent, bias last), sum squared error)."""
    nat.require_gpu_native()
    n, ldx = x.shape[0], x.stride(0)
    F = w.numel() - 1
    dtype = 1 if x.dtype == torch.bfloat16 else 0
    lim = 4096 if dtype else 2048
    if F > lim or ldx % (8 if dtype else 4):
        return None
    nblk = max(1, min(nblk, (n + 3) // 4))
    part = torch.empty(nblk, F + 1, dtype=torch.float32, device=x.device)
    ep = torch.empty(nblk, dtype=torch.float64, device=x.device)
    rc = nat.call_hip("shifu_lr_grad", x, ldx, n, F, dtype, w, y, s, part, ep, nblk, nat.stream_of(x))
    if rc:
        raise RuntimeError(f"shifu_lr_grad failed rc={rc}")
    return part.sum(0), ep.sum()


def rowdot(x: torch.Tensor, w: torch.Tensor, b: float = 0.0, act_out: int = -1) -> torch.Tensor:
    """act_out(x [n, k] @ w [k] + b) on the own row-dot kernels (bf16 or fp32 rows; fp32 out)."""
    nat.require_gpu_native()
    n, k = x.shape
    out = torch.empty(n, dtype=torch.float32, device=x.device)
    w = w.float().contiguous()
    if x.dtype == torch.bfloat16:
        nat.call_hip("shifu_rowdot_bf16", x, x.stride(0), n, k, w, out, nat.stream_of(x))
        if b or act_out >= 0:
            from ..models.nn import ACT_IDS, act_fwd
            out = out + b
            if act_out >= 0:
                out = act_fwd({v: kk for kk, v in ACT_IDS.items()}[act_out], out)
    else:
        nat.call_hip("shifu_rowdot_f32_act", x.float(), x.stride(0), n, k, w, float(b), -1, act_out, out,
                     nat.stream_of(x))
    return out


def coldot(d: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """sum_i d[i] x[i, :] -> [k] fp32 (per-256-row partials, fixed-order sum: deterministic)."""
    nat.require_gpu_native()
    n, k = x.shape
    part = torch.empty(max(1, -(-n // 256)) * k, dtype=torch.float32, device=x.device)
    out = torch.empty(k, dtype=torch.float32, device=x.device)
    d = d.float().contiguous()
    name = "shifu_coldot_bf16" if x.dtype == torch.bfloat16 else "shifu_coldot_f32"
    nat.call_hip(name, d, x, x.stride(0), n, k, part, out, nat.stream_of(x))
    return out


def se_perturb(S: torch.Tensor, X: torch.Tensor, W1t: torch.Tensor, f0: int, fc: int, act: int, hpad: int,
               out: torch.Tensor | None = None) -> torch.Tensor:
    """Perturbed first hidden layer of every (row, input in [f0, f0+fc)) pair as bf16 MLP rows
    [R*fc, hpad] (bias column = 1) for the MFMA tail of deep-net SE (K14b)."""
    nat.require_gpu_native()
    R, H = S.shape
    F = X.shape[1]
    if out is None:
        out = torch.empty(R * fc, hpad, dtype=torch.bfloat16, device=S.device)
    nat.call_hip("shifu_se_perturb", S, S.stride(0), X, X.stride(0), W1t, int(f0), int(fc), F, H, int(hpad),
                 int(act), out, R, nat.stream_of(S))
    return out


def sensitivity_1h(S: torch.Tensor, X: torch.Tensor, W1t: torch.Tensor, W2: torch.Tensor, b2: float,
                   base: torch.Tensor, act1: int, act_o: int, acc: torch.Tensor, nchunks: int | None = None):
    """Accumulate sum|d| and sum d^2 per input into ``acc`` [F, 2] fp64 (1-hidden-layer nets)."""
    nat.require_gpu_native()
    n, H = S.shape
    F = X.shape[1]
    if not nchunks:                     # >= ~2048 blocks over (row chunks x 32-input groups)
        fblocks = (F + 31) // 32                   # SFT = 32 inputs per block
        nchunks = max(1, min((n + 63) // 64, -(-2048 // fblocks)))
    rc = nat.call_hip("shifu_sensitivity", S, S.stride(0), X, X.stride(0), W1t, W2, float(b2), base, n, F, H,
                      int(act1), int(act_o), nchunks, acc, nat.stream_of(S))
    if rc:
        raise RuntimeError(f"shifu_sensitivity failed rc={rc}")
    return acc


def keyed_hist(keys: torch.Tensor, K: int, weights: torch.Tensor | None = None):
    """Keyed counts (K17 PSI (unit, bin) counts, K18 post-train per-bin score sums) through
    ``scoring_kernels.hip: keyed_hist_kernel``.

    keys [F, N] or [N] int (rows with key < 0 or >= K are skipped; a 1-D key vector is shared by
    every column of ``weights``); weights None, [N] (shared) or [F, N] fp64.
    -> (counts [F, K] fp64, weighted sums [F, K] fp64 | None).  Weighted sums are accumulated as
    int64 fixed point (scale from max |w| and N), so they are order-independent: identical run to
    run and to a fixed-point host sum."""
    nat.require_gpu_native()
    dev = keys.device
    shared_keys = keys.dim() == 1
    N = keys.shape[-1]
    F = 1 if shared_keys and (weights is None or weights.dim() == 1) else \
        (weights.shape[0] if shared_keys else keys.shape[0])
    k = keys.to(torch.int32).contiguous()
    ks = 0 if shared_keys else N
    w, ws, scale = None, 0, 0.0
    if weights is not None:
        w = weights.to(device=dev, dtype=torch.float64).contiguous()
        ws = 0 if w.dim() == 1 else N
        amax = float(w.abs().max()) if w.numel() else 0.0
        if amax > 0:
            # |sum| <= N * amax < 2^62  ->  scale = 2^(62 - ceil(log2(N * amax)))
            scale = math.ldexp(1.0, 62 - max(1, math.ceil(math.log2(max(N, 1) * amax))))
    cnt = torch.zeros(F, K, dtype=torch.int64, device=dev)
    wsum = torch.zeros(F, K, dtype=torch.int64, device=dev) if w is not None else None
    if N and K:
        nat.call_hip("shifu_keyed_hist", k, ks, w, ws, N, F, int(K), scale, cnt, wsum, nat.stream_of(k))
    c = cnt.to(torch.float64)
    if wsum is None:
        return c, None
    return c, (wsum.to(torch.float64) / scale if scale else torch.zeros_like(c))


def column_metrics_batch(negs, poss, dev):
    """K3 for many columns in one launch (``stats_kernels.hip: column_metrics_kernel``).

    negs / poss: per column a pair (counts, weighted) of equal-length bin arrays.
    -> per column ((ks*100, iv, woe, bin_woe) | None, same for the weighted bins)."""
    nat.require_gpu_native()
    F = len(negs)
    if F == 0:
        return []
    lens = [len(n[0]) for n in negs]
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    total = int(off[-1])
    hn = np.zeros((2, max(1, total)))
    hp = np.zeros((2, max(1, total)))
    for k in range(F):
        for v in range(2):
            hn[v, off[k]:off[k + 1]] = negs[k][v]
            hp[v, off[k]:off[k + 1]] = poss[k][v]
    dn, dp = _dev_tensor(hn, torch.float64, dev), _dev_tensor(hp, torch.float64, dev)
    doff = _dev_tensor(off, torch.int32, dev)
    out = torch.zeros(F, 2, 4, dtype=torch.float64, device=dev)
    bw = torch.zeros(2, max(1, total), dtype=torch.float64, device=dev)
    nat.call_hip("shifu_column_metrics", dn, dp, doff, F, max(1, total), out, bw, nat.stream_of(dn))
    out, bw = out.cpu().numpy(), bw.cpu().numpy()
    res = []
    for k in range(F):
        pair = []
        for v in range(2):
            o = out[k, v]
            pair.append((float(o[0]), float(o[1]), float(o[2]), [float(x) for x in bw[v, off[k]:off[k + 1]]])
                        if o[3] > 0 else None)
        res.append(tuple(pair))
    return res


def sort_desc(x: torch.Tensor) -> torch.Tensor:
    """K16: stable descending order of fp64 scores on the device (hand-written LSD radix sort,
    ops/csrc/sort_kernels.hip): int32 row ids, ties in row order, NaN last."""
    nat.require_gpu_native()
    x = x.to(torch.float64).contiguous()
    n = x.numel()
    order = torch.empty(n, dtype=torch.int32, device=x.device)
    if n == 0:
        return order
    ws = torch.empty(int(nat.hip().shifu_sort_ws(n)), dtype=torch.uint8, device=x.device)
    rc = nat.call_hip("shifu_sort_desc", x, n, order, ws, nat.stream_of(x))
    if rc:
        raise RuntimeError(f"shifu_sort_desc failed rc={rc}")
    return order
