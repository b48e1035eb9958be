"""Normalization (H7) and tree-input binning (CleanedData).

All 22 ``NormType``s of ``J/core/Normalizer.java`` (normalize :233-333, zScoreNormalize :444,
parseRawValue :522-577, woeNormalize :619-648, woeZScoreNormalize :664, calculateWoeMeanAndStdDev
:728-754, computeZScore :769-785), vectorized per column over the purified table:

* ZSCALE/ZSCORE: numeric value (missing/invalid/inf -> mean), clipped to mean +- cutoff*std,
  then (v-mean)/std (std <= 1e-5 -> 0); categorical -> bin pos-rate (missing/unknown -> last
  bin's pos rate) then z-scored.  OLD_*: categorical pos-rate not z-scored.
* WOE / WEIGHT_WOE: bin WOE (missing -> last bin).  *_WOE_ZSCORE: z-score of WOE with the
  count-weighted WOE mean/std.  HYBRID: numeric z-score, categorical WOE.
* ONEHOT: one column per bin incl. missing; ZSCALE_ONEHOT: numeric z-score, categorical one-hot.
* ASIS_WOE / ASIS_PR: numeric raw value, categorical WOE / pos-rate.
* DISCRETE_Z*: numeric -> lower bound of its bin (first bin -> min, missing -> mean), z-scored.
* *_INDEX: categorical -> category index (for embeddings); numeric per the prefix.

Tree models use ``tree_bin_codes``: numeric rows -> bin index of their value (missing -> 0.0 as
``DTWorker.getFloatValue``), categorical -> category index (missing/unknown -> last bin).
"""
from __future__ import annotations

import numpy as np

from ..config.enums import is_index_norm
from . import binning as B

STD_DEV_CUTOFF = 4.0


def _cat_index(cc, col) -> np.ndarray:
    cats = cc.bin_category or []
    lut = {}
    for i, c in enumerate(cats):
        for sub in str(c).split("^"):
            lut.setdefault(sub, i)
    if col.kind == "str":
        d = col.dictionary
        m = np.array([lut.get(s, -1) for s in d] + [-1], dtype=np.int64)
        return m[np.where(col.values >= 0, col.values, len(d))]
    s = col.strings()
    return np.array([lut.get(v, -1) if v != "" else -1 for v in s], dtype=np.int64)


def _num_values(cc, col) -> np.ndarray:
    v = col.numeric().astype(np.float64)
    mean = cc.mean if cc.mean is not None else 0.0
    bad = ~np.isfinite(v)
    if bad.any():
        v = v.copy()
        v[bad] = mean
    return v


def zscore(v: np.ndarray, mean: float, std: float, cutoff: float) -> np.ndarray:
    mean = 0.0 if mean is None else float(mean)
    std = 0.0 if std is None else float(std)
    v = np.minimum(v, mean + cutoff * std)
    v = np.maximum(v, mean - cutoff * std)
    if std > 0.00001:
        return (v - mean) / std
    return np.zeros_like(v)


def woe_mean_std(cc, weighted: bool):
    ov = cc.d.get("_woeMeanStd") if hasattr(cc, "d") else None
    if ov is not None:            # binary .nn NNColumnStats carry the WOE mean/std explicitly
        return (ov[2], ov[3]) if weighted else (ov[0], ov[1])
    woe = np.asarray(cc.bin_weighted_woe if weighted else cc.bin_count_woe, dtype=np.float64)
    cnt = np.asarray(cc.bin_count_neg, dtype=np.float64) + np.asarray(cc.bin_count_pos, dtype=np.float64)
    tot = cnt.sum()
    s = (woe * cnt).sum()
    sq = (woe * woe * cnt).sum()
    mean = s / tot
    std = np.sqrt(abs((sq - s * s / tot) / (tot - 1))) if tot > 1 else 0.0
    return mean, std


def _bin_num(cc, col) -> np.ndarray:
    """BinUtils.getBinNum: -1 for missing/invalid."""
    if cc.is_categorical():
        return _cat_index(cc, col)
    v = col.numeric().astype(np.float64)
    bb = cc.bin_boundary or [float("-inf")]
    idx = B.bin_index_numeric(v, bb).astype(np.int64)
    idx[np.isnan(v)] = -1
    return idx


def _lookup_last(table_vals, idx):
    t = np.asarray(table_vals, dtype=np.float64)
    return np.where(idx >= 0, t[np.clip(idx, 0, len(t) - 1)], t[-1])


def norm_width(cc, norm_type: str) -> int:
    if norm_type == "ONEHOT":
        return (len(cc.bin_boundary or []) + 1) if not cc.is_categorical() else len(cc.bin_category or []) + 1
    if norm_type == "ZSCALE_ONEHOT" and cc.is_categorical():
        return len(cc.bin_category or []) + 1
    return 1


def normalize_column(cc, col, norm_type: str, cutoff: float | None) -> np.ndarray:
    """-> [N, width] float64."""
    cutoff = STD_DEV_CUTOFF if cutoff is None or not np.isfinite(cutoff) else float(cutoff)
    nt = norm_type
    n = len(col.values)
    cat = cc.is_categorical()
    if nt in ("ZSCALE", "ZSCORE", "OLD_ZSCALE", "OLD_ZSCORE"):
        if cat:
            idx = _cat_index(cc, col)
            v = _lookup_last(cc.bin_pos_rate, idx)
            if nt.startswith("OLD_"):
                return v[:, None]
        else:
            v = _num_values(cc, col)
        return zscore(v, cc.mean, cc.std_dev, cutoff)[:, None]
    if nt in ("WOE", "WEIGHT_WOE"):
        return _lookup_last(cc.bin_weighted_woe if nt == "WEIGHT_WOE" else cc.bin_count_woe,
                            _bin_num(cc, col))[:, None]
    if nt in ("WOE_ZSCORE", "WOE_ZSCALE", "WEIGHT_WOE_ZSCORE", "WEIGHT_WOE_ZSCALE"):
        w = nt.startswith("WEIGHT")
        woe = _lookup_last(cc.bin_weighted_woe if w else cc.bin_count_woe, _bin_num(cc, col))
        m, s = woe_mean_std(cc, w)
        return zscore(woe, m, s, cutoff)[:, None]
    if nt in ("HYBRID", "WEIGHT_HYBRID"):
        if cat:
            return _lookup_last(cc.bin_weighted_woe if nt == "WEIGHT_HYBRID" else cc.bin_count_woe,
                                _bin_num(cc, col))[:, None]
        return zscore(_num_values(cc, col), cc.mean, cc.std_dev, cutoff)[:, None]
    if nt == "ONEHOT" or (nt == "ZSCALE_ONEHOT" and cat):
        width = norm_width(cc, "ONEHOT")
        idx = _bin_num(cc, col)
        idx = np.where(idx < 0, width - 1, idx)
        out = np.zeros((n, width))
        out[np.arange(n), idx] = 1.0
        return out
    if nt == "ZSCALE_ONEHOT":
        return zscore(_num_values(cc, col), cc.mean, cc.std_dev, cutoff)[:, None]
    if nt in ("ASIS_WOE", "ASIS_PR"):
        if cat:
            tbl = cc.bin_count_woe if nt == "ASIS_WOE" else cc.bin_pos_rate
            return _lookup_last(tbl, _cat_index(cc, col))[:, None]
        return _num_values(cc, col)[:, None]
    if nt in ("DISCRETE_ZSCORE", "DISCRETE_ZSCALE"):
        if cat:
            v = _lookup_last(cc.bin_pos_rate, _cat_index(cc, col))
        else:
            idx = _bin_num(cc, col)
            bb = np.asarray(cc.bin_boundary, dtype=np.float64)
            lo = bb.copy()
            lo[0] = cc.stat("min", 0.0) if cc.stat("min") is not None else 0.0
            mean = cc.mean or 0.0
            v = np.where((idx < 0) | (idx >= len(bb)), mean, lo[np.clip(idx, 0, len(bb) - 1)])
        return zscore(v, cc.mean, cc.std_dev, cutoff)[:, None]
    if is_index_norm(nt):
        if cat:
            idx = _cat_index(cc, col)
            return np.where(idx < 0, len(cc.bin_category or []), idx).astype(np.float64)[:, None]
        if nt in ("ZSCALE_INDEX", "ZSCORE_INDEX"):
            return zscore(_num_values(cc, col), cc.mean, cc.std_dev, cutoff)[:, None]
        if nt == "WOE_INDEX":
            return _lookup_last(cc.bin_count_woe, _bin_num(cc, col))[:, None]
        # WOE_ZSCALE_INDEX (Normalizer.fullNormalize :305-315): z-scored WOE for numeric columns
        woe = _lookup_last(cc.bin_count_woe, _bin_num(cc, col))
        m, s = woe_mean_std(cc, False)
        return zscore(woe, m, s, cutoff)[:, None]
    raise ValueError(f"unsupported norm type {nt}")


def normalize_table(mc, ccs, table, columns=None, norm_type: str | None = None):
    """Normalize the selected columns -> (float32 [N, F'], names, column_nums)."""
    nt = norm_type or mc.norm_type
    cutoff = float(mc.normalize.get("stdDevCutOff", 6.0))
    cols = columns if columns is not None else [c for c in ccs if c.final_select and not c.is_target()
                                                 and not c.is_meta()]
    mats, names, nums = [], [], []
    for cc in cols:
        if cc.name not in table:
            raise KeyError(f"column {cc.name} missing from data")
        m = normalize_column(cc, table[cc.name], nt, cutoff)
        mats.append(m.astype(np.float32))
        if m.shape[1] == 1:
            names.append(cc.name)
        else:
            names.extend(f"{cc.name}_{i}" for i in range(m.shape[1]))
        nums.extend([cc.num] * m.shape[1])
    X = np.concatenate(mats, axis=1) if mats else np.zeros((table.n, 0), np.float32)
    return X, names, nums


def tree_bin_codes(ccs, table, columns):
    """CleanedData equivalent for GBT/RF: int32 codes [N, F] and bins per feature."""
    codes, nbins, is_cat = [], [], []
    for cc in columns:
        col = table[cc.name]
        if cc.is_categorical():
            idx = _cat_index(cc, col)
            ncat = len(cc.bin_category or [])
            codes.append(np.where(idx < 0, ncat, idx).astype(np.int32))
            nbins.append(ncat + 1)
            is_cat.append(1)
        else:
            v = col.numeric().astype(np.float64)
            v = np.where(np.isfinite(v) | np.isinf(v), v, 0.0)     # DTWorker.getFloatValue: missing -> 0f
            bb = cc.bin_boundary or [float("-inf")]
            codes.append(B.bin_index_numeric(v, bb).astype(np.int32))
            nbins.append(max(1, len(bb)))
            is_cat.append(0)
    C = np.stack(codes, 1) if codes else np.zeros((table.n, 0), np.int32)
    return C, np.array(nbins, np.int32), np.array(is_cat, np.uint8)


# ---- HIP path (K5 / K1') ---------------------------------------------------------------------------
def _raw_matrix(cols, table):
    """Column-major fp64 raw values: numeric value (NaN missing) or categorical index (-1 missing)."""
    out = np.empty((len(cols), table.n), dtype=np.float64)
    for j, cc in enumerate(cols):
        col = table[cc.name]
        out[j] = _cat_index(cc, col) if cc.is_categorical() else col.numeric()
    return out


def _to_dev(a, dev):
    """Host array -> ``dev`` without a host stall: page-locked staging (torch's caching host
    allocator) and a non-blocking copy on the current stream; a pageable ``as_tensor(device=)``
    waits for the stream's queued kernels first."""
    import torch
    t = torch.from_numpy(np.ascontiguousarray(a))
    if torch.device(dev).type != "cuda":
        return t.to(dev)
    return t.pin_memory().to(dev, non_blocking=True)


def _raw_matrix_dev(cols, table, dev):
    """:func:`_raw_matrix` on ``dev``.  The numeric columns that are rows of the parser's block
    matrix are uploaded in place (the block's spanned rows as one copy, placed by a device-side
    gather); only the others (categorical indices, filtered tables) go through a host gather."""
    import torch
    from ..data.gpu_parse import device_rows
    from ..data.reader import numeric_rows
    num_j = [j for j, cc in enumerate(cols) if not cc.is_categorical() and table[cc.name].kind == "num"]
    blk = device_rows([table[cols[j].name] for j in num_j], dev) if num_j else None
    if blk is not None:                      # GPU-parsed columns (K0): already in HBM
        if len(num_j) == len(cols):
            return blk
        out = torch.empty((len(cols), table.n), dtype=torch.float64, device=dev)
        out.index_copy_(0, _to_dev(np.asarray(num_j, np.int64), dev), blk)
        in_blk = set(num_j)
        rest = [j for j in range(len(cols)) if j not in in_blk]
        host = _raw_matrix([cols[j] for j in rest], table)
        out.index_copy_(0, _to_dev(np.asarray(rest, np.int64), dev), _to_dev(host, dev))
        return out
    hit = numeric_rows([table[cols[j].name].values for j in num_j]) if len(num_j) > 1 else None
    if hit is None:
        return torch.as_tensor(_raw_matrix(cols, table), device=dev)
    base, idx = hit
    lo, hi = int(idx.min()), int(idx.max()) + 1
    if hi - lo <= 2 * len(idx):
        blk = torch.as_tensor(base[lo:hi], device=dev)              # one H2D copy, no host gather
        if len(num_j) == len(cols) and np.array_equal(idx, np.arange(lo, hi)):
            return blk
        blk = blk.index_select(0, torch.as_tensor(idx - lo, device=dev))
    else:                                   # a sparse pick of a wide block: gather just those rows
        blk = torch.as_tensor(base[idx], device=dev)
    out = torch.empty((len(cols), table.n), dtype=torch.float64, device=dev)
    jt = torch.as_tensor(np.asarray(num_j, np.int64), device=dev)
    out.index_copy_(0, jt, blk)
    in_blk = set(num_j)
    rest = [j for j in range(len(cols)) if j not in in_blk]
    if rest:
        host = _raw_matrix([cols[j] for j in rest], table)
        out.index_copy_(0, torch.as_tensor(np.asarray(rest, np.int64), device=dev), torch.as_tensor(host, device=dev))
    return out


def _gpu_spec(cc, nt, cutoff):
    """Kernel spec for one width-1 column (None -> handled on the host, e.g. one-hot)."""
    cat = cc.is_categorical()
    mean, std = cc.mean or 0.0, cc.std_dev or 0.0
    base = dict(mean=mean, std=std, cutoff=cutoff)
    woe = lambda weighted: list(cc.bin_weighted_woe if weighted else cc.bin_count_woe)   # noqa: E731
    if nt in ("ZSCALE", "ZSCORE", "OLD_ZSCALE", "OLD_ZSCORE"):
        if cat:
            return dict(base, mode="cat_table", table=list(cc.bin_pos_rate), zflag=0 if nt.startswith("OLD_") else 1,
                        zmean=mean, zstd=std)
        return dict(base, mode="zscore")
    if nt in ("WOE", "WEIGHT_WOE"):
        t = woe(nt == "WEIGHT_WOE")
        return dict(base, mode="cat_table", table=t) if cat else dict(base, mode="num_table", table=t,
                                                                      bounds=list(cc.bin_boundary))
    if nt in ("WOE_ZSCORE", "WOE_ZSCALE", "WEIGHT_WOE_ZSCORE", "WEIGHT_WOE_ZSCALE"):
        wt = nt.startswith("WEIGHT")
        m, s = woe_mean_std(cc, wt)
        d = dict(base, table=woe(wt), zflag=1, zmean=m, zstd=s)
        return dict(d, mode="cat_table") if cat else dict(d, mode="num_table", bounds=list(cc.bin_boundary))
    if nt in ("HYBRID", "WEIGHT_HYBRID"):
        return dict(base, mode="cat_table", table=woe(nt == "WEIGHT_HYBRID")) if cat else dict(base, mode="zscore")
    if nt == "ONEHOT" or (nt == "ZSCALE_ONEHOT" and cat):
        return None
    if nt == "ZSCALE_ONEHOT":
        return dict(base, mode="zscore")
    if nt in ("ASIS_WOE", "ASIS_PR"):
        if cat:
            return dict(base, mode="cat_table", table=list(cc.bin_count_woe if nt == "ASIS_WOE" else cc.bin_pos_rate))
        return dict(base, mode="raw")
    if nt in ("DISCRETE_ZSCORE", "DISCRETE_ZSCALE"):
        if cat:
            return dict(base, mode="cat_table", table=list(cc.bin_pos_rate), zflag=1, zmean=mean, zstd=std)
        lo = list(np.asarray(cc.bin_boundary, dtype=np.float64))
        lo[0] = cc.stat("min") if cc.stat("min") is not None else 0.0
        return dict(base, mode="discrete", bounds=list(cc.bin_boundary), table=lo)
    if is_index_norm(nt):
        if cat:
            return dict(base, mode="cat_index", ncat=len(cc.bin_category or []))
        if nt in ("ZSCALE_INDEX", "ZSCORE_INDEX"):
            return dict(base, mode="zscore")
        if nt == "WOE_INDEX":
            return dict(base, mode="num_table", table=woe(False), bounds=list(cc.bin_boundary))
        m, s = woe_mean_std(cc, False)
        return dict(base, mode="num_table", table=woe(False), bounds=list(cc.bin_boundary), zflag=1, zmean=m, zstd=s)
    raise ValueError(f"unsupported norm type {nt}")


def normalize_table_gpu(mc, ccs, table, columns=None, norm_type: str | None = None, device="cuda",
                        return_device: bool = False):
    """HIP normalization (one launch for every width-1 column); identical output to
    :func:`normalize_table`.  ``return_device`` keeps X resident in HBM (training path)."""
    import torch
    from ..ops import stats_ops
    nt = norm_type or mc.norm_type
    cutoff = float(mc.normalize.get("stdDevCutOff", 6.0))
    cols = columns if columns is not None else [c for c in ccs if c.final_select and not c.is_target()
                                                 and not c.is_meta()]
    specs, names, nums, host_cols = [], [], [], []
    pos = 0
    gpu_cols = []
    for cc in cols:
        if cc.name not in table:
            raise KeyError(f"column {cc.name} missing from data")
        s = _gpu_spec(cc, nt, cutoff)
        if s is None:
            width = norm_width(cc, "ONEHOT")
            host_cols.append((cc, pos, width))
            names.extend(f"{cc.name}_{i}" for i in range(width))
            nums.extend([cc.num] * width)
            pos += width
        else:
            s["out_col"] = pos
            specs.append(s)
            gpu_cols.append(cc)
            names.append(cc.name)
            nums.append(cc.num)
            pos += 1
    dev = torch.device(device)
    out = torch.zeros(table.n, max(pos, 1), dtype=torch.float32, device=dev)
    if gpu_cols:
        vals = _raw_matrix_dev(gpu_cols, table, dev)
        stats_ops.normalize(vals, specs, out)
    for cc, p0, width in host_cols:
        out[:, p0: p0 + width] = torch.as_tensor(normalize_column(cc, table[cc.name], nt, cutoff), dtype=torch.float32,
                                                 device=dev)
    out = out[:, :pos]
    return (out if return_device else out.cpu().numpy()), names, nums


def tree_bin_codes_gpu(ccs, table, columns, device="cuda"):
    """HIP CleanedData codes (uint8, nbins <= 256)."""
    import torch
    from ..ops import stats_ops
    nbins, is_cat, ncat, bounds = [], [], [], []
    for cc in columns:
        if cc.is_categorical():
            k = len(cc.bin_category or [])
            nbins.append(k + 1); is_cat.append(1); ncat.append(k); bounds.append(None)
        else:
            bb = cc.bin_boundary or [float("-inf")]
            nbins.append(max(1, len(bb))); is_cat.append(0); ncat.append(0); bounds.append(bb)
    if max(nbins, default=1) > 256:
        return None
    dev = torch.device(device)
    vals = _raw_matrix_dev(columns, table, dev)
    out = torch.zeros(table.n, max(1, len(columns)), dtype=torch.uint8, device=dev)
    stats_ops.bin_codes(vals, is_cat, bounds, ncat, out)
    return out.cpu().numpy().astype(np.int32), np.array(nbins, np.int32), np.array(is_cat, np.uint8)


# ---- streamed norm: one plan, one fused kernel pass per chunk (K5) ------------------------------
class NormPlan:
    """Everything the per-chunk pass needs, built once for the ``norm`` columns: the width-1
    columns' kernel specs (device tensors), the host-side one-hot columns, and the tree-code spec.
    ``run(table)`` normalizes one chunk: on the GPU one ``norm_codes`` launch reads the raw values
    once and writes the fp32 rows and/or the bf16 GEMM-ready rows (``kpad`` wide, bias column =
    1 at ``width``) and/or the uint8 CleanedData codes; on the CPU the numpy oracle does the same."""

    def __init__(self, mc, ccs, cols, norm_type: str | None = None, want_x: bool = True,
                 want_codes: bool = False, x_dtype: str = "float32", device=None, pinned_out: int = 0):
        import torch
        self.mc, self.cols = mc, list(cols)
        self.pinned_out, self._pins, self._pin_i = int(pinned_out), {}, {}
        self.async_out, self.last_event = False, None     # async D2H into the pinned buffers
        self.nt = norm_type or mc.norm_type
        self.cutoff = float(mc.normalize.get("stdDevCutOff", 6.0))
        self.want_x, self.want_codes = want_x, want_codes
        self.x_dtype = x_dtype
        self.dev = torch.device(device) if device is not None else None
        self.gpu = self.dev is not None and self.dev.type == "cuda"
        specs, names, nums, host_cols, gpu_cols = [], [], [], [], []
        pos = 0
        for cc in self.cols:
            s = _gpu_spec(cc, self.nt, self.cutoff)
            if s is None:
                width = norm_width(cc, self.nt if self.nt == "ONEHOT" else "ONEHOT")
                host_cols.append((cc, pos, width))
                names.extend(f"{cc.name}_{i}" for i in range(width))
                nums.extend([cc.num] * width)
                pos += width
            else:
                s["out_col"] = pos
                specs.append(s)
                gpu_cols.append(cc)
                names.append(cc.name)
                nums.append(cc.num)
                pos += 1
        self.width, self.names, self.nums = pos, names, nums
        self.specs, self.gpu_cols, self.host_cols = specs, gpu_cols, host_cols
        self.kpad = ((pos + 1 + 127) // 128) * 128            # bf16 rows: values + bias + zero padding
        nb, ic, ncat, bounds = [], [], [], []
        for cc in self.cols:
            if cc.is_categorical():
                k = len(cc.bin_category or [])
                nb.append(k + 1); ic.append(1); ncat.append(k); bounds.append(None)
            else:
                bb = cc.bin_boundary or [float("-inf")]
                nb.append(max(1, len(bb))); ic.append(0); ncat.append(0); bounds.append(bb)
        self.nbins, self.is_cat = np.array(nb, np.int32), np.array(ic, np.uint8)
        self.code_dtype = np.uint8 if self.nbins.max(initial=1) <= 256 else np.int16
        self._ncat, self._cbounds = ncat, bounds
        self._dev_specs = None
        self._bufs = {}

    def _device_specs(self):
        import torch
        from ..ops import stats_ops as so
        if self._dev_specs is not None:
            return self._dev_specs
        F = len(self.gpu_cols)
        ip = np.zeros((max(F, 1), 8), np.int32)
        dp = np.zeros((max(F, 1), 8), np.float64)
        bounds, tables = [], []
        for f, s in enumerate(self.specs):
            b = list(s.get("bounds") or [float("-inf")])
            t = list(s.get("table") or [0.0])
            nt = int(s["ncat"]) if s["mode"] == "cat_index" else len(t)
            ip[f] = [so.NM[s["mode"]], s["out_col"], len(bounds), len(b), len(tables), nt, int(s.get("zflag", 0)), 0]
            bounds.extend(b)
            tables.extend(t)
            dp[f, :5] = [s.get("mean", 0.0) or 0.0, s.get("std", 0.0) or 0.0, s.get("cutoff", 6.0),
                         s.get("zmean", 0.0) or 0.0, s.get("zstd", 0.0) or 0.0]
        cb, coff = so.pack_bounds(self._cbounds)
        cip = np.zeros((len(self.cols), 4), np.int32)
        for f in range(len(self.cols)):
            cip[f] = [int(self.is_cat[f]), coff[f], coff[f + 1] - coff[f], int(self._ncat[f])]
        t = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a), dtype=dt).to(self.dev)   # noqa: E731
        self._dev_specs = dict(ip=t(ip, torch.int32), dp=t(dp, torch.float64),
                               bounds=t(np.asarray(bounds or [0.0], np.float64), torch.float64),
                               tables=t(np.asarray(tables or [0.0], np.float64), torch.float64),
                               cip=t(cip, torch.int32), cbounds=t(cb, torch.float64))
        return self._dev_specs

    def _host(self, key, t):
        """D2H of one output.  ``pinned_out`` = k: into the next of k rotating page-locked buffers
        (DMA rate instead of a pageable copy; the returned array is overwritten k calls later --
        the streamed norm keeps at most one chunk in its writer)."""
        import torch
        if not self.pinned_out:
            return t.cpu().numpy()
        i = self._pin_i[key] = (self._pin_i.get(key, -1) + 1) % self.pinned_out
        buf = self._pins.get((key, i))
        if buf is None or buf.numel() < t.numel():
            buf = self._pins[(key, i)] = torch.empty(t.numel(), dtype=t.dtype, pin_memory=True)
        h = buf[: t.numel()].view(t.shape)
        if self.async_out:
            # the caller synchronises on ``last_event`` before reading (streamed norm: the writer
            # thread), so the consumer queues the next chunk instead of waiting for this DMA
            h.copy_(t, non_blocking=True)
            self.last_event = torch.cuda.Event()
            self.last_event.record(torch.cuda.current_stream(self.dev))
        else:
            h.copy_(t)
        return h.numpy()

    def _onehot_specs(self):
        """Device [F][5] (is_cat, bnd_off, nbnd, width, out_col) + packed numeric boundaries."""
        import torch
        if getattr(self, "_oh", None) is None:
            ip, bounds = np.zeros((len(self.host_cols), 5), np.int32), []
            for f, (cc, p0, width) in enumerate(self.host_cols):
                bb = [] if cc.is_categorical() else list(cc.bin_boundary or [float("-inf")])
                ip[f] = [int(cc.is_categorical()), len(bounds), len(bb), width, p0]
                bounds.extend(bb)
            self._oh = (torch.as_tensor(ip).to(self.dev),
                        torch.as_tensor(np.asarray(bounds or [0.0], np.float64)).to(self.dev))
        return self._oh

    def _buf(self, key, shape, dtype, init=None):
        import torch
        b = self._bufs.get(key)
        if b is None or b.shape[0] < shape[0] or tuple(b.shape[1:]) != tuple(shape[1:]):
            b = torch.zeros(shape, dtype=dtype, device=self.dev)
            if init is not None:
                init(b)
            self._bufs[key] = b
        return b[: shape[0]]

    def run(self, table, keep_device: bool = False) -> dict:
        """-> {"X": fp32 [n, width] | "Xb": uint16 (bf16 bits) [n, kpad], "codes": [n, F]} (numpy;
        ``keep_device`` on a GPU: "X" as a device tensor -- a fresh copy, not the reused buffer)."""
        n = table.n
        out = {}
        bf16 = self.want_x and self.x_dtype == "bf16"
        if not self.gpu:
            if self.want_x:
                X, _, _ = normalize_table(self.mc, None, table, columns=self.cols, norm_type=self.nt)
                if bf16:
                    import torch
                    xb = np.zeros((n, self.kpad), np.uint16)
                    xb[:, : self.width] = torch.from_numpy(np.ascontiguousarray(X)).to(torch.bfloat16) \
                        .view(torch.int16).numpy().view(np.uint16)
                    xb[:, self.width] = 0x3F80                       # bf16 1.0 (bias neuron)
                    out["Xb"] = xb
                else:
                    out["X"] = X
            if self.want_codes:
                C, _, _ = tree_bin_codes(None, table, self.cols)
                out["codes"] = C.astype(self.code_dtype)
            return out
        import torch
        from ..ops import _native as nat
        need_codes = self.want_codes and self.code_dtype == np.uint8
        dev_cols = self.gpu_cols if not need_codes else self.cols
        vals = _raw_matrix_dev(dev_cols, table, self.dev) if dev_cols else None
        ds = self._device_specs()
        outf = self._buf("f", (n, max(self.width, 1)), torch.float32) if (self.want_x and not bf16) else None
        outb = self._buf("b", (n, self.kpad), torch.bfloat16,
                         init=lambda b: b[:, self.width].fill_(1.0)) if bf16 else None
        codes = self._buf("c", (n, max(1, len(self.cols))), torch.uint8) if need_codes else None
        if vals is not None and n:
            if need_codes and len(self.gpu_cols) != len(self.cols):
                # one-hot columns present: the width-1 specs index the gpu columns only -> two passes
                sub = _raw_matrix_dev(self.gpu_cols, table, self.dev)
                rc = nat.call_hip("shifu_norm_codes", sub, sub.stride(0), n, len(self.gpu_cols), ds["ip"], ds["dp"],
                                  ds["bounds"], ds["tables"], None, None, outf, 0 if outf is None else outf.stride(0),
                                  outb, 0 if outb is None else outb.stride(0), None, 0, nat.stream_of(sub)) \
                    if self.gpu_cols and (outf is not None or outb is not None) else 0
                rc2 = nat.call_hip("shifu_norm_codes", vals, vals.stride(0), n, len(self.cols), None, None, None, None,
                                   ds["cip"], ds["cbounds"], None, 0, None, 0, codes, codes.stride(0),
                                   nat.stream_of(vals))
                rc = rc or rc2
            else:
                want_v = outf is not None or outb is not None
                rc = nat.call_hip("shifu_norm_codes", vals, vals.stride(0), n, vals.shape[0],
                                  ds["ip"] if want_v else None, ds["dp"] if want_v else None, ds["bounds"], ds["tables"],
                                  ds["cip"] if need_codes else None, ds["cbounds"] if need_codes else None,
                                  outf, 0 if outf is None else outf.stride(0), outb,
                                  0 if outb is None else outb.stride(0), codes,
                                  0 if codes is None else codes.stride(0), nat.stream_of(vals))
            if rc:
                raise RuntimeError(f"shifu_norm_codes failed rc={rc}")
        if self.host_cols and n and (outf is not None or outb is not None):
            # one-hot columns: one K5 one-hot launch (raw values / category indices -> 0/1 blocks)
            ohv = _raw_matrix_dev([cc for cc, _, _ in self.host_cols], table, self.dev)
            oip, obnd = self._onehot_specs()
            rc = nat.call_hip("shifu_onehot", ohv, ohv.stride(0), n, len(self.host_cols), oip, obnd,
                              outf, 0 if outf is None else outf.stride(0), outb, 0 if outb is None else outb.stride(0),
                              nat.stream_of(ohv))
            if rc:
                raise RuntimeError(f"shifu_onehot failed rc={rc}")
        if outf is not None:
            out["X"] = outf[:, : self.width].clone() if keep_device else self._host("X", outf[:, : self.width])
        if outb is not None:
            out["Xb"] = self._host("Xb", outb.view(torch.int16)).view(np.uint16)
        if self.want_codes:
            if codes is not None:
                out["codes"] = self._host("codes", codes)
            else:
                C, _, _ = tree_bin_codes(None, table, self.cols)
                out["codes"] = C.astype(self.code_dtype)
        return out
