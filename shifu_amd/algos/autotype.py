"""Data-parallel auto-type statistics for ``init`` (H5; InitModelProcessor.java:105-120, 143-254,
AutoTypeDistinctCountMapper.java:134-219, AutoTypeDistinctCountReducer).

Every rank streams ITS byte ranges of the training data (``data/stream.byte_ranges``, the same
split ``stats`` uses) through the native scanner (``runtime/csrc/autotype_scan.cpp``): per column
the row count, the missing-or-invalid count (lower-cased field in the missing-value list), the
count of values ``Double.parseDouble`` accepts, the set of value hashes (exact while below the
scanner's cap) plus a 2^14-register HyperLogLog sketch, and the first distinct values
("frequent items").  Rows whose trimmed tag is not a configured tag are skipped, and the data set's
filter expression is applied per row, as in the reference mapper.  Host memory is bounded by the
read block plus the per-column sketches; no column is ever materialised.

Ranks merge by all-reduce (counts: sum; HLL registers: max) and by gathering the exact hash sets
(union; a column that overflowed the cap anywhere uses the merged sketch) and the item lists
(ordered union, 200 items).
"""
from __future__ import annotations

import ctypes
import time

import numpy as np

from ..data.join import raw_blocks
from ..utils.log import get_logger

_log = get_logger("algos.autotype")

ITEMS_CAP = 200
STATS: dict = {}          # cumulative native scan seconds (tools/join_lab.py)
BLOCK_BYTES = 256 << 20


class ColumnCounts:
    __slots__ = ("count", "invalid", "validnum", "distinct", "items", "exact")

    def __init__(self, count, invalid, validnum, distinct, items, exact):
        self.count, self.invalid, self.validnum = int(count), int(invalid), int(validnum)
        self.distinct, self.items, self.exact = int(distinct), list(items), bool(exact)


def _native():
    from ..ops import _native as nat
    lib = nat.rt()
    if lib is None or not hasattr(lib, "shifu_at_new"):
        raise RuntimeError("auto-type scan needs the native runtime (python -m shifu_amd.build_native)")
    return lib


def _filter_mask(plan, data) -> np.ndarray | None:
    """Per non-blank line of the block: the data set's filter expression (None: keep all)."""
    if not (plan.filt and str(plan.filt).strip()):
        return None
    from ..data.expr import Evaluator
    from ..data.reader import parse_block, table_from_parts
    strs, nums = set(plan.strs), set(plan.nums)
    kinds = [2 if h in strs else (1 if h in nums else 0) for h in plan.header]
    t = table_from_parts(plan.header, kinds, [parse_block(data, plan.delim, kinds, plan.missing, 4)])
    try:
        return np.ascontiguousarray(Evaluator(plan.filt).mask(t), dtype=np.uint8)
    except Exception as e:   # the reference keeps the row on expression errors
        _log.warning("filter expression %r failed (%s); no rows filtered", plan.filt, e)
        return None


def _gpu_device():
    """The CUDA device of a GPU auto-type scan (``shifu.autoType.gpu``: auto / true / false), or None."""
    from ..config import environment
    mode = str(environment.get("shifu.autoType.gpu", "auto")).lower()
    if mode in ("false", "0", "off"):
        return None
    import torch
    from ..utils.device import is_gpu_available
    if not is_gpu_available():                     # SHIFU_FORCE_CPU=1 or no visible GPU
        if mode in ("true", "1", "on"):
            raise RuntimeError("shifu.autoType.gpu=true but no GPU is visible")
        return None
    from ..ops import _native as nat
    if mode in ("true", "1", "on"):
        nat.hip()
    elif not nat.hip_available():
        return None
    return torch.device("cuda", torch.cuda.current_device())


def scan(mc, header: list, cols: list, rank: int = 0, world: int = 1, nthreads: int | None = None,
         block_bytes: int = BLOCK_BYTES) -> dict:
    """Auto-type statistics of columns ``cols`` (indices into ``header``) over this rank's share,
    merged over the ranks: {column index: ColumnCounts}.  On a GPU the blocks are coded and counted
    on the device (:func:`_scan_gpu`) when the data set's format allows it, else by the host scanner."""
    import os
    nthreads = nthreads or min(16, os.cpu_count() or 4)
    from ..data.purifier import plan_dataset
    lib = _native()
    ds = mc.dataSet
    plan = plan_dataset(mc, ds, [], [])
    target = ds.get("targetColumnName")
    tag_col = header.index(target) if (target in header and not mc.is_linear_target()) else -1
    tag_list = [str(t).strip() for t in mc.flatten_tags()] if tag_col >= 0 else []
    dev = _gpu_device()
    if dev is not None:
        res = _scan_gpu(plan, header, cols, rank, world, dev, tag_col, tag_list, block_bytes)
        if res is not None:
            return _merge(lib, res, cols)
    return _merge(lib, _scan_host(lib, plan, header, cols, rank, world, nthreads, block_bytes, tag_col, tag_list), cols)


def _scan_host(lib, plan, header, cols, rank, world, nthreads, block_bytes, tag_col, tag_list):
    """The native host scanner over this rank's share: (counts [3F], regs [sel][M] u8,
    {col: exact hashes or None}, {col: items}, rows, skipped)."""
    tags = "\n".join(tag_list)
    missing = "\n".join(str(m) for m in plan.missing)
    h = lib.shifu_at_new(len(header), tag_col, tags.encode(), missing.encode(), plan.delim.encode())
    if not h:
        raise RuntimeError("auto-type scanner: bad arguments")
    try:
        rows = 0
        from ..data.stream import prefetched
        # blocks are read on a background thread one ahead of the scan (three rotating buffers)
        for _, _, data in prefetched(lambda: raw_blocks(plan, rank, world, block_bytes, nbuf=3), 1):
            mask = _filter_mask(plan, data)
            arr = np.frombuffer(data, dtype=np.uint8)          # the block's bytes, no copy
            t0 = time.perf_counter()
            got = lib.shifu_at_feed(h, arr.ctypes.data, len(arr), None if mask is None else mask.ctypes.data,
                                    int(nthreads))
            STATS["feed_s"] = STATS.get("feed_s", 0.0) + time.perf_counter() - t0
            if got < 0:
                raise RuntimeError("auto-type scanner failed on a block")
            rows += got
        t0 = time.perf_counter()
        F = len(header)
        counts = np.zeros(3 * F, dtype=np.int64)
        lib.shifu_at_counts(h, counts.ctypes.data)
        P = int(lib.shifu_at_hll_p())
        M = 1 << P
        cap = int(lib.shifu_at_exact_cap())
        sel = list(cols)
        regs = np.zeros((len(sel), M), dtype=np.uint8)
        allregs = np.zeros((F, M), dtype=np.uint8)
        lib.shifu_at_hll(h, allregs.ctypes.data)
        regs[:] = allregs[sel]
        del allregs
        exact, items = {}, {}
        buf = np.zeros(cap, dtype=np.uint64)
        ibuf = ctypes.create_string_buffer(1 << 22)
        for c in sel:
            n = lib.shifu_at_exact(h, c, buf.ctypes.data, cap)
            exact[c] = buf[:n].copy() if n >= 0 else None
            k = lib.shifu_at_items(h, c, ibuf, len(ibuf))
            items[c] = ibuf.raw[:k].decode("utf-8", "replace").split("\n")[:-1] if k > 0 else []
        skipped = int(lib.shifu_at_skipped(h))
        STATS["finish_s"] = STATS.get("finish_s", 0.0) + time.perf_counter() - t0
    finally:
        lib.shifu_at_free(h)
    return counts, regs, exact, items, rows, skipped


def _merge(lib, res, cols) -> dict:
    """Merge one rank's statistics over the ranks and finish the distinct counts."""
    from ..parallel import dist
    counts, regs, exact, items, rows, skipped = res
    sel = list(cols)
    cap = int(lib.shifu_at_exact_cap())
    info = dist.info()
    if info.world_size > 1:
        counts = dist.all_reduce_np(counts, "sum")
        regs = dist.all_reduce_np(regs.astype(np.int32), "max").astype(np.uint8)
        parts = dist.all_gather_objects((exact, items))
        exact = {c: None if any(p[0][c] is None for p in parts) else
                 np.unique(np.concatenate([p[0][c] for p in parts])) for c in sel}
        items = {}
        for c in sel:
            seen, lst = set(), []
            for p in parts:
                for s in p[1][c]:
                    if s not in seen and len(lst) < ITEMS_CAP:
                        seen.add(s)
                        lst.append(s)
            items[c] = lst
        tot = dist.all_reduce_np(np.array([rows, skipped], dtype=np.int64), "sum")
        rows, skipped = int(tot[0]), int(tot[1])
    out = {}
    for j, c in enumerate(sel):
        if exact[c] is not None and len(exact[c]) <= cap:
            d, ex = len(exact[c]), True
        else:
            r = np.ascontiguousarray(regs[j])
            d, ex = int(round(lib.shifu_at_hll_estimate(r.ctypes.data))), False
        out[c] = ColumnCounts(counts[3 * c], counts[3 * c + 1], counts[3 * c + 2], d, items[c], ex)
    _log.info("auto type scan: %d rows (%d with an invalid tag skipped) over %d columns", rows, skipped, len(sel))
    return out


def _gpu_lines(dbuf, L: int, dev):
    """Line bounds of a block in HBM (the K0 newline kernels): int64 starts / ends ('\\n' excluded)."""
    import torch
    from ..ops import _native as nat
    h = nat.hip()
    ws = torch.empty(int(h.shifu_newline_ws_bytes(L)) + 64, dtype=torch.uint8, device=dev)
    st = nat.stream_of(dbuf)
    nat.call_hip("shifu_newline_count", dbuf, L, ws, st)
    o = int(h.shifu_newline_count_offset(L))
    cnt = int(ws[o:o + 8].view(torch.int64).item())
    ends = torch.empty(cnt, dtype=torch.long, device=dev)
    if cnt:
        nat.call_hip("shifu_newline_write", dbuf, L, ws, ends, st)
    if L and int(dbuf[L - 1].item()) != 10:
        ends = torch.cat([ends, torch.tensor([L], dtype=torch.long, device=dev)])
    starts = torch.zeros(ends.numel(), dtype=torch.long, device=dev)
    if ends.numel() > 1:
        starts[1:] = ends[:-1] + 1
    return starts, ends


def _scan_gpu(plan, header, cols, rank, world, dev, tag_col, tag_list, block_bytes):
    """The device scan (ops/csrc/autotype_kernels.hip) over this rank's share, or None when the data
    set needs the host scanner (multi-byte delimiter, a filter expression, gz / parquet parts, more
    or longer missing tokens / tags than the kernel holds).  Same per-field codes, counts, exact sets
    and HyperLogLog registers as the host scanner; the items are the column's first distinct values
    in the rank's row order (the host scanner's depend on its thread split)."""
    import torch
    from ..data.reader import list_data_files
    from ..data.stream import _lines_in_range, byte_ranges, prefetched
    from ..ops import _native as nat
    caps = np.zeros(8, np.int32)
    nat.hip().shifu_at_gpu_caps(caps.ctypes.data)
    hll_p, exact_cap, slots, n_items, maxtok, toklen, maxtag, taglen = (int(v) for v in caps)
    d = (plan.delim or "|").encode()
    toks = [str(m).encode() for m in plan.missing]
    tgs = [t.encode() for t in tag_list]
    files = list_data_files(plan.data_path)
    if (len(d) != 1 or d == b"\n" or (plan.filt and str(plan.filt).strip()) or not files or
            any(f.endswith((".gz", ".parquet")) for f in files) or len(toks) > maxtok or
            any(len(t) >= toklen or b"\0" in t for t in toks) or len(tgs) > maxtag or
            any(len(t) >= taglen or b"\0" in t for t in tgs)):
        return None
    F = len(header)
    sel = list(cols)
    csel = torch.as_tensor(np.asarray(sel, np.int32), device=dev)
    cnt = torch.zeros(F, 3, dtype=torch.int64, device=dev)
    hset = torch.zeros(F, slots, dtype=torch.int64, device=dev)
    first = torch.full((F, slots), -1, dtype=torch.int64, device=dev)      # u64 max: "no line yet"
    used = torch.zeros(F, dtype=torch.int32, device=dev)
    ovf = torch.zeros(F, dtype=torch.int32, device=dev)
    hll = torch.zeros(F, 1 << hll_p, dtype=torch.int32, device=dev)
    tok_blob = b"".join(t + b"\0" for t in toks) or b"\0"
    tag_blob = b"".join(t + b"\0" for t in tgs) or b"\0"
    items = {c: {} for c in sel}             # column -> {hash: (first line, raw value)}
    full = set()                            # columns whose first n_items values are all known
    st = nat.stream_of(cnt)
    rows = skipped = 0
    line0 = 0
    t_feed = 0.0

    def blocks():
        for fi, path, a, b in byte_ranges(files, rank, world):
            for off, data in _lines_in_range(path, a, b, block_bytes, nbuf=4, pinned=True):
                if plan.skip_header_line and fi == 0 and off == 0:
                    k = bytes(data[: 1 << 20]).find(b"\n")
                    if k < 0 and len(data) > (1 << 20):
                        k = bytes(data).find(b"\n")
                    data = data[k + 1:] if k >= 0 else data[len(data):]
                if len(data):
                    yield data

    for data in prefetched(blocks, 1):
        t0 = time.perf_counter()
        L = len(data)
        host = np.frombuffer(data, dtype=np.uint8)
        dbuf = torch.empty(L + 64, dtype=torch.uint8, device=dev)
        dbuf[:L].copy_(torch.from_numpy(host), non_blocking=True)
        ls, le = _gpu_lines(dbuf, L, dev)
        nl = int(ls.numel())
        if nl == 0:
            continue
        codes = torch.empty(F, nl, dtype=torch.int64, device=dev)
        lflags = torch.empty(nl, dtype=torch.int32, device=dev)
        nat.call_hip("shifu_at_gpu_codes", dbuf, ls, le, nl, F, codes, nl, lflags, d[0], len(toks), tok_blob,
                     tag_col, len(tgs), tag_blob, st)
        nat.call_hip("shifu_at_gpu_apply", codes, nl, nl, lflags, line0, csel, len(sel), cnt, hset, first, used,
                     ovf, hll, st)
        fl = lflags.cpu().numpy()
        rows += int((fl == 0).sum())
        skipped += int((fl == 2).sum())
        # first distinct values: the columns still short of n_items known values
        want = [c for c in sel if c not in full]
        if want:
            wt = torch.as_tensor(np.asarray(want, np.int32), device=dev)
            out = torch.empty(len(want), n_items, 2, dtype=torch.int64, device=dev)
            nat.call_hip("shifu_at_gpu_items", wt, len(want), hset, first, out, st)
            o = out.cpu().numpy()
            need = {}                         # line in block -> [(column, hash)]
            for j, c in enumerate(want):
                known = items[c]
                hs, ln = o[j, :, 0], o[j, :, 1]
                for h_, l_ in zip(hs, ln):
                    if h_ == 0:
                        break
                    if int(h_) in known:
                        continue
                    l_ = int(l_)
                    if line0 <= l_ < line0 + nl:
                        need.setdefault(l_ - line0, []).append((c, int(h_)))
                if int(hs[-1]) != 0 and int(o[j, -1, 1]) < line0 + nl:
                    full.add(c)               # n_items values, all first seen up to this block
            if need:
                idx = np.asarray(sorted(need), np.int64)
                bounds = torch.stack([ls, le])[:, torch.as_tensor(idx, device=dev)].cpu().numpy()
                for k, li in enumerate(idx):
                    a_, b_ = int(bounds[0, k]), int(bounds[1, k])
                    raw = bytes(host[a_:b_])
                    if raw.endswith(b"\r"):
                        raw = raw[:-1]
                    fields = raw.split(d)
                    for c, h_ in need[int(li)]:
                        items[c][h_] = (line0 + int(li), fields[c].decode("utf-8", "replace"))
        line0 += nl
        t_feed += time.perf_counter() - t0
        del codes, dbuf
    STATS["feed_s"] = STATS.get("feed_s", 0.0) + t_feed
    t0 = time.perf_counter()
    nat.call_hip("shifu_at_gpu_hll_from_sets", csel, len(sel), hset, hll, st)   # every column's sketch
    counts = cnt.cpu().numpy().reshape(-1)
    ov = ovf.cpu().numpy()
    hs_all = hset[csel.long()].cpu().numpy().view(np.uint64)
    regs = np.minimum(hll[csel.long()].cpu().numpy(), 255).astype(np.uint8)
    exact, its = {}, {}
    for j, c in enumerate(sel):
        exact[c] = None if ov[c] else np.sort(hs_all[j][hs_all[j] != 0])
        its[c] = [v for _, v in sorted(items[c].values())][:ITEMS_CAP]
    STATS["finish_s"] = STATS.get("finish_s", 0.0) + time.perf_counter() - t0
    STATS["gpu"] = True
    _log.info("auto type GPU scan: %d rows, %d lines coded, %.1f s", rows, line0, t_feed)
    return counts, regs, exact, its, rows, skipped
