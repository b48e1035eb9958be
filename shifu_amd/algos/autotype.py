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


def scan(mc, header: list, cols: list, rank: int = 0, world: int = 1, nthreads: int | None = None,
         block_bytes: int = BLOCK_BYTES) -> dict:
    """Auto-type statistics of columns ``cols`` (indices into ``header``) over this rank's share,
    merged over the ranks: {column index: ColumnCounts}."""
    import os
    nthreads = nthreads or min(16, os.cpu_count() or 4)
    from ..data.purifier import plan_dataset
    from ..parallel import dist
    lib = _native()
    ds = mc.dataSet
    plan = plan_dataset(mc, ds, [], [])
    target = ds.get("targetColumnName")
    tag_col = header.index(target) if (target in header and not mc.is_linear_target()) else -1
    tags = "\n".join(str(t).strip() for t in mc.flatten_tags()) if tag_col >= 0 else ""
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
