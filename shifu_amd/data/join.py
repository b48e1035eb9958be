"""Streamed, data-parallel row joins: raw input lines + computed columns (B11 combo, B13 encode).

The reference appends the sub-model scores to the raw rows with a Pig join
(``ComboModelProcessor.runComboModels`` J/core/processor/ComboModelProcessor.java:278-356, the
``DataJoin`` of the sub model EvalScore outputs) and the tree leaf-path codes with a MapReduce
pass (``EncodeDataProcessor`` / ``IndependentTreeModel.encode``).  Here every rank streams ITS
byte ranges of the data set (``data/stream.byte_ranges``, the split every other step uses), parses
only the columns the computation needs, computes the new columns block by block (the scorers run
on the device when one is present) and writes each non-blank raw line -- its bytes untouched,
cut or padded to the header width -- followed by the new columns, formatted natively
(``runtime/csrc/eval_rows.cpp``: ``shifu_format_rows_sep`` + ``shifu_join_lines``), into its own
part file ``part-<rank>``.  Parts in rank order hold the rows in file order.  Host memory is
bounded by one block: no table-wide string column is ever built.
"""
from __future__ import annotations

import gzip
import os
import time

import numpy as np

from ..utils.log import get_logger

_log = get_logger("data.join")

BLOCK_BYTES = 256 << 20
FIXED6, REPR, DICT, REPR_OR_EMPTY = 0, 1, 2, 3


def _rt():
    from ..ops import _native as nat
    lib = nat.rt()
    if lib is None or not hasattr(lib, "shifu_join_lines"):
        raise RuntimeError("row join needs the native runtime (python -m shifu_amd.build_native)")
    return lib


def raw_blocks(plan, rank: int, world: int, block_bytes: int = BLOCK_BYTES, nbuf: int = 1):
    """(file index, offset, bytes of complete lines) of this rank's share, header line removed;
    ``.gz`` parts are decompressed in blocks, ``.parquet`` parts rendered as delimited text.
    A plain-text block stays valid until ``nbuf - 1`` further blocks have been produced."""
    from .reader import list_data_files
    from .stream import _lines_in_range, byte_ranges
    files = list_data_files(plan.data_path)
    if not files:
        raise FileNotFoundError(f"no data under {plan.data_path}")
    for fi, path, a, b in byte_ranges(files, rank, world):
        if a is None:                                       # indivisible unit: gz / parquet
            if path.endswith(".parquet"):
                yield fi, 0, parquet_text(path, plan)
                continue
            with gzip.open(path, "rb") as fh:
                carry = b""
                first = True
                while True:
                    chunk = fh.read(block_bytes)
                    if not chunk:
                        if carry:
                            yield fi, 0, carry
                        break
                    data = carry + chunk
                    cut = data.rfind(b"\n")
                    if cut < 0:
                        carry = data
                        continue
                    blk, carry = data[:cut + 1], data[cut + 1:]
                    if first and plan.skip_header_line and fi == 0:
                        nl = blk.find(b"\n")
                        blk = blk[nl + 1:]
                    first = False
                    yield fi, 0, blk
            continue
        for off, data in _lines_in_range(path, a, b, block_bytes, nbuf=nbuf):
            if plan.skip_header_line and fi == 0 and off == 0:
                nl = bytes(data[: 1 << 20]).find(b"\n")
                if nl < 0 and len(data) > (1 << 20):
                    nl = bytes(data).find(b"\n")
                data = data[nl + 1:] if nl >= 0 else b""
            if len(data):
                yield fi, off, data


def parquet_text(path, plan) -> bytes:
    """A parquet part as delimited text lines (string form of every value; nulls as empty fields)."""
    import pyarrow.parquet as pq
    t = pq.read_table(path)
    cols = []
    for h in plan.header:
        if h in t.column_names:
            cols.append(["" if v is None else str(v) for v in t.column(h).to_pylist()])
        else:
            cols.append([""] * t.num_rows)
    lines = (plan.delim.join(r) for r in zip(*cols))
    return ("\n".join(lines) + "\n").encode() if t.num_rows else b""


def format_fields(fields, n: int, sep: str = "|"):
    """``n`` rows of (kind, values[, dictionary]) fields -> ('\\n'-terminated lines, int64 ends)."""
    import ctypes
    lib = _rt()
    ncols = len(fields)
    keep, cols, blobs, offs, dn, kinds = [], [], [], [], [], []
    for f in fields:
        kind, v = f[0], f[1]
        if kind == DICT:
            v = np.ascontiguousarray(v, dtype=np.int32)
            enc = [str(x).encode("utf-8") for x in f[2]]
            blob = np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8)
            off = np.zeros(len(enc) + 1, np.int64)
            if enc:
                off[1:] = np.cumsum([len(e) for e in enc])
            keep += [v, blob, off]
            blobs.append(blob.ctypes.data)
            offs.append(off.ctypes.data)
            dn.append(len(enc))
        else:
            v = np.ascontiguousarray(v, dtype=np.float64)
            keep.append(v)
            blobs.append(None)
            offs.append(None)
            dn.append(0)
        cols.append(v.ctypes.data)
        kinds.append(kind)
    ends = np.zeros(n, np.int64)
    sb = sep.encode()
    widest = sum(max((len(str(x).encode("utf-8")) for x in f[2]), default=0) for f in fields if f[0] == DICT)
    cap = max(1024, n * (ncols * (26 + len(sb)) + 16 + widest))
    while True:
        buf = np.empty(cap, np.uint8)
        got = lib.shifu_format_rows_sep(n, ncols, (ctypes.c_int * ncols)(*kinds), (ctypes.c_void_p * ncols)(*cols),
                                        (ctypes.c_void_p * ncols)(*blobs), (ctypes.c_void_p * ncols)(*offs),
                                        (ctypes.c_long * ncols)(*dn), buf.ctypes.data, cap, ends.ctypes.data, sb,
                                        len(sb))
        if got >= 0:
            return buf[:got], ends
        cap *= 2


def join_block(data, sep: str, nf: int, suffix, ends: np.ndarray, n: int, nthreads: int = 8) -> memoryview:
    """The block's non-blank lines, each cut/padded to ``nf`` fields, + ``sep`` + suffix line i
    (``suffix``: bytes or a uint8 array) -> a view of the joined bytes."""
    lib = _rt()
    arr = np.frombuffer(data, dtype=np.uint8)
    sb = sep.encode()
    sfx = np.frombuffer(suffix, dtype=np.uint8) if isinstance(suffix, (bytes, bytearray)) else suffix
    if not len(sfx):
        sfx = np.zeros(1, np.uint8)
    ends = np.ascontiguousarray(ends, dtype=np.int64)
    cap = len(arr) + len(sfx) + n * (nf + 2) * len(sb) + 1024
    while True:
        out = np.empty(cap, np.uint8)
        got = lib.shifu_join_lines(arr.ctypes.data, len(arr), sb, len(sb), nf, sfx.ctypes.data, ends.ctypes.data,
                                   n, out.ctypes.data, cap, int(nthreads))
        if got >= 0:
            return memoryview(out[:got])
        if got == -2:
            raise RuntimeError(f"row join: the block does not hold the {n} rows its parse produced")
        cap *= 2


STATS: dict = {}          # cumulative seconds per stage of stream_join (tools/join_lab.py)


def _tick(st, key, t0):
    t = time.perf_counter()
    st[key] = st.get(key, 0.0) + t - t0
    return t


def stream_join(plan, out_dir: str, new_names: list, parse_kinds: list, compute, rank: int = 0, world: int = 1,
                block_bytes: int = BLOCK_BYTES, nthreads: int | None = None) -> int:
    """Write this rank's rows of ``plan``'s data set + the columns ``compute(table, n)`` returns
    (a list of format fields, one per name in ``new_names``) to ``out_dir/part-<rank>``; rank 0
    (re)creates ``out_dir`` and writes ``.pig_header`` (header + new names, data delimiter).
    ``parse_kinds``: per header column 0 skip / 1 numeric / 2 string (what ``compute`` reads).
    Returns this rank's row count.  Collective when world > 1."""
    from ..parallel import dist
    from .reader import parse_block, table_from_parts
    sep = plan.delim or "|"
    nf = len(plan.header)
    nthreads = nthreads or min(16, os.cpu_count() or 4)
    if rank == 0:
        os.makedirs(out_dir, exist_ok=True)
        for f in os.listdir(out_dir):
            if f.startswith("part-") or f == ".pig_header":
                os.remove(os.path.join(out_dir, f))
        with open(os.path.join(out_dir, ".pig_header"), "w") as f:
            f.write(sep.join(list(plan.header) + list(new_names)) + "\n")
    if world > 1:
        dist.barrier()
    from concurrent.futures import ThreadPoolExecutor
    from .stream import prefetched
    rows = 0
    st = STATS
    # the next block is read on a background thread and finished blocks are written on another:
    # three block buffers (being read, queued, being joined), two joined blocks in flight
    blocks = prefetched(lambda: raw_blocks(plan, rank, world, block_bytes, nbuf=3), 1)
    pending = []
    t = time.perf_counter()
    with open(os.path.join(out_dir, f"part-{rank:05d}"), "wb") as out, ThreadPoolExecutor(1) as wr:
        for _, _, data in blocks:
            t = _tick(st, "read", t)
            part = parse_block(data, sep, parse_kinds, plan.missing, nthreads)
            n = int(part[0])
            if not n:
                continue
            table = table_from_parts(plan.header, parse_kinds, [part], plan.data_path)
            t = _tick(st, "parse", t)
            fields = compute(table, n)
            t = _tick(st, "compute", t)
            suffix, ends = format_fields(fields, n, sep)
            t = _tick(st, "format", t)
            joined = join_block(data, sep, nf, suffix, ends, n, nthreads)
            t = _tick(st, "join", t)
            while len(pending) >= 2:
                pending.pop(0).result()
            pending.append(wr.submit(out.write, joined))
            del joined
            t = _tick(st, "write", t)
            rows += n
        for f in pending:
            f.result()
    if world > 1:
        dist.barrier()
    _log.info("join: rank %d wrote %d rows + %d columns -> %s", rank, rows, len(new_names), out_dir)
    return rows
