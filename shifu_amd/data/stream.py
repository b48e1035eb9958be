"""Streamed, per-rank data reading (out-of-core stats / per-rank parsing).

The reference streams rows through Hadoop input splits: every mapper parses only its own byte
range of the part files (``UpdateBinningInfoMapper`` J/core/binning/UpdateBinningInfoMapper.java:
349-599 over ``CombineInputFormat`` splits; Guagua workers over ``GuaguaLineRecordReader``).  Here:

* the plain-text files of a data set form one global byte space; rank ``r`` of ``W`` owns
  ``[T*r/W, T*(r+1)/W)`` and every line whose first byte falls in that range (a line straddling
  a boundary belongs to the rank where it starts) -- so ranks partition the rows exactly, in file
  order, and never parse each other's bytes.  ``.gz`` / ``.parquet`` files are indivisible units
  dealt round-robin by file index;
* a rank reads its range in blocks of ``chunk_bytes`` (cut at line ends), parses each block with
  the native parser and yields a purified :class:`ModelData` chunk, so host memory is bounded by
  one block plus its parsed columns, whatever the data set size.

Sampling (``stats.sampleRate``) draws from a generator seeded by (seed, file, block offset), so
every pass over the stream sees the same rows.
"""
from __future__ import annotations

import gzip
import os

from .purifier import DatasetPlan, finish_table
from .reader import column_kinds, list_data_files, parse_block, table_from_parts, _parse_parquet

DEFAULT_CHUNK_BYTES = 256 << 20


def _units(files):
    plain = [f for f in files if not (f.endswith(".gz") or f.endswith(".parquet"))]
    whole = [f for f in files if f.endswith(".gz") or f.endswith(".parquet")]
    return plain, whole


def byte_ranges(files, rank: int = 0, world: int = 1):
    """-> list of (file index, path, start, end) byte ranges of the plain files owned by ``rank``
    plus (file index, path, None, None) for the whole (gz/parquet) files it owns."""
    plain, whole = _units(files)
    sizes = [os.path.getsize(f) for f in plain]
    total = sum(sizes)
    lo, hi = total * rank // world, total * (rank + 1) // world
    out = []
    off = 0
    for f, sz in zip(plain, sizes):
        a, b = max(lo, off), min(hi, off + sz)
        if a < b:
            out.append((files.index(f), f, a - off, b - off))
        off += sz
    for k, f in enumerate(whole):
        if k % world == rank:
            out.append((files.index(f), f, None, None))
    return sorted(out)


def _lines_in_range(path: str, start: int, end: int, chunk_bytes: int):
    """Yield (offset, bytes) blocks of complete lines whose first byte lies in [start, end)."""
    with open(path, "rb") as fh:
        pos = start
        if start > 0:
            fh.seek(start - 1)
            if fh.read(1) != b"\n":           # mid-line: that line belongs to the previous range
                rest = fh.readline()
                pos = start + len(rest)
        fh.seek(pos)
        carry = b""
        while pos < end:
            blk = fh.read(chunk_bytes)
            if not blk:
                if carry:
                    yield pos, carry
                return
            buf = carry + blk
            cut = buf.rfind(b"\n")
            if cut < 0:
                carry = buf
                continue
            lines, carry = buf[:cut + 1], buf[cut + 1:]
            if pos + len(lines) > end:            # stop after the line that starts before `end`
                i = lines.find(b"\n", max(0, end - pos - 1))
                lines = lines[:i + 1]
                yield pos, lines
                return
            yield pos, lines
            pos += len(lines)


def iter_tables(plan: DatasetPlan, chunk_bytes: int = DEFAULT_CHUNK_BYTES, rank: int = 0, world: int = 1,
                nthreads: int | None = None):
    """Yield (key, RawTable) row chunks of this rank's share of the data set, in file order."""
    files = list_data_files(plan.data_path)
    if not files:
        raise FileNotFoundError(f"no data under {plan.data_path}")
    kinds = column_kinds(plan.header, plan.nums, plan.strs)
    nthreads = nthreads or min(16, os.cpu_count() or 4)
    for fi, path, a, b in byte_ranges(files, rank, world):
        if a is None:                              # indivisible unit
            if path.endswith(".parquet"):
                part = _parse_parquet(path, plan.header, kinds, plan.missing)
            else:
                with gzip.open(path, "rb") as fh:
                    data = fh.read()
                if plan.skip_header_line and fi == 0:
                    nl = data.find(b"\n")
                    data = data[nl + 1:] if nl >= 0 else b""
                part = parse_block(data, plan.delim, kinds, plan.missing, nthreads)
            yield (fi, 0), table_from_parts(plan.header, kinds, [part], path)
            continue
        for off, data in _lines_in_range(path, a, b, chunk_bytes):
            if plan.skip_header_line and fi == 0 and off == 0:
                nl = data.find(b"\n")
                data = data[nl + 1:] if nl >= 0 else b""
                if not data:
                    continue
            part = parse_block(data, plan.delim, kinds, plan.missing, nthreads)
            yield (fi, off), table_from_parts(plan.header, kinds, [part], path)


def iter_model_data(mc, plan: DatasetPlan, chunk_bytes: int = DEFAULT_CHUNK_BYTES, rank: int = 0, world: int = 1,
                    sample_rate: float = 1.0, sample_neg_only: bool = False, seed: int = 0,
                    require_target: bool = True):
    """Yield purified :class:`ModelData` chunks of this rank's byte range."""
    for (fi, off), table in iter_tables(plan, chunk_bytes, rank, world):
        md = finish_table(mc, plan, table, sample_rate, sample_neg_only, [seed, fi, off], require_target)
        if md.n:
            yield md


def data_bytes(plan: DatasetPlan) -> int:
    return sum(os.path.getsize(f) for f in list_data_files(plan.data_path))
