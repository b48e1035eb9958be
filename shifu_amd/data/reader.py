"""Delimited data reader (L1, D2/D3/E3 replacement).

* headers: ``headerPath`` (``.pig_header``), or the data file's first line when no header file
  is given (``InitModelProcessor.initColumnConfigList`` J/core/processor/InitModelProcessor.java:424-502)
* data: a file, a directory of part files (hidden ``.``/``_`` files skipped, ``.gz`` inflated),
  or a glob (``ShifuFileUtils`` / ``PathFinder`` semantics)
* parsing: the native multithreaded C++ parser (``runtime/csrc/csv_parser.cpp``) into a columnar
  :class:`RawTable`; pure-Python fallback for environments without a toolchain.
"""
from __future__ import annotations

import ctypes
import glob
import gzip
import io
import os
from dataclasses import dataclass, field

import numpy as np

from ..utils.log import get_logger

_log = get_logger("data.reader")


def read_column_name_file(path: str) -> list:
    """Column-name files: one name per line, '#' comments, blank lines ignored; a line may hold
    several names separated by ','."""
    if not path or not os.path.isfile(path):
        return []
    out = []
    with open(path, encoding="utf-8") as f:
        for line in f:
            line = line.strip()
            if not line or line.startswith("#"):
                continue
            for n in line.split(","):
                if n.strip():
                    out.append(n.strip())
    return out


def list_data_files(path: str) -> list:
    if path is None:
        return []
    if any(ch in path for ch in "*?[") and not os.path.exists(path):
        files = sorted(glob.glob(path))
    elif os.path.isdir(path):
        files = sorted(os.path.join(path, f) for f in os.listdir(path)
                       if not f.startswith(".") and not f.startswith("_"))
        files = [f for f in files if os.path.isfile(f)]
    elif os.path.isfile(path):
        files = [path]
    else:
        files = []
    return files


def _read_bytes(path: str) -> bytes:
    if path.endswith(".gz"):
        with gzip.open(path, "rb") as f:
            return f.read()
    with open(path, "rb") as f:
        return f.read()


def _first_line(path: str, limit: int = 1 << 24) -> str:
    """First non-blank line of a (possibly gzipped) text file, reading only what it needs."""
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rb") as f:
        for _ in range(1 << 20):
            line = f.readline(limit)
            if not line:
                return ""
            if line.strip():
                return line.decode("utf-8", errors="replace").rstrip("\r\n")
    return ""


def read_header(header_path: str | None, header_delim: str = "|", data_path: str | None = None,
                data_delim: str = "|") -> list:
    if header_path:
        files = list_data_files(header_path)
        if files:
            return [h.strip() for h in _first_line(files[0]).split(header_delim or "|")]
    files = list_data_files(data_path)
    if not files:
        raise FileNotFoundError(f"no header file and no data under {data_path}")
    if files[0].endswith(".parquet"):           # schema carries the header
        import pyarrow.parquet as pq
        return list(pq.read_schema(files[0]).names)
    return [h.strip() for h in _first_line(files[0]).split(data_delim or "|")]


class Column:
    """One parsed column: ``values`` float64 (num, NaN = missing) | int32 codes (str, -1 =
    missing).  A numeric column parsed on the GPU (data/gpu_parse.py) carries ``dev`` (its row of
    a device block) and materializes host ``values`` only when asked."""
    __slots__ = ("name", "kind", "_values", "dictionary", "dev")

    def __init__(self, name: str, kind: str, values=None, dictionary=None, dev=None):
        self.name, self.kind, self._values = name, kind, values
        self.dictionary = dictionary if dictionary is not None else []
        self.dev = dev

    @property
    def values(self) -> np.ndarray:
        if self._values is None and self.dev is not None:
            self._values = self.dev.host()
        return self._values

    @values.setter
    def values(self, v):
        self._values, self.dev = v, None

    def __len__(self):
        return len(self.dev) if self._values is None and self.dev is not None else len(self._values)

    def strings(self) -> np.ndarray:
        if self.kind == "str":
            d = np.array(self.dictionary + [""], dtype=object)
            return d[np.where(self.values >= 0, self.values, len(self.dictionary))]
        out = np.array([("" if v != v else _java_num_str(v)) for v in self.values], dtype=object)
        return out

    def numeric(self) -> np.ndarray:
        if self.kind == "num":
            return self.values
        lut = np.full(len(self.dictionary) + 1, np.nan)
        for i, s in enumerate(self.dictionary):
            try:
                lut[i] = float(s)
            except ValueError:
                pass
        return lut[np.where(self.values >= 0, self.values, len(self.dictionary))]

    def missing_mask(self) -> np.ndarray:
        return np.isnan(self.values) if self.kind == "num" else self.values < 0

    def slice(self, a: int, b: int) -> "Column":
        """Rows [a, b) (a view of the values, same dictionary)."""
        return Column(self.name, self.kind, self.values[a:b], self.dictionary)


def _java_num_str(v: float) -> str:
    """A parsed numeric value as text (shortest round-trip digits, like Double.toString for the
    common range); a numpy scalar is converted first (numpy 2's repr is 'np.float64(...)')."""
    return repr(float(v))


@dataclass
class RawTable:
    header: list
    columns: dict                     # name -> Column (only parsed columns)
    n: int
    bad_rows: int = 0

    def __getitem__(self, name) -> Column:
        return self.columns[name]

    def __contains__(self, name):
        return name in self.columns

    def take(self, idx: np.ndarray) -> "RawTable":
        cols, blocks = {}, {}
        for k, c in self.columns.items():
            if c._values is None and c.dev is not None:      # GPU-parsed: gather each block once
                from .gpu_parse import DevRef
                b = c.dev.block
                if id(b) not in blocks:
                    blocks[id(b)] = b.take(idx)
                cols[k] = Column(c.name, c.kind, dev=DevRef(blocks[id(b)], c.dev.row))
            else:
                cols[k] = Column(c.name, c.kind, c.values[idx], c.dictionary)
        return RawTable(self.header, cols, int(len(idx)) if idx.dtype != bool else int(idx.sum()), self.bad_rows)


def _parse_native(data: bytes, delim: str, kinds: list, missing: list, nthreads: int):
    from ..ops import _native
    lib = _native.rt()
    if lib is None:
        return None
    kinds_arr = (ctypes.c_int * len(kinds))(*kinds)
    miss = "\n".join(missing).encode("utf-8")
    if isinstance(data, bytes):              # immutable: parse it in place (no copy of the block)
        buf = data
        addr = ctypes.cast(ctypes.c_char_p(data), ctypes.c_void_p).value
    elif isinstance(data, memoryview) and not data.readonly and data.contiguous and len(data):
        buf = data                           # a block of a read buffer (data/stream.py): in place
        addr = ctypes.addressof(ctypes.c_char.from_buffer(data))
    else:
        buf = ctypes.create_string_buffer(bytes(data), len(data))
        addr = ctypes.addressof(buf)
    h = lib.shifu_csv_scan(addr, len(data), delim.encode("utf-8"), len(kinds), kinds_arr, miss, nthreads)
    if not h:
        return None
    try:
        n = lib.shifu_csv_nrows(h)
        # numeric columns are parsed straight into the rows of ONE column-major matrix: each
        # column is a row view, and consumers that need several columns as a matrix (normalize,
        # stats uploads) use the rows in place (see ``numeric_rows``) instead of gathering them
        num_ci = [ci for ci, k in enumerate(kinds) if k == 1]
        M = np.empty((len(num_ci), n), dtype=np.float64)
        if lib.shifu_csv_fill(h, M.ctypes.data if M.size else None, max(n, 1)) != 0:
            return None
        bad = lib.shifu_csv_bad_rows(h)
        out = {}
        for r, ci in enumerate(num_ci):
            out[ci] = ("num", M[r], [])
        for ci, k in enumerate(kinds):
            if k == 1:
                continue
            elif k == 2:
                a = np.empty(n, dtype=np.int32)
                lib.shifu_csv_codes(h, ci, a.ctypes.data)
                need = lib.shifu_csv_dict(h, ci, None, 0)
                sz = lib.shifu_csv_dict_size(h, ci)
                if sz > 0:
                    b = ctypes.create_string_buffer(max(1, need))
                    lib.shifu_csv_dict(h, ci, b, need)
                    d = b.raw[:need].decode("utf-8", errors="replace").split("\n")
                else:
                    d = []
                out[ci] = ("str", a, d)
        return n, bad, out
    finally:
        lib.shifu_csv_free(h)


def _parse_python(data: bytes, delim: str, kinds: list, missing: list):
    text = bytes(data).decode("utf-8", errors="replace")
    lines = [l for l in text.split("\n") if l.strip()]
    n = len(lines)
    miss = set(m.strip() for m in missing)
    cols = {ci: [] for ci, k in enumerate(kinds) if k}
    bad = 0
    for line in lines:
        parts = line.split(delim)
        if len(parts) != len(kinds):
            bad += 1
        for ci in cols:
            v = parts[ci].strip() if ci < len(parts) else ""
            cols[ci].append(v)
    out = {}
    for ci, vals in cols.items():
        if kinds[ci] == 1:
            a = np.empty(n)
            for i, v in enumerate(vals):
                if v in miss:
                    a[i] = np.nan
                    continue
                try:
                    a[i] = float(v.rstrip("dDfF")) if v else np.nan
                except ValueError:
                    a[i] = np.nan
            out[ci] = ("num", a, [])
        else:
            d, codes = {}, np.empty(n, dtype=np.int32)
            for i, v in enumerate(vals):
                if v in miss:
                    codes[i] = -1
                else:
                    codes[i] = d.setdefault(v, len(d))
            out[ci] = ("str", codes, list(d.keys()))
    return n, bad, out


def _parse_parquet(path: str, header: list, kinds: list, missing: list):
    """Parquet part file (D3: GuaguaParquetRecordReader, column projection): only the requested
    columns are read; numeric -> float64 (NaN missing), string -> dictionary codes."""
    import pyarrow.parquet as pq
    names = [h for h, k in zip(header, kinds) if k]
    tbl = pq.read_table(path, columns=[n for n in names if n in pq.read_schema(path).names])
    n = tbl.num_rows
    miss = set(missing)
    out = [None] * len(header)
    for ci, (h, k) in enumerate(zip(header, kinds)):
        if not k:
            continue
        if h not in tbl.column_names:
            out[ci] = ("num", np.full(n, np.nan), []) if k == 1 else ("str", np.full(n, -1, np.int32), [])
            continue
        col = tbl.column(h).to_pylist()
        if k == 1:
            a = np.empty(n, dtype=np.float64)
            for i, v in enumerate(col):
                try:
                    a[i] = float(v) if v is not None and str(v) not in miss else np.nan
                except (TypeError, ValueError):
                    a[i] = np.nan
            out[ci] = ("num", a, [])
        else:
            d, codes = {}, np.empty(n, dtype=np.int32)
            for i, v in enumerate(col):
                s = "" if v is None else str(v)
                codes[i] = -1 if s in miss else d.setdefault(s, len(d))
            out[ci] = ("str", codes, list(d.keys()))
    return n, 0, out


def numeric_rows(arrays: list):
    """If every array is a full row of one C-contiguous 2-D float64 matrix (the parser's
    column-major block, see ``_parse_native``) -> (matrix, row indices); else None."""
    if not arrays:
        return None
    base = arrays[0].base
    if not isinstance(base, np.ndarray) or base.ndim != 2 or base.dtype != np.float64 \
            or not base.flags.c_contiguous or base.shape[1] != len(arrays[0]):
        return None
    p0, rb = base.ctypes.data, base.strides[0]
    idx = np.empty(len(arrays), dtype=np.int64)
    for j, a in enumerate(arrays):
        if a.base is not base or a.dtype != np.float64 or a.ndim != 1 or a.strides[0] != 8:
            return None
        off = a.ctypes.data - p0
        if off % rb or len(a) != base.shape[1]:
            return None
        idx[j] = off // rb
    return base, idx


def column_kinds(header: list, numeric: list | None = None, strings: list | None = None) -> list:
    """Per header column: 1 numeric, 2 string, 0 skipped (by default every column is a string)."""
    idx = {h: i for i, h in enumerate(header)}
    kinds = [0] * len(header)
    for nm in numeric or []:
        if nm in idx:
            kinds[idx[nm]] = 1
    for nm in (strings if strings is not None else ([] if numeric else header)):
        if nm in idx:
            kinds[idx[nm]] = 2
    return kinds


def parse_block(data: bytes, delim: str, kinds: list, missing: list, nthreads: int):
    """One in-memory block of complete lines -> (n, bad, {column index: (kind, values, dict)})."""
    res = _parse_native(data, delim or "|", kinds, missing, nthreads)
    if res is None:
        res = _parse_python(data, delim or "|", kinds, missing)
    return res


def table_from_parts(header: list, kinds: list, parts: list, data_path: str = "") -> RawTable:
    """Concatenate parsed parts (file order) into a RawTable; string dictionaries are merged in
    first-appearance order."""
    n = sum(p[0] for p in parts)
    bad = sum(p[1] for p in parts)
    cols = {}
    for ci, k in enumerate(kinds):
        if not k:
            continue
        name = header[ci]
        if k == 1:
            if len(parts) == 1 and not isinstance(parts[0][2][ci][1], np.ndarray):
                cols[name] = Column(name, "num", dev=parts[0][2][ci][1])   # GPU-parsed (DevRef)
                continue
            arrs = [p[2][ci][1] if isinstance(p[2][ci][1], np.ndarray) else p[2][ci][1].host() for p in parts]
            if len(arrs) == 1:              # one parsed block: its array as is (no copy)
                vals = arrs[0]
            else:
                vals = np.concatenate(arrs) if arrs else np.empty(0)
            cols[name] = Column(name, "num", vals)
        else:
            gdict, remapped = {}, []
            for p in parts:
                _, codes, d = p[2][ci]
                lut = np.array([gdict.setdefault(s, len(gdict)) for s in d] + [-1], dtype=np.int32)
                remapped.append(lut[np.where(codes >= 0, codes, len(d))])
            cols[name] = Column(name, "str", np.concatenate(remapped) if remapped else np.empty(0, np.int32),
                                list(gdict.keys()))
    if bad:
        _log.warning("%d rows under %s have a column count != %d (padded as missing)", bad, data_path,
                     len(header))
    return RawTable(header, cols, n, bad)


def read_table(data_path: str, header: list, delim: str = "|", numeric: list | None = None,
               strings: list | None = None, missing: list | None = None, skip_header_line: bool = False,
               nthreads: int | None = None, max_rows: int | None = None) -> RawTable:
    """Parse every file under ``data_path`` into a columnar table.  ``numeric``/``strings``
    are column names (others skipped); by default every column is parsed as a string.
    (Out-of-core / per-rank byte ranges: ``data/stream.py``.)"""
    files = list_data_files(data_path)
    if not files:
        raise FileNotFoundError(f"no data under {data_path}")
    kinds = column_kinds(header, numeric, strings)
    missing = list(missing) if missing is not None else ["", "?"]
    nthreads = nthreads or min(16, os.cpu_count() or 4)
    parts = []
    for fi, f in enumerate(files):
        if f.endswith(".parquet"):
            parts.append(_parse_parquet(f, header, kinds, missing))
            continue
        data = _read_bytes(f)
        if skip_header_line and fi == 0:
            nl = data.find(b"\n")
            data = data[nl + 1:] if nl >= 0 else b""
        parts.append(parse_block(data, delim, kinds, missing, nthreads))
    t = table_from_parts(header, kinds, parts, data_path)
    if max_rows is not None and t.n > max_rows:
        for c in t.columns.values():
            c.values = c.values[:max_rows]
        t.n = max_rows
    return t


def first_line_is_header(data_path: str, header: list, delim: str) -> bool:
    """Data files that start with their own header line (no separate header file)."""
    files = list_data_files(data_path)
    if not files or files[0].endswith(".parquet"):
        return False
    return [h.strip() for h in _first_line(files[0]).split(delim)] == header
