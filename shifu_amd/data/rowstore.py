"""Out-of-core row stores for the step caches (NormalizedData / CleanedData / eval scores).

SURVEY §5.7: ``norm`` and ``eval`` stream a rank's byte range chunk by chunk (the reference
streams rows through Pig, ``P/Normalize.pig:35-46`` / ``P/Eval.pig:29-41``), so a cache is
written without its row count known in advance and without the whole shard in host memory:

* :class:`NpyAppender` appends row blocks to a ``.npy`` file whose header reserves room for the
  final shape and is rewritten on close (a plain ``np.load``-able file, memory-mappable).
* a data-parallel cache is one ``part-RRRRR/`` directory per rank plus a top-level
  ``meta.json`` listing ``parts`` and their row counts; :class:`RowParts` presents the parts
  of one array as a single row-indexable array (slices copy only the rows they touch), so
  training's row shards and chunk streams read straight from the part files.
"""
from __future__ import annotations

import json
import os

import numpy as np

HEADER_BYTES = 256          # reserved .npy header: magic + version + len + dict, padded to 256


def _header(dtype: np.dtype, shape: tuple) -> bytes:
    d = {"descr": np.lib.format.dtype_to_descr(np.dtype(dtype)), "fortran_order": False, "shape": tuple(shape)}
    body = repr(d).encode("latin1")
    head = b"\x93NUMPY\x01\x00"
    room = HEADER_BYTES - len(head) - 2
    if len(body) + 1 > room:
        raise ValueError("npy header does not fit the reserved space")
    body = body + b" " * (room - len(body) - 1) + b"\n"
    return head + len(body).to_bytes(2, "little") + body


class NpyAppender:
    """Append ``[k, *row_shape]`` blocks of one dtype to ``path``; ``close()`` fixes the header.
    Blocks of >= 64 MB are written as ``WRITE_THREADS`` concurrent pwrites at their offsets (one
    writer thread copies a few GB/s into the page cache / tmpfs; a 1600-column bf16 chunk is
    ~0.5 GB)."""

    WRITE_THREADS = int(os.environ.get("SHIFU_WRITE_THREADS", "4"))

    def __init__(self, path: str, dtype, row_shape: tuple = ()):
        self.path, self.dtype, self.row_shape = path, np.dtype(dtype), tuple(row_shape)
        self.rows = 0
        self.fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
        self._pwrite(_header(self.dtype, (0,) + self.row_shape), 0)
        self.off = HEADER_BYTES

    def _pwrite(self, mv, off: int) -> None:
        mv = memoryview(mv)
        while len(mv):
            k = os.pwrite(self.fd, mv, off)
            mv, off = mv[k:], off + k

    def append(self, a) -> None:
        a = np.ascontiguousarray(a, dtype=self.dtype)
        if a.shape[1:] != self.row_shape:
            raise ValueError(f"{self.path}: row shape {a.shape[1:]} != {self.row_shape}")
        mv = memoryview(a.reshape(-1).view(np.uint8)) if a.size else memoryview(b"")   # no tobytes() copy
        n = len(mv)
        nt = self.WRITE_THREADS if n >= (64 << 20) else 1
        if nt <= 1:
            self._pwrite(mv, self.off)
        else:
            from concurrent.futures import ThreadPoolExecutor
            cuts = [n * i // nt for i in range(nt + 1)]
            with ThreadPoolExecutor(nt) as ex:
                list(ex.map(lambda i: self._pwrite(mv[cuts[i]:cuts[i + 1]], self.off + cuts[i]), range(nt)))
        self.off += n
        self.rows += a.shape[0]

    def close(self) -> int:
        if self.fd is not None:
            self._pwrite(_header(self.dtype, (self.rows,) + self.row_shape), 0)
            os.close(self.fd)
            self.fd = None
        return self.rows

    def abort(self) -> None:
        if self.fd is not None:
            os.close(self.fd)
            self.fd = None
        if os.path.exists(self.path):
            os.remove(self.path)


SEG = "@"                  # segment files of one array: <name>@<k:06d>.npy, rows in k order


def _write_npy(path: str, a: np.ndarray) -> None:
    """One whole .npy file (reserved-size header + the rows) with pwrite, no temporary copy."""
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    try:
        os.pwrite(fd, _header(a.dtype, a.shape), 0)
        mv = memoryview(a.reshape(-1).view(np.uint8)) if a.size else memoryview(b"")
        off = HEADER_BYTES
        while len(mv):
            k = os.pwrite(fd, mv, off)
            mv, off = mv[k:], off + k
    finally:
        os.close(fd)


class SegmentAppender:
    """Append ``[k, *row_shape]`` blocks as a sequence of segment files ``<name>@<k>.npy`` in one
    directory.  A large block is cut into ``SPLIT`` row slices written by as many threads, each
    into its own file: tmpfs serialises the writers of one inode (one file took ~5.7 GB/s on the
    GPU box whatever the thread count; 4 / 8 files at once 21 / 36 GB/s,
    profiles/r5/write_lab_shm_r5.txt).  Readers concatenate the segments in name order
    (:func:`part_arrays`)."""

    SPLIT = int(os.environ.get("SHIFU_WRITE_SPLIT", "8"))
    MIN_SPLIT_BYTES = 64 << 20                   # smaller blocks go out as one file

    def __init__(self, dirpath: str, name: str, dtype, row_shape: tuple = ()):
        self.dir, self.name = dirpath, name
        self.dtype, self.row_shape = np.dtype(dtype), tuple(row_shape)
        self.rows, self.k = 0, 0
        self._pool = None
        for fn in os.listdir(dirpath):            # a rewrite replaces every old segment
            if fn.startswith(name + SEG) and fn.endswith(".npy"):
                os.remove(os.path.join(dirpath, fn))

    def _path(self, k: int) -> str:
        return os.path.join(self.dir, f"{self.name}{SEG}{k:06d}.npy")

    def append(self, a) -> None:
        a = np.ascontiguousarray(a, dtype=self.dtype)
        if a.shape[1:] != self.row_shape:
            raise ValueError(f"{self.name}: row shape {a.shape[1:]} != {self.row_shape}")
        if not len(a):
            return
        ns = max(1, min(self.SPLIT, len(a))) if a.nbytes >= self.MIN_SPLIT_BYTES else 1
        cuts = [len(a) * i // ns for i in range(ns + 1)]
        jobs = [(self._path(self.k + i), a[cuts[i]:cuts[i + 1]]) for i in range(ns)]
        self.k += ns
        if ns == 1:
            _write_npy(*jobs[0])
        else:
            if self._pool is None:
                from concurrent.futures import ThreadPoolExecutor
                self._pool = ThreadPoolExecutor(self.SPLIT, thread_name_prefix="shifu-seg-write")
            list(self._pool.map(lambda j: _write_npy(*j), jobs))
        self.rows += len(a)

    def close(self) -> int:
        if self.k == 0:                           # an empty array still names its segment
            _write_npy(self._path(0), np.empty((0,) + self.row_shape, self.dtype))
            self.k = 1
        if self._pool is not None:
            self._pool.shutdown()
            self._pool = None
        return self.rows

    def abort(self) -> None:
        if self._pool is not None:
            self._pool.shutdown()
            self._pool = None
        for fn in os.listdir(self.dir):
            if fn.startswith(self.name + SEG) and fn.endswith(".npy"):
                os.remove(os.path.join(self.dir, fn))


def part_names(pdir: str) -> list:
    """Array names in a part directory (plain ``<name>.npy`` or segmented ``<name>@<k>.npy``)."""
    return sorted({fn[:-4].split(SEG)[0] for fn in os.listdir(pdir) if fn.endswith(".npy")})


def part_arrays(pdir: str, name: str, mmap: bool = True) -> list:
    """The arrays holding ``name`` in a part directory, in row order (segments opened by a
    thread pool: a 20M-row cache has a few thousand)."""
    mode = "r" if mmap else None
    one = os.path.join(pdir, f"{name}.npy")
    if os.path.exists(one):
        return [np.load(one, mmap_mode=mode)]
    segs = sorted(fn for fn in os.listdir(pdir) if fn.startswith(name + SEG) and fn.endswith(".npy"))
    if len(segs) < 64:
        return [np.load(os.path.join(pdir, fn), mmap_mode=mode) for fn in segs]
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(8) as ex:
        return list(ex.map(lambda fn: np.load(os.path.join(pdir, fn), mmap_mode=mode), segs))


class RowParts:
    """Row-wise concatenation of memory-mapped part arrays (same dtype / trailing shape).

    Supports ``len``, ``shape``, ``dtype``, ``ndim``, basic row slices (``a[lo:hi]``, ``a[lo:hi, cols]``),
    integer / boolean row indexing, and ``np.asarray`` (which materialises every row)."""

    def __init__(self, parts: list):
        if not parts:
            raise ValueError("RowParts needs at least one part")
        self.parts = parts
        self.offsets = np.cumsum([0] + [len(p) for p in parts])
        self.dtype = parts[0].dtype
        self.shape = (int(self.offsets[-1]),) + tuple(parts[0].shape[1:])
        self.ndim = len(self.shape)

    def __len__(self):
        return self.shape[0]

    @property
    def nbytes(self) -> int:
        return int(np.prod(self.shape)) * self.dtype.itemsize

    def _rows(self, lo: int, hi: int):
        """Views of the parts covering rows [lo, hi), in order."""
        out = []
        k0 = max(0, int(np.searchsorted(self.offsets, lo, side="right")) - 1)
        for k in range(k0, len(self.parts)):
            if self.offsets[k] >= hi:
                break
            a, b = max(lo, self.offsets[k]), min(hi, self.offsets[k + 1])
            if a < b:
                out.append(self.parts[k][a - self.offsets[k]: b - self.offsets[k]])
        return out

    blocks = _rows

    def __getitem__(self, idx):
        rest = ()
        if isinstance(idx, tuple):
            idx, rest = idx[0], idx[1:]
        if isinstance(idx, slice):
            lo, hi, step = idx.indices(len(self))
            if step != 1:
                return self[np.arange(lo, hi, step)][(slice(None),) + rest] if rest else self[np.arange(lo, hi, step)]
            blocks = self._rows(lo, hi)
            if len(blocks) == 1:
                out = blocks[0]
            elif blocks:
                out = np.concatenate(blocks)
            else:
                out = np.empty((0,) + self.shape[1:], self.dtype)
        elif isinstance(idx, (int, np.integer)):
            i = int(idx) + (len(self) if idx < 0 else 0)
            k = int(np.searchsorted(self.offsets, i, side="right") - 1)
            out = self.parts[k][i - self.offsets[k]]
        else:
            ix = np.asarray(idx)
            if ix.dtype == bool:
                ix = np.nonzero(ix)[0]
            out = np.empty((len(ix),) + self.shape[1:], self.dtype)
            k = np.searchsorted(self.offsets, ix, side="right") - 1
            for pk in np.unique(k):
                sel = k == pk
                out[sel] = self.parts[pk][ix[sel] - self.offsets[pk]]
        return out[(slice(None),) + rest] if rest else out

    def __array__(self, dtype=None, copy=None):
        a = self[0: len(self)]
        a = np.array(a) if not isinstance(a, np.ndarray) or isinstance(a, np.memmap) else a
        return a.astype(dtype) if dtype is not None else a


def write_parts_meta(path: str, meta: dict, part_rows: list) -> None:
    """Top-level meta.json of a partitioned cache (rank 0, after every rank closed its part)."""
    parts = [{"dir": f"part-{r:05d}", "n": int(n)} for r, n in enumerate(part_rows)]
    meta = dict(meta, n=int(sum(part_rows)), parts=parts)
    tmp = os.path.join(path, ".meta.json.tmp")
    with open(tmp, "w") as f:
        json.dump(meta, f, indent=1)
    os.replace(tmp, os.path.join(path, "meta.json"))


def load_parts(path: str, meta: dict, mmap: bool = True) -> dict:
    """name -> RowParts (or the single part's array) of a partitioned cache."""
    arrays = {}
    parts = [p for p in meta["parts"] if p["n"] > 0] or meta["parts"][:1]
    names = sorted({nm for p in parts for nm in part_names(os.path.join(path, p["dir"]))})
    for name in names:
        arrs = [x for p in parts for x in part_arrays(os.path.join(path, p["dir"]), name, mmap)]
        arrays[name] = arrs[0] if len(arrs) == 1 else RowParts(arrs)
    return arrays


class Bf16Rows:
    """Float view of a bf16 GEMM-ready NormalizedData matrix (``Xb``: uint16 bf16 bits
    [n, kpad], values in the first ``width`` columns, bias column 1.0 at ``width``).  Row /
    column indexing returns float32 values of the input columns; ``raw`` is the padded
    bf16 matrix that the MLP trainer streams to HBM without any cast or padding pass.
    ``cols``: the raw columns this view exposes (a model's input subset, :meth:`subset`);
    :meth:`device_rows` moves the bf16 bits to the GPU as they are (no host fp32 expansion)."""

    COPY_THREADS = int(os.environ.get("SHIFU_COPY_THREADS", "8"))
    LAST_STATS: dict = {}                        # device_rows: allocation / host copy / DMA wait seconds

    def __init__(self, raw, width: int, cols=None):
        self.raw = raw
        self.cols = None if cols is None else np.asarray(cols, dtype=np.int64)
        self.width = int(width) if self.cols is None else len(self.cols)
        self.shape = (len(raw), self.width)
        self.dtype = np.dtype(np.float32)
        self.ndim = 2

    def __len__(self):
        return self.shape[0]

    @property
    def nbytes(self) -> int:
        return self.shape[0] * self.width * 4

    @staticmethod
    def to_f32(u16) -> np.ndarray:
        u = np.ascontiguousarray(u16, dtype=np.uint16)
        return (u.astype(np.uint32) << 16).view(np.float32)

    def subset(self, idx) -> "Bf16Rows":
        """The view of input columns ``idx`` (positions in this view)."""
        base = np.arange(self.width) if self.cols is None else self.cols
        return Bf16Rows(self.raw, len(idx), base[np.asarray(idx, dtype=np.int64)])

    def device_rows(self, device, rows=None, block: int = 1 << 18):
        """bf16 torch tensor [len(rows), width] on ``device``: the raw bits are uploaded in row
        blocks (``rows``: optional SORTED row index array, gathered on the device) and the
        columns picked on the device.  ``COPY_THREADS`` > 0 (``SHIFU_COPY_THREADS``): each block
        is copied by that many threads into one of two page-locked buffers and sent with an async
        H2D on a copy stream, so the host copy of block i + 1 overlaps the DMA of block i:
        50 GB/s from a /dev/shm cache with 8 threads against 13.6 GB/s for the plain pageable
        upload (``COPY_THREADS = 0``; profiles/r4/upload_lab_r4n.txt)."""
        return self.device_rows_multi(device, [rows], block)[0]

    def device_rows_multi(self, device, row_sets, block: int = 1 << 18) -> list:
        """:meth:`device_rows` for several SORTED row sets (None = every row) in ONE pass over the
        host rows: each block is copied and uploaded once and every set gathers its rows from it
        (the training and validation rows of a split are one read of the cache, not two)."""
        import time
        import torch
        st = {"alloc_s": 0.0, "copy_s": 0.0, "wait_s": 0.0, "blocks": 0}
        Bf16Rows.LAST_STATS = st
        t_a = time.perf_counter()
        n = len(self.raw)
        dev = torch.device(device)
        sets = [None if r is None else np.asarray(r, dtype=np.int64) for r in row_sets]
        outs = [torch.empty((n if r is None else len(r), self.width), dtype=torch.bfloat16, device=dev) for r in sets]
        st["alloc_s"] = time.perf_counter() - t_a
        cols_d = None if self.cols is None else torch.as_tensor(self.cols, device=dev)
        gpu = dev.type == "cuda" and self.COPY_THREADS > 0
        if gpu:
            kp = self.raw.shape[1]
            pins = [torch.empty(block * kp, dtype=torch.int16, pin_memory=True) for _ in range(2)]
            # two device staging blocks reused in turn (a fresh 0.8 GB allocation per block kept
            # the caching allocator busy): the copy stream waits until the main stream is done
            # with a block's previous contents before the next DMA into it
            dbufs = [torch.empty((min(block, n), kp), dtype=torch.int16, device=dev) for _ in range(2)]
            used = [None, None]
            evs = [None, None]
            cstream = torch.cuda.Stream(dev)
            main = torch.cuda.current_stream(dev)
            from concurrent.futures import ThreadPoolExecutor
            pool = ThreadPoolExecutor(self.COPY_THREADS)
        los, i = [0] * len(sets), 0
        try:
            for b0 in range(0, n, block):
                b1 = min(n, b0 + block)
                sels = []
                r0, r1 = b1, b0
                for r in sets:
                    if r is None:
                        sels.append(None)
                        r0, r1 = b0, b1
                        continue
                    a_, c_ = np.searchsorted(r, b0), np.searchsorted(r, b1)
                    sels.append(r[a_:c_])
                    if c_ > a_:
                        r0, r1 = min(r0, int(r[a_])), max(r1, int(r[c_ - 1]) + 1)
                if r1 <= r0:
                    continue
                if gpu:
                    k = i & 1
                    i += 1
                    t_w = time.perf_counter()
                    if evs[k] is not None:
                        evs[k].synchronize()          # the DMA that last read this buffer is done
                    t_c = time.perf_counter()
                    st["wait_s"] += t_c - t_w
                    st["blocks"] += 1
                    h = pins[k][: (r1 - r0) * kp].numpy().reshape(r1 - r0, kp)
                    # (dst row, source view) pieces: a segmented cache's slice is several views;
                    # each piece is cut over the copy threads (never concatenated first)
                    srcs = self.raw.blocks(r0, r1) if hasattr(self.raw, "blocks") else [self.raw[r0:r1]]
                    jobs, d0 = [], 0
                    for sv in srcs:
                        sv = sv.view(np.int16)
                        cuts = np.linspace(0, len(sv), self.COPY_THREADS + 1).astype(np.int64)
                        jobs += [(d0 + int(cuts[t]), sv[cuts[t]:cuts[t + 1]]) for t in range(self.COPY_THREADS)
                                 if cuts[t + 1] > cuts[t]]
                        d0 += len(sv)
                    list(pool.map(lambda j: np.copyto(h[j[0]: j[0] + len(j[1])], j[1]), jobs))
                    st["copy_s"] += time.perf_counter() - t_c
                    with torch.cuda.stream(cstream):
                        if used[k] is not None:
                            cstream.wait_event(used[k])
                        blk = dbufs[k][: r1 - r0]
                        blk.copy_(pins[k][: (r1 - r0) * kp].view(r1 - r0, kp), non_blocking=True)
                        evs[k] = torch.cuda.Event()
                        evs[k].record(cstream)
                    main.wait_event(evs[k])
                else:
                    blk = torch.as_tensor(np.ascontiguousarray(self.raw[r0:r1]).view(np.int16), device=dev)
                blk = blk.view(torch.bfloat16)
                for s_, sel in enumerate(sels):
                    if sel is not None and not len(sel):
                        continue
                    if sel is None:
                        part = blk[b0 - r0: b1 - r0]
                    else:
                        ix = torch.from_numpy(sel - r0)
                        ix = ix.pin_memory().to(dev, non_blocking=True) if gpu else ix.to(dev)
                        part = blk.index_select(0, ix)
                    part = part[:, : self.width] if cols_d is None else part.index_select(1, cols_d)
                    outs[s_][los[s_]: los[s_] + len(part)] = part
                    los[s_] += len(part)
                if gpu:
                    used[k] = torch.cuda.Event()
                    used[k].record(main)
        finally:
            if gpu:
                pool.shutdown()
                for e in evs + used:
                    if e is not None:
                        e.synchronize()
        return outs

    def __getitem__(self, idx):
        rest = ()
        if isinstance(idx, tuple):
            idx, rest = idx[0], idx[1:]
        rows = self.raw[idx]
        out = self.to_f32(rows[..., : self.width] if self.cols is None else rows[..., self.cols])
        return out[(slice(None),) + rest] if rest else out

    def __array__(self, dtype=None, copy=None):
        a = self[0: len(self)]
        return a.astype(dtype) if dtype is not None else a
