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

Sampling (``*.sampleRate``) is a counter-based draw per global raw row (``purifier.row_uniform``):
a row's decision is the same whole, chunked or split over ranks (plain-text files; gz / parquet
units dealt round-robin keep their rank-local row numbering).
"""
from __future__ import annotations

import gzip
import os
import threading
import time

from .purifier import DatasetPlan, finish_table
from .reader import column_kinds, list_data_files, parse_block, table_from_parts, _parse_parquet

DEFAULT_CHUNK_BYTES = 256 << 20
PREFETCH_READ = int(os.environ.get("SHIFU_READ_PREFETCH", "1"))   # blocks read ahead of the parse
PREFETCH_UPLOAD = int(os.environ.get("SHIFU_UPLOAD_PREFETCH", "1"))   # uploaded blocks queued for the parse


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


READ_THREADS = int(os.environ.get("SHIFU_READ_THREADS", "8"))   # parallel preads per block
# SHIFU_STREAM_TRACE=1: every pipeline stage appends (stage, thread, t_start, t_end) per block to
# TRACE (tools/stream_trace_lab.py turns them into a per-stage overlap table)
TRACE_ON = os.environ.get("SHIFU_STREAM_TRACE") == "1"
TRACE: list = []


class _span:
    __slots__ = ("stage", "t0")

    def __init__(self, stage):
        self.stage = stage

    def __enter__(self):
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        if TRACE_ON:
            TRACE.append((self.stage, threading.current_thread().name, self.t0, time.perf_counter()))
        return False
READ_STATS = {"read_s": 0.0, "bytes": 0}          # cumulative pread time / bytes (logged per pass)


def _pread_into(fd: int, mv, off: int, want: int) -> int:
    """Fill ``mv[:want]`` from file offset ``off`` -> bytes read (short only at end of file).
    Blocks of >= 32 MB are read as READ_THREADS concurrent preads (page-cache copies run at a few
    GB/s per thread; one block of a 1600-column text is ~256 MB)."""
    def one(a, b):
        got = 0
        while a + got < b:
            r = os.preadv(fd, [mv[a + got: b]], off + a + got)
            if not r:
                break
            got += r
        return got
    nt = READ_THREADS if want >= (32 << 20) else 1
    if nt <= 1:
        return one(0, want)
    from concurrent.futures import ThreadPoolExecutor
    cuts = [want * i // nt for i in range(nt + 1)]
    with ThreadPoolExecutor(nt) as ex:
        got = list(ex.map(lambda i: one(cuts[i], cuts[i + 1]), range(nt)))
    total = 0
    for i, g in enumerate(got):
        total += g
        if g < cuts[i + 1] - cuts[i]:
            break
    return total


def _find_nl(buf, lo: int, hi: int, last: bool) -> int:
    """First (``last``: last) '\n' in buf[lo:hi] -> index or -1 (bytearray or uint8 ndarray)."""
    if isinstance(buf, bytearray):
        return buf.rfind(b"\n", lo, hi) if last else buf.find(b"\n", lo, hi)
    import numpy as np
    step = 1 << 16
    if last:
        b = hi
        while b > lo:
            a = max(lo, b - step)
            idx = np.flatnonzero(buf[a:b] == 10)
            if len(idx):
                return a + int(idx[-1])
            b, step = a, step * 2
    else:
        a = lo
        while a < hi:
            b = min(hi, a + step)
            idx = np.flatnonzero(buf[a:b] == 10)
            if len(idx):
                return a + int(idx[0])
            a, step = b, step * 2
    return -1


_PIN_POOL: list = []            # page-locked block buffers kept for the process (see _new_buf)
_PIN_LOCK = threading.Lock()


def _new_buf(n: int, pinned: bool):
    """A block buffer of >= n bytes.  Page-locked buffers come from a process-wide pool and are
    sized to whole 64 MiB steps: pinning 1 GB takes ~0.3 s and holds a HIP runtime lock that stalls
    every other thread's kernel launches (rocprofv3 trace, profiles/r4/NOTES_r4.md), so a pass must
    not allocate one per file or whenever a block's carried line makes it a few KB bigger.  A pooled
    buffer is handed out again only when nothing else references it (no reader, no block view
    still queued or being parsed downstream)."""
    if not pinned:
        return bytearray(n)
    import sys
    n = -(-n // (64 << 20)) * (64 << 20)
    with _PIN_LOCK:
        for arr in _PIN_POOL:
            # references: the pool list, this loop variable, getrefcount's argument
            if len(arr) >= n and sys.getrefcount(arr) <= 3:
                return arr
        import torch
        # the ndarray's base holds the tensor's storage: views of a block keep its pages alive
        arr = torch.empty(n, dtype=torch.uint8, pin_memory=True).numpy()
        _PIN_POOL.append(arr)
        return arr


def _lines_in_range(path: str, start: int, end: int, chunk_bytes: int, nbuf: int = 1, pinned: bool = False):
    """Yield (offset, block) blocks of complete lines whose first byte lies in [start, end).

    Blocks are memoryviews into ``nbuf`` rotating buffers, filled by (parallel) preads (no copy of
    the text): a block stays valid until ``nbuf - 1`` further blocks have been produced (1: until
    the next is requested).  ``pinned``: the buffers are page-locked host memory (uint8 ndarrays
    of pinned torch tensors) so a GPU parse can DMA a block straight to HBM."""
    bufs = [None] * max(1, nbuf)
    k = 0
    fd = os.open(path, os.O_RDONLY)
    try:
        pos = start
        if start > 0:
            if os.pread(fd, 1, start - 1) != b"\n":     # mid-line: that line belongs to the previous range
                with open(path, "rb") as fl:
                    fl.seek(start)
                    pos = start + len(fl.readline())
        carry = b""
        while pos < end:
            # never read (much) past the range: the line straddling `end` is completed by the
            # small follow-up reads of the carry logic
            want = min(chunk_bytes, max(end - pos - len(carry), 0) + (1 << 16))
            if pinned:                         # device-parse blocks: carry + read < the parser's limit
                from .gpu_parse import BLOCK_LIMIT
                want = max(1, min(want, BLOCK_LIMIT - 1 - len(carry)))
            need = len(carry) + want
            buf = bufs[k]
            if buf is None or len(buf) < need:
                buf = bufs[k] = _new_buf(need + (1 << 16), pinned)   # sized to the block
            mv = memoryview(buf)
            c = len(carry)
            mv[:c] = carry
            t_read = time.perf_counter()
            got = _pread_into(fd, mv[c:], pos + c, want)
            READ_STATS["read_s"] += time.perf_counter() - t_read
            READ_STATS["bytes"] += got
            filled = c + got
            if got == 0:
                if carry:
                    yield pos, mv[:c]
                return
            cut = _find_nl(buf, 0, filled, last=True)
            if cut < 0:
                carry = bytes(mv[:filled])     # one line longer than the block: read on
                continue
            carry = bytes(mv[cut + 1:filled])
            k = (k + 1) % len(bufs)
            if pos + cut + 1 > end:           # stop after the line that starts before `end`
                i = _find_nl(buf, max(0, end - pos - 1), filled, last=False)
                yield pos, mv[:i + 1]
                return
            yield pos, mv[:cut + 1]
            pos += cut + 1
    finally:
        os.close(fd)


def _iter_parts(plan: DatasetPlan, chunk_bytes: int, rank: int, world: int, kinds: list, nthreads: int,
                resume=None, gpu=None):
    """Yield ((file index, offset), parsed part) for this rank's share, in file order.  ``resume``
    = (file index, offset) of a block yielded by an earlier pass: start there (earlier blocks are
    neither read nor parsed; an offset is always a line start).  ``gpu``: a
    :class:`~.gpu_parse.GpuBlockParser` -- plain-text blocks are read into page-locked buffers and
    its columns parsed on the device."""
    pinned = gpu is not None and gpu.usable
    parse = (lambda data: gpu.parse(data, nthreads)) if pinned else \
        (lambda data: parse_block(data, plan.delim, kinds, plan.missing, nthreads))
    files = list_data_files(plan.data_path)
    if not files:
        raise FileNotFoundError(f"no data under {plan.data_path}")
    units = []
    for fi, path, a, b in byte_ranges(files, rank, world):
        if resume is not None:
            if fi < resume[0]:
                continue
            if fi == resume[0] and a is not None:
                a = max(a, resume[1])
                if a >= b:
                    continue
        units.append((fi, path, a, b))

    # ONE read | upload | parse pipeline over all of the rank's units, so the stages stay busy
    # across file boundaries (a pipeline per file drained and refilled at every part file:
    # tools/stream_trace_lab.py).  The reads run on their own thread, PREFETCH_READ blocks ahead
    # (preads and the native parser release the GIL); PREFETCH_READ + 2 rotating buffers per file
    # (+2 more with the GPU upload stage in between: block k's buffer is refilled only after
    # block k has been parsed).  An indivisible unit (gz / parquet) passes through as a marker
    # and is parsed whole on the host, in order.
    def blocks():
        for fi, path, a, b in units:
            if a is None:
                yield (fi, 0, path), None
                continue
            it = _lines_in_range(path, a, b, chunk_bytes,
                                 nbuf=PREFETCH_READ + (3 + PREFETCH_UPLOAD if pinned else 2), pinned=pinned)
            while True:
                with _span("read"):
                    nxt = next(it, None)
                if nxt is None:
                    break
                off, data = nxt
                if plan.skip_header_line and fi == 0 and off == 0:
                    nl = bytes(data[: 1 << 20]).find(b"\n")
                    if nl < 0 and len(data) > (1 << 20):      # a header line wider than 1 MiB
                        nl = bytes(data).find(b"\n")
                    data = data[nl + 1:] if nl >= 0 else b""
                    if not len(data):
                        continue
                yield (fi, off, None), data

    def whole_unit(fi, path):
        if path.endswith(".parquet"):
            return _parse_parquet(path, plan.header, kinds, plan.missing)
        with gzip.open(path, "rb") as fh:
            data = fh.read()
        if plan.skip_header_line and fi == 0:
            nl = data.find(b"\n")
            data = data[nl + 1:] if nl >= 0 else b""
        return parse_block(data, plan.delim, kinds, plan.missing, nthreads)

    src = prefetched(blocks, PREFETCH_READ) if PREFETCH_READ > 0 else blocks()
    if pinned:
        for (fi, off, path), data, dbuf in prefetched(lambda: gpu.uploads(src), PREFETCH_UPLOAD):
            if data is None:
                yield (fi, 0), whole_unit(fi, path)
                continue
            with _span("parse"):
                part = gpu.parse(data, nthreads, dbuf)
            yield (fi, off), part
    else:
        for (fi, off, path), data in src:
            if data is None:
                yield (fi, 0), whole_unit(fi, path)
                continue
            with _span("parse"):
                part = parse(data)
            yield (fi, off), part


def gpu_parser(plan: DatasetPlan, gpu_cols, dev):
    """A GpuBlockParser for the numeric plan columns named in ``gpu_cols`` (minus the weight and
    the filter / segment expression inputs, which the purifier reads on the host), or None when
    GPU parsing is off (``shifu.data.gpuParse``) or nothing qualifies."""
    if not gpu_cols or dev is None or plan.seg_names:
        return None
    from . import gpu_parse as G
    if not G.enabled(dev):
        return None
    kinds = column_kinds(plan.header, plan.nums, plan.strs)
    skip = set()
    if plan.weight:
        skip.add(plan.weight)
    from .expr import Evaluator
    for e in (plan.filt, plan.weight):
        if e and str(e).strip():
            try:
                skip |= set(Evaluator(str(e)).columns())
            except Exception:
                pass
    want = set(gpu_cols) - skip
    idx = [i for i, h in enumerate(plan.header) if h in want and kinds[i] == 1]
    if not idx:
        return None
    p = G.GpuBlockParser(kinds, idx, plan.delim, plan.missing, dev)
    return p if p.usable else None


def iter_tables(plan: DatasetPlan, chunk_bytes: int = DEFAULT_CHUNK_BYTES, rank: int = 0, world: int = 1,
                nthreads: int | None = None, resume=None, gpu=None):
    """Yield (key, RawTable) row chunks of this rank's share of the data set, in file order
    (``gpu``: see :func:`_iter_parts`)."""
    kinds = column_kinds(plan.header, plan.nums, plan.strs)
    nthreads = nthreads or min(16, os.cpu_count() or 4)
    for key, part in _iter_parts(plan, chunk_bytes, rank, world, kinds, nthreads, resume, gpu):
        yield key, table_from_parts(plan.header, kinds, [part], plan.data_path)


def count_rows(plan: DatasetPlan, rank: int = 0, world: int = 1, chunk_bytes: int = DEFAULT_CHUNK_BYTES) -> int:
    """Raw data rows in this rank's share (a parse with no columns selected: row framing only)."""
    kinds = [0] * len(plan.header)
    return int(sum(p[0] for _, p in _iter_parts(plan, chunk_bytes, rank, world, kinds, min(16, os.cpu_count() or 4))))


def rank_row_offset(plan: DatasetPlan, rank: int, world: int) -> int:
    """Global raw-row index of this rank's first row (row counts all-gathered over ranks)."""
    if world <= 1:
        return 0
    import torch
    from ..parallel import dist
    counts = dist.all_gather_objects(count_rows(plan, rank, world))
    return int(sum(counts[:rank]))


class _Raised:
    def __init__(self, exc):
        self.exc = exc


def prefetched(gen_fn, depth: int = 2):
    """Run the generator ``gen_fn()`` on a background thread, ``depth`` items ahead of the
    consumer: the next chunk's file read + native parse (both release the GIL) overlap the
    consumer's uploads and kernels on the current one.  Exceptions re-raise in the consumer;
    closing the consumer stops the producer."""
    import queue
    import threading
    if depth <= 0:
        yield from gen_fn()
        return
    q = queue.Queue(maxsize=depth)
    stop = threading.Event()
    end = object()

    def put(item):
        while not stop.is_set():
            try:
                q.put(item, timeout=0.1)
                return True
            except queue.Full:
                continue
        return False

    def run():
        try:
            for item in gen_fn():
                if not put(item):
                    return
            put(end)
        except BaseException as e:          # noqa: BLE001 - handed to the consumer
            put(_Raised(e))
    t = threading.Thread(target=run, name="shifu-prefetch", daemon=True)
    t.start()
    try:
        while True:
            item = q.get()
            if item is end:
                break
            if isinstance(item, _Raised):
                raise item.exc
            yield item
    finally:
        stop.set()
        while t.is_alive():
            try:
                q.get_nowait()
            except queue.Empty:
                t.join(0.05)


def iter_model_data(mc, plan: DatasetPlan, chunk_bytes: int = DEFAULT_CHUNK_BYTES, rank: int = 0, world: int = 1,
                    sample_rate: float = 1.0, sample_neg_only: bool = False, seed: int = 0,
                    require_target: bool = True, row0: int = 0, resume=None, with_keys: bool = False,
                    gpu_cols=None, dev=None):
    """Yield purified :class:`ModelData` chunks of this rank's byte range; ``row0`` = the global
    raw-row index of the rank's first row (sampling draws are per global row).  Chunks are
    produced ``shifu.data.prefetch`` (default 1) ahead on a background thread.

    ``with_keys``: yield (key, md) with key = (file index, offset, raw row index of the block),
    which a later pass hands back as ``resume`` to start at that block (stats passes whose first
    blocks are cached in HBM re-parse only the rest).

    ``gpu_cols`` + ``dev``: those numeric columns are parsed on the GPU (data/gpu_parse.py) and
    stay in HBM as device-block rows (``gpu_parse.device_rows``)."""
    from ..config import environment
    gp = gpu_parser(plan, gpu_cols, dev)
    sw = os.environ.get("SHIFU_GIL_SWITCH_MS")
    if gp is not None and sw:
        # reader / upload / parse / consumer threads hand the GIL over after every C call: a short
        # switch interval keeps a thread coming back from a pread or a DMA from waiting a whole
        # interval (5 ms default) behind another thread's Python work
        import sys
        sys.setswitchinterval(float(sw) / 1e3)

    def produce():
        r = row0 if resume is None else resume[2]
        r0 = dict(READ_STATS)
        t0 = time.perf_counter()
        for key, table in iter_tables(plan, chunk_bytes, rank, world,
                                      resume=None if resume is None else resume[:2], gpu=gp):
            n = table.n
            with _span("purify"):
                md = finish_table(mc, plan, table, sample_rate, sample_neg_only, seed, require_target, r)
            k = (key[0], key[1], r)
            r += n
            if md.n:
                yield (k, md) if with_keys else md
        if gp is not None:
            from ..utils.log import get_logger
            rd = READ_STATS["read_s"] - r0["read_s"]
            gb = (READ_STATS["bytes"] - r0["bytes"]) / 1e9
            get_logger("data.stream").info("%s; reads %.2fs (%.1f GB); pass %.2fs", gp.summary(), rd, gb,
                                           time.perf_counter() - t0)
    yield from prefetched(produce, int(environment.get("shifu.data.prefetch", 1)))


def load_rank_dataset(mc, data_conf, columns_num=None, columns_str=None, sample_rate=1.0, sample_neg_only=False,
                      seed=0, require_target=True, extra_filter=None, rank: int = 0, world: int = 1):
    """This rank's rows only (its byte ranges, parsed block by block into one table) -- the
    data-parallel replacement of parse-everything-then-slice; equals the rank's contiguous slice
    of ``load_dataset`` over the whole data set, sampling included."""
    from .purifier import plan_dataset
    plan = plan_dataset(mc, data_conf, columns_num, columns_str, extra_filter)
    row0 = rank_row_offset(plan, rank, world) if (world > 1 and sample_rate < 1.0) else 0
    kinds = column_kinds(plan.header, plan.nums, plan.strs)
    parts = [p for _, p in _iter_parts(plan, DEFAULT_CHUNK_BYTES, rank, world, kinds, min(16, os.cpu_count() or 4))]
    table = table_from_parts(plan.header, kinds, parts, plan.data_path)
    return finish_table(mc, plan, table, sample_rate, sample_neg_only, seed, require_target, row0)


def data_bytes(plan: DatasetPlan) -> int:
    return sum(os.path.getsize(f) for f in list_data_files(plan.data_path))
