"""GPU parse of text blocks (K0, host side of ``ops/csrc/csv_kernels.hip``).

SURVEY §7.1 choice 2 asks that the raw text stop being re-tokenized on the host for every step
(``stats``, ``norm``, ``eval``; the reference re-reads text per step: ``P/Normalize.pig:35-46``).
On a GPU run the bulk numeric columns of each block are parsed on the device instead:

1. the block reader (``data/stream._lines_in_range``) fills page-locked buffers with parallel
   preads, so a block goes to HBM as ONE DMA (``torch`` copy from pinned memory);
2. the host parser (``runtime/csrc/csv_parser.cpp``) runs over the same bytes with only the few
   "meta" columns requested (target, weight, filter / categorical columns): it frames the rows,
   counts bad rows and builds the string dictionaries, skipping the unparsed column runs with a
   16-byte delimiter count;
3. ``shifu_csv_gpu_parse`` tokenizes and converts every bulk numeric field (one wave per line) into
   a column-major fp64 block in HBM; fields outside the Clinger fast path come back as a short list
   the host finishes with its own strtod path (``shifu_parse_fields``), blank lines are dropped.

The result is bit-identical to the host parse (tests/test_gpu_parse.py).  Parsed columns stay in
HBM as :class:`DeviceBlock` rows: ``stats`` batches and the ``norm`` K5 pass read them in place
(``device_rows``); anything that asks for host values gets one D2H copy of the block.
"""
from __future__ import annotations

import ctypes
import time

import numpy as np

from ..utils.log import get_logger

_log = get_logger("data.gpu_parse")

# largest block the device parse takes: field bounds are int32 offsets into the block (+64 B pad)
BLOCK_LIMIT = (1 << 31) - 64
FB_CAP = 1 << 20          # fallback fields per block before the whole block is parsed on the host
MAX_TOKENS, TOKEN_BYTES = 8, 15


class DeviceBlock:
    """Numeric columns of one parsed block: ``D`` [k, n] fp64 in HBM; a host copy on demand."""
    __slots__ = ("D", "_host")

    def __init__(self, D):
        self.D = D
        self._host = None

    def host(self) -> np.ndarray:
        if self._host is None:
            self._host = self.D.cpu().numpy()
        return self._host

    def take(self, idx) -> "DeviceBlock":
        import torch
        idx = np.asarray(idx)
        if idx.dtype == bool:
            idx = np.flatnonzero(idx)
        return DeviceBlock(self.D.index_select(1, torch.as_tensor(idx, dtype=torch.long, device=self.D.device)))


class DevRef:
    """Row ``row`` of a :class:`DeviceBlock` (one column's values)."""
    __slots__ = ("block", "row")

    def __init__(self, block: DeviceBlock, row: int):
        self.block, self.row = block, row

    def host(self) -> np.ndarray:
        return self.block.host()[self.row]

    def tensor(self):
        return self.block.D[self.row]

    def __len__(self):
        return int(self.block.D.shape[1])


def device_rows(cols, dev):
    """[C, n] fp64 device tensor of the columns when all of them are rows of ONE device block on
    ``dev`` (a view for a consecutive run, else one gather), else None."""
    import torch
    refs = [getattr(c, "dev", None) if c is not None else None for c in cols]
    if not refs or any(r is None for r in refs):
        return None
    blk = refs[0].block
    want = torch.device(dev)
    if want.type == "cuda" and want.index is None:
        want = torch.device("cuda", torch.cuda.current_device())
    if any(r.block is not blk for r in refs) or blk.D.device != want:
        return None
    rows = [r.row for r in refs]
    if rows == list(range(rows[0], rows[0] + len(rows))):
        return blk.D[rows[0]: rows[0] + len(rows)]
    return blk.D.index_select(0, torch.as_tensor(rows, dtype=torch.long, device=blk.D.device))


def enabled(dev) -> bool:
    """``shifu.data.gpuParse`` (default auto: on for a CUDA device with the HIP library present)."""
    from ..config import environment
    mode = str(environment.get("shifu.data.gpuParse", "auto")).lower()
    if mode in ("false", "0", "off") or dev is None:
        return False
    import torch
    if torch.device(dev).type != "cuda":
        return False
    from ..ops import _native as nat
    if mode in ("true", "1", "on"):
        nat.hip()
        return True
    return nat.hip_available() and nat.rt() is not None


class GpuBlockParser:
    """Parses blocks with the numeric header columns ``gpu_cols`` on the device and the rest of
    ``kinds`` on the host.  ``usable`` is False when the data set's format needs the host parser
    throughout (multi-byte delimiter, more / longer missing tokens than the kernel holds)."""

    def __init__(self, kinds: list, gpu_cols: list, delim: str, missing: list, dev):
        import torch
        self.dev = torch.device(dev)
        self.kinds = list(kinds)
        self.gpu_cols = sorted(c for c in gpu_cols if kinds[c] == 1)
        self.kinds_host = list(kinds)
        for c in self.gpu_cols:
            self.kinds_host[c] = 0
        toks = []
        for t in missing:
            t = str(t).strip()
            if t and t not in toks:
                toks.append(t)
        enc = [t.encode("utf-8") for t in toks]
        d = (delim or "|").encode("utf-8")
        self.usable = (len(d) == 1 and d != b"\n" and len(enc) <= MAX_TOKENS and
                       all(len(t) <= TOKEN_BYTES and b"\0" not in t for t in enc) and bool(self.gpu_cols))
        self.delim, self.missing = delim or "|", list(missing)
        self.dbyte = d[0] if len(d) == 1 else 0
        self.toks = b"".join(t + b"\0" for t in enc)
        self.ntok = len(enc)
        slot = np.full(len(kinds), -1, np.int32)
        slot[self.gpu_cols] = np.arange(len(self.gpu_cols), dtype=np.int32)
        self.slot = torch.as_tensor(slot, device=self.dev)
        # the host-parsed columns: the kernel hands back their field bounds, the host parses just
        # those bytes (one short line per row) instead of scanning the whole block
        self.host_cols = [c for c, k in enumerate(self.kinds_host) if k]
        self.kinds_mini = [self.kinds_host[c] for c in self.host_cols] + [0]
        mslot = np.full(len(kinds), -1, np.int32)
        mslot[self.host_cols] = np.arange(len(self.host_cols), dtype=np.int32)
        self.mslot = torch.as_tensor(mslot, device=self.dev) if self.host_cols else None
        self.fb = torch.empty(4 * FB_CAP, dtype=torch.long, device=self.dev)
        self.fb_n = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self.stream = None
        self.h2d_stream = None
        self.stats = {"blocks": 0, "fallback_fields": 0, "host_blocks": 0, "bytes": 0}
        self.times = {"h2d": 0.0, "index": 0.0, "kernel": 0.0, "fallback": 0.0, "host_cols": 0.0}

    def uploads(self, blocks):
        """(key, block) -> (key, block, device copy of the block): the H2D stage of the streamed
        read (its own thread and stream; a copy is complete when yielded).  A None block (an
        indivisible gz / parquet unit) passes through."""
        import torch
        if self.h2d_stream is None:
            self.h2d_stream = torch.cuda.Stream(self.dev)
        for off, data in blocks:
            if data is None:
                yield off, None, None
                continue
            L = len(data)
            if L == 0 or L >= BLOCK_LIMIT:
                yield off, data, None
                continue
            t0 = time.perf_counter()
            with torch.cuda.device(self.dev), torch.cuda.stream(self.h2d_stream):
                dbuf = torch.empty(L + 64, dtype=torch.uint8, device=self.dev)
                dbuf[:L].copy_(torch.from_numpy(np.frombuffer(data, dtype=np.uint8)), non_blocking=True)
                self.h2d_stream.synchronize()
            t1 = time.perf_counter()
            self.times["h2d"] += t1 - t0
            from . import stream as _S
            if _S.TRACE_ON:
                _S.TRACE.append(("h2d", "upload", t0, t1))
            yield off, data, dbuf

    def parse(self, data, nthreads: int, dbuf=None):
        """``data``: a memoryview of complete lines inside a page-locked uint8 ndarray (or any
        buffer: then it is staged) -> the host parser's (n, bad, {column: (kind, values, dict)})
        with the GPU columns as ``("num", DevRef, [])``."""
        import torch
        from ..ops import _native as nat
        from .reader import parse_block
        # a reader thread: HIP's current device = ours, and a stream of its own, so the block's
        # host syncs wait for the parse only -- not for the consumer's kernels on the compute
        # stream (they overlap); the block is complete when handed over (stream synchronized)
        if self.stream is None:
            self.stream = torch.cuda.Stream(self.dev)
        with torch.cuda.device(self.dev), torch.cuda.stream(self.stream):
            if dbuf is not None:
                dbuf.record_stream(self.stream)     # the upload stage's block: reuse waits for us
            n, bad, out = self._parse(data, nthreads, dbuf)
            self.stream.synchronize()
        consumer = torch.cuda.default_stream(self.dev)
        for c in self.gpu_cols:
            ref = out[c][1]
            if isinstance(ref, DevRef):
                ref.block.D.record_stream(consumer)     # freed by the consumer: reuse waits for it
                break
        return n, bad, out

    def _parse(self, data, nthreads: int, dbuf=None):
        import torch
        from ..ops import _native as nat
        from .reader import parse_block
        data = memoryview(data)
        L = len(data)
        self.stats["blocks"] += 1
        if L == 0:
            return self._host_framing(data, nthreads, None)
        if L >= BLOCK_LIMIT:                     # field bounds are int32 block offsets
            self.stats["host_blocks"] += 1
            return parse_block(data, self.delim, self.kinds, self.missing, nthreads)
        T = self.times
        t0 = time.perf_counter()
        self.stats["bytes"] += L
        host = np.frombuffer(data, dtype=np.uint8)
        if dbuf is None:
            dbuf = torch.empty(L + 64, dtype=torch.uint8, device=self.dev)
            dbuf[:L].copy_(torch.from_numpy(host))
        t1 = time.perf_counter()
        T["h2d"] += t1 - t0
        ends = self._newlines(dbuf, L)
        if int(host[-1]) != 10:
            ends = torch.cat([ends, torch.tensor([L], dtype=torch.long, device=self.dev)])
        nl = int(ends.numel())
        starts = torch.zeros(nl, dtype=torch.long, device=self.dev)
        if nl > 1:
            starts[1:] = ends[:-1] + 1
        vals = torch.empty((len(self.gpu_cols), nl), dtype=torch.float64, device=self.dev)
        lflags = torch.empty(nl, dtype=torch.int32, device=self.dev)
        nh = len(self.host_cols)
        moffs = torch.empty((max(nh, 1), nl, 2), dtype=torch.int32, device=self.dev) if nh else None
        self.fb_n.zero_()
        t2 = time.perf_counter()
        T["index"] += t2 - t1
        nat.call_hip("shifu_csv_gpu_parse", dbuf, starts, ends, nl, self.slot, len(self.kinds), vals, nl, lflags,
                     self.fb, FB_CAP, self.fb_n, self.dbyte, self.ntok, self.toks, self.mslot, moffs,
                     nat.stream_of(dbuf))
        nfb = int(self.fb_n.item())
        t3 = time.perf_counter()
        T["kernel"] += t3 - t2
        if nfb > FB_CAP:                         # a mostly non-decimal block: host parse throughout
            self.stats["host_blocks"] += 1
            return parse_block(data, self.delim, self.kinds, self.missing, nthreads)
        addr = ctypes.addressof(ctypes.c_char.from_buffer(data)) if not data.readonly else host.ctypes.data
        if nfb:
            self.stats["fallback_fields"] += nfb
            fb = self.fb[: 4 * nfb].view(nfb, 4).cpu().numpy()
            fv = np.empty(nfb, np.float64)
            nat.rt().shifu_parse_fields(addr, fb.ctypes.data, nfb, fv.ctypes.data)
            fbt = torch.as_tensor(fb, device=self.dev)
            vals[fbt[:, 1], fbt[:, 0]] = torch.as_tensor(fv, device=self.dev)
        fl = lflags.cpu().numpy()
        t4 = time.perf_counter()
        T["fallback"] += t4 - t3
        blank = (fl & 1) != 0
        if blank.any():
            vals = vals[:, torch.as_tensor(np.flatnonzero(~blank), device=self.dev)]
        if ((fl & 2) != 0)[~blank].any():
            # rows with a field count != ncols: the host parser's short / long row rules throughout
            n, bad, out = self._host_framing(data, nthreads, vals)
        else:
            n, bad, out = int((~blank).sum()), 0, {}
            if nh:
                mo = moffs.cpu().numpy()
                # the kernel writes only column 0's bounds on a blank line: the other entries are
                # whatever the allocator left there, so they must not size the gather buffer
                if blank.any():
                    mo[:, blank, :] = 0
                cap =int(np.clip(mo[..., 1] - mo[..., 0], 0, None).sum()) + nl * (nh + 3)
                mini = np.empty(cap, np.uint8)
                nb = nat.rt().shifu_gather_fields(addr, mo.ctypes.data, nl, nh, fl.ctypes.data,
                                                  self.delim.encode(), mini.ctypes.data, cap)
                if nb < 0:
                    raise RuntimeError("GPU parse: gathering the host columns failed")
                n2, _, o2 = parse_block(memoryview(mini[:nb]), self.delim, self.kinds_mini, self.missing,
                                        max(1, min(nthreads, nb >> 20)))
                if n2 != n:
                    raise RuntimeError(f"GPU parse: {n} rows framed, {n2} host-column rows")
                out = {c: o2[j] for j, c in enumerate(self.host_cols)}
            self.stats["gathered_blocks"] = self.stats.get("gathered_blocks", 0) + 1
        if vals.shape[1] != n:
            raise RuntimeError(f"GPU parse framed {vals.shape[1]} rows, host parser {n}")
        T["host_cols"] += time.perf_counter() - t4
        blk = DeviceBlock(vals)
        out.update({c: ("num", DevRef(blk, j), []) for j, c in enumerate(self.gpu_cols)})
        return n, bad, out

    def _newlines(self, dbuf, L: int):
        """int64 positions of every '\\n' in dbuf[:L] (own kernels, csv_kernels.hip: segment
        counts, one scan, ordered writes; one host read of the count)."""
        import torch
        from ..ops import _native as nat
        h = nat.hip()
        need = int(h.shifu_newline_ws_bytes(L))
        if getattr(self, "_nl_ws", None) is None or self._nl_ws.numel() < need:
            self._nl_ws = torch.empty(need + 64, dtype=torch.uint8, device=self.dev)
        ws = self._nl_ws
        st = nat.stream_of(dbuf)
        nat.call_hip("shifu_newline_count", dbuf, L, ws, st)
        o = int(h.shifu_newline_count_offset(L))
        cnt = int(ws[o:o + 8].view(torch.int64).item())
        ends = torch.empty(cnt, dtype=torch.long, device=self.dev)
        if cnt:
            nat.call_hip("shifu_newline_write", dbuf, L, ws, ends, st)
        return ends

    def summary(self) -> str:
        s = self.stats
        tt = " ".join(f"{k} {v:.2f}s" for k, v in self.times.items())
        return (f"GPU parse: {s['blocks']} blocks, {s['bytes'] / 1e9:.1f} GB, {s['fallback_fields']} fallback fields, "
                f"{s['host_blocks']} host blocks; {tt}")

    def _host_framing(self, data, nthreads, vals):
        """The host parser over the whole block for the host columns (row framing, bad rows)."""
        import torch
        from .reader import parse_block
        n, bad, out = parse_block(data, self.delim, self.kinds_host, self.missing, nthreads)
        if vals is None:
            blk = DeviceBlock(torch.empty((len(self.gpu_cols), n), dtype=torch.float64, device=self.dev))
            if n:
                raise RuntimeError("GPU parse: rows without a device block")
            out.update({c: ("num", DevRef(blk, j), []) for j, c in enumerate(self.gpu_cols)})
        return n, bad, out
