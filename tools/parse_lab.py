"""Throughput of each stage of the streamed text path (data/stream.py + data/gpu_parse.py) on a
generated '|'-delimited data set: block reads (pinned, parallel preads), the host framing parse
(meta columns only), the full host parse, the H2D copy and the GPU field parser.

    python tools/parse_lab.py [--rows 1000000] [--cols 1600] [--chunk-mb 256] [--threads 4]
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--cols", type=int, default=1600)
    ap.add_argument("--chunk-mb", type=int, default=256)
    ap.add_argument("--threads", type=int, nargs="*", default=[1, 4, 8])
    a = ap.parse_args()
    import numpy as np
    import torch
    from shifu_amd.data import stream as DS
    from shifu_amd.data.gpu_parse import GpuBlockParser
    from shifu_amd.data.reader import parse_block
    from shifu_amd.ops import _native as nat
    work = os.path.join(tempfile.gettempdir(), "shifu_parse_lab")
    shutil.rmtree(work, ignore_errors=True)
    os.makedirs(work)
    t0 = time.perf_counter()
    if nat.rt().shifu_gen_csv(work.encode(), a.rows, a.cols, 3, 11, 0.02, 20, 16):
        raise SystemExit("generation failed")
    files = sorted(os.path.join(work, f) for f in os.listdir(work) if not f.startswith("."))
    total = sum(os.path.getsize(f) for f in files)
    res = {"rows": a.rows, "cols": a.cols, "text_gb": total / 1e9, "gen_s": time.perf_counter() - t0}
    ncols = 3 + a.cols + 3
    chunk = a.chunk_mb << 20
    kinds_meta = [0] * ncols
    kinds_meta[1] = 2                                      # target
    kinds_meta[2] = 1                                      # weight
    for j in range(3):
        kinds_meta[3 + a.cols + j] = 2                     # categoricals
    kinds_all = list(kinds_meta)
    for j in range(a.cols):
        kinds_all[3 + j] = 1

    def blocks(pinned):
        for f in files:
            yield from DS._lines_in_range(f, 0, os.path.getsize(f), chunk, nbuf=1, pinned=pinned)

    def timed(name, fn):
        t = time.perf_counter()
        n = fn()
        dt = time.perf_counter() - t
        res[name] = {"s": round(dt, 3), "GB_per_s": round(total / dt / 1e9, 2), "n": n}
        print(name, res[name], flush=True)

    for th in a.threads:
        DS.READ_THREADS = th
        timed(f"read_pinned_t{th}", lambda: sum(len(b) for _, b in blocks(True)))
    DS.READ_THREADS = 4
    timed("read_bytearray_t4", lambda: sum(len(b) for _, b in blocks(False)))
    timed("host_parse_meta_only", lambda: sum(parse_block(b, "|", kinds_meta, ["", "?"], 16)[0] for _, b in blocks(True)))
    timed("host_parse_all", lambda: sum(parse_block(b, "|", kinds_all, ["", "?"], 16)[0] for _, b in blocks(True)))
    dev = torch.device("cuda", 0)
    gp = GpuBlockParser(kinds_all, [3 + j for j in range(a.cols)], "|", ["", "?"], dev)

    def h2d():
        n = 0
        for _, b in blocks(True):
            t = torch.from_numpy(np.frombuffer(b, np.uint8))
            d = torch.empty(len(b), dtype=torch.uint8, device=dev)
            d.copy_(t)
            n += len(b)
        torch.cuda.synchronize()
        return n
    timed("read_plus_h2d", h2d)

    def gpu_parse():
        n = 0
        for _, b in blocks(True):
            n += gp.parse(b, 16)[0]
        torch.cuda.synchronize()
        return n
    timed("read_plus_gpu_parse", gpu_parse)
    # kernel alone on one block
    blk = next(iter(blocks(True)))[1]
    L = len(blk)
    d = torch.empty(L + 64, dtype=torch.uint8, device=dev)
    d[:L].copy_(torch.from_numpy(np.frombuffer(blk, np.uint8)))
    ends = torch.nonzero(d[:L] == 10).flatten()
    starts = torch.zeros_like(ends)
    starts[1:] = ends[:-1] + 1
    nl = int(ends.numel())
    vals = torch.empty((a.cols, nl), dtype=torch.float64, device=dev)
    lf = torch.empty(nl, dtype=torch.int32, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for it in range(3):
        gp.fb_n.zero_()
        e0.record()
        nat.call_hip("shifu_csv_gpu_parse", d, starts, ends, nl, gp.slot, ncols, vals, nl, lf, gp.fb, 1 << 20, gp.fb_n,
                     ord("|"), gp.ntok, gp.toks, None, None, nat.stream_of(d))
        e1.record()
        torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    res["gpu_kernel_one_block"] = {"bytes": L, "lines": nl, "ms": round(ms, 3), "GB_per_s": round(L / ms / 1e6, 1)}
    print("gpu_kernel_one_block", res["gpu_kernel_one_block"], flush=True)
    e0.record()
    torch.nonzero(d[:L] == 10)
    e1.record()
    torch.cuda.synchronize()
    res["newline_index_ms"] = round(e0.elapsed_time(e1), 3)
    print(json.dumps(res))
    shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
