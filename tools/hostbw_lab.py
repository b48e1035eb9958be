"""Is the streamed text pipeline coupled through host memory bandwidth?  

Measures, on one generated '|'-delimited text set (native generator, page-cache resident after
the first pass), each stage of the GPU-parse read path alone and then concurrently:

  pread   8-thread preads of 256 MiB blocks into pooled page-locked buffers (data/stream.py)
  h2d     hipMemcpyAsync of page-locked blocks to HBM (the upload thread)
  memcpy  a plain host memcpy between two large buffers (host DRAM bandwidth reference)
  pread+h2d, pread+memcpy, h2d+memcpy   two of them at once on separate threads

If pread and h2d each run near their own rates when concurrent, the host is not the coupling;
if the concurrent rate of each drops to about half, they share one host-memory budget.

    python tools/hostbw_lab.py [--rows 3000000] [--cols 1600] [--seconds 3]
"""
import argparse
import json
import os
import shutil
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=3_000_000)
    ap.add_argument("--cols", type=int, default=1600)
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--work", default="/tmp/hostbw_lab")
    a = ap.parse_args()
    import torch
    from shifu_amd.data.stream import _new_buf, _pread_into
    from shifu_amd.ops import _native
    shutil.rmtree(a.work, ignore_errors=True)
    d = os.path.join(a.work, "data")
    os.makedirs(d)
    if _native.rt().shifu_gen_csv(d.encode(), a.rows, a.cols, 3, 11, 0.02, 20, 16):
        raise SystemExit("generation failed")
    files = sorted(os.path.join(d, f) for f in os.listdir(d))
    total = sum(os.path.getsize(f) for f in files)
    BLK = 256 << 20
    dev = torch.device("cuda")
    out = {"rows": a.rows, "cols": a.cols, "gb": round(total / 1e9, 2)}

    # warm the page cache
    for f in files:
        with open(f, "rb") as fh:
            while fh.read(1 << 28):
                pass

    stop = threading.Event()
    res = {}

    def pread_loop(key):
        bufs = [_new_buf(BLK, True) for _ in range(2)]
        nbytes, k, t0 = 0, 0, time.perf_counter()
        while not stop.is_set():
            for f in files:
                fd = os.open(f, os.O_RDONLY)
                try:
                    size = os.path.getsize(f)
                    for off in range(0, size, BLK):
                        if stop.is_set():
                            break
                        want = min(BLK, size - off)
                        nbytes += _pread_into(fd, memoryview(bufs[k & 1])[:want], off, want)
                        k += 1
                finally:
                    os.close(fd)
                if stop.is_set():
                    break
        res[key] = nbytes / (time.perf_counter() - t0) / 1e9

    def h2d_loop(key):
        src = [_new_buf(BLK, True) for _ in range(2)]
        srct = [torch.from_numpy(s[:BLK]) for s in src]
        dst = torch.empty(BLK, dtype=torch.uint8, device=dev)
        st = torch.cuda.Stream()
        nbytes, k, t0 = 0, 0, time.perf_counter()
        with torch.cuda.stream(st):
            while not stop.is_set():
                dst.copy_(srct[k & 1], non_blocking=True)
                st.synchronize()
                nbytes += BLK
                k += 1
        res[key] = nbytes / (time.perf_counter() - t0) / 1e9

    def memcpy_loop(key):
        x = np.ones(BLK, np.uint8)
        y = np.empty_like(x)
        nbytes, t0 = 0, time.perf_counter()
        while not stop.is_set():
            np.copyto(y, x)
            nbytes += BLK
        res[key] = nbytes / (time.perf_counter() - t0) / 1e9

    loops = {"pread": pread_loop, "h2d": h2d_loop, "memcpy": memcpy_loop}

    def run(names):
        res.clear()
        stop.clear()
        ts = [threading.Thread(target=loops[n], args=(n,)) for n in names]
        for t in ts:
            t.start()
        time.sleep(a.seconds)
        stop.set()
        for t in ts:
            t.join()
        return {n: round(res[n], 2) for n in names}

    for combo in (["pread"], ["h2d"], ["memcpy"], ["pread", "h2d"], ["pread", "memcpy"], ["h2d", "memcpy"],
                  ["pread", "h2d", "memcpy"]):
        out["+".join(combo) + " GB/s"] = run(combo)
        print(json.dumps({"+".join(combo): out["+".join(combo) + " GB/s"]}), flush=True)
    print(json.dumps(out))
    shutil.rmtree(a.work, ignore_errors=True)


if __name__ == "__main__":
    main()
