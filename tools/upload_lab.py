"""Bf16Rows.device_rows upload rates from a /dev/shm memmap (the pipeline's NormalizedData on
tmpfs): the pinned multi-thread staging at several thread counts vs the plain pageable upload.

    python tools/upload_lab.py [--rows 4000000] [--kpad 1664]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=4_000_000)
    ap.add_argument("--kpad", type=int, default=1664)
    ap.add_argument("--dir", default="/dev/shm")
    a = ap.parse_args()
    import numpy as np
    import torch
    from shifu_amd.data.rowstore import Bf16Rows
    path = os.path.join(a.dir, "upload_lab.npy")
    arr = np.lib.format.open_memmap(path, mode="w+", dtype=np.uint16, shape=(a.rows, a.kpad))
    step = 1 << 18
    for r0 in range(0, a.rows, step):
        arr[r0:r0 + step] = np.uint16(0x3F80)
    arr.flush()
    del arr
    dev = torch.device("cuda", 0)
    gb = a.rows * a.kpad * 2 / 1e9
    res = {"gb": gb}
    for mode in ("pageable", 1, 4, 8, 16):  # COPY_THREADS (0 = pageable default)
        raw = np.load(path, mmap_mode="r")
        v = Bf16Rows(raw, a.kpad - 64)
        torch.cuda.synchronize()
        t = time.perf_counter()
        if mode == "pageable":
            out = torch.empty((a.rows, a.kpad), dtype=torch.int16, device=dev)
            for r0 in range(0, a.rows, step):
                out[r0:r0 + step] = torch.as_tensor(np.ascontiguousarray(raw[r0:r0 + step]).view(np.int16), device=dev)
        else:
            Bf16Rows.COPY_THREADS = mode
            out = v.device_rows(dev)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        res[str(mode)] = {"s": round(dt, 3), "GB_per_s": round(gb / dt, 2)}
        print(mode, res[str(mode)], flush=True)
        del out, raw, v
    os.remove(path)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
