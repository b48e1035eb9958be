"""Write rate into a file on tmpfs or disk from a page-locked-sized host buffer: N-thread pwrite
(tmpfs serialises writers of one inode), N threads writing one file each, and N-thread copies
into a shared mapping of the file.  The norm step's NormalizedData writer is the client.

    python tools/write_lab.py [--dir /dev/shm] [--gb 4]
"""
import argparse
import json
import mmap
import os
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default="/dev/shm")
    ap.add_argument("--gb", type=float, default=4.0)
    a = ap.parse_args()
    n = int(a.gb * (1 << 30))
    src = np.ones(n, np.uint8)
    path = os.path.join(a.dir, "write_lab.bin")
    out = {"dir": a.dir, "gb": a.gb}

    def run(kind, nt):
        cuts = [n * i // nt for i in range(nt + 1)]
        if kind == "files":                      # one file per thread (one inode each)
            mv = memoryview(src)

            def g(i):
                fdi = os.open(f"{path}.{i}", os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
                m, off = mv[cuts[i]:cuts[i + 1]], 0
                while len(m):
                    k = os.pwrite(fdi, m, off)
                    m, off = m[k:], off + k
                os.close(fdi)
            t = time.perf_counter()
            with ThreadPoolExecutor(nt) as ex:
                list(ex.map(g, range(nt)))
            dt = time.perf_counter() - t
            for i in range(nt):
                os.remove(f"{path}.{i}")
            return round(n / dt / 1e9, 2)
        fd = os.open(path, os.O_RDWR | os.O_CREAT | os.O_TRUNC, 0o644)
        t = time.perf_counter()
        if kind == "pwrite":
            mv = memoryview(src)

            def f(i):
                m, off = mv[cuts[i]:cuts[i + 1]], cuts[i]
                while len(m):
                    k = os.pwrite(fd, m, off)
                    m, off = m[k:], off + k
            with ThreadPoolExecutor(nt) as ex:
                list(ex.map(f, range(nt)))
        else:
            os.ftruncate(fd, n)
            m = mmap.mmap(fd, n)
            dst = np.frombuffer(m, np.uint8)

            def f(i):
                np.copyto(dst[cuts[i]:cuts[i + 1]], src[cuts[i]:cuts[i + 1]])
            with ThreadPoolExecutor(nt) as ex:
                list(ex.map(f, range(nt)))
            del dst
            m.close()
        dt = time.perf_counter() - t
        os.close(fd)
        os.remove(path)
        return round(n / dt / 1e9, 2)

    for kind in ("pwrite", "files", "mmap"):
        for nt in (1, 4, 8, 16):
            out[f"{kind}_{nt}_GBps"] = run(kind, nt)
            print(json.dumps({f"{kind}_{nt}": out[f"{kind}_{nt}_GBps"]}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
