"""Host vs device time of each K4 stage for one 64-column batch (100M rows by default): every
QuantileEngine stage is bracketed by torch.cuda.synchronize(), so 'ms' is the stage's wall time
with the GPU drained on entry; pass_* stages are device work, finish_* / planning are host work
(plus their small syncs).

    PYTHONPATH=. python tools/stats_host_timing.py [--rows 100000000]
"""
import argparse
import collections
import json
import time

import torch

import bench
from shifu_amd.algos import quantile as Q
from shifu_amd.algos.stats import batch_histograms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    a = ap.parse_args()
    dev = torch.device("cuda")
    n = a.rows
    y = (torch.rand(n, device=dev) < 0.3).float()
    w = torch.ones(n, dtype=torch.float64, device=dev)
    acc = collections.defaultdict(float)
    calls = collections.Counter()

    def wrap(name):
        orig = getattr(Q.QuantileEngine, name)

        def f(self, *args, **kw):
            torch.cuda.synchronize()
            t = time.perf_counter()
            r = orig(self, *args, **kw)
            torch.cuda.synchronize()
            acc[name] += (time.perf_counter() - t) * 1e3
            calls[name] += 1
            return r
        setattr(Q.QuantileEngine, name, f)

    for name in ("pass_a", "finish_a", "pass_b", "finish_b", "pass_c", "finish"):
        wrap(name)
    res = {}
    for step in range(3):
        acc.clear()
        calls.clear()
        v = bench._stats_batch(64, n, 64 * step, dev, 11 + step)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        bounds, _ = Q.column_cuts(v, y, w, 10, "EqualPositive", True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        batch_histograms(v, y, w, bounds, True)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        res = {"column_cuts_ms": round((t1 - t0) * 1e3, 2), "batch_histograms_ms": round((t2 - t1) * 1e3, 2),
               "stages_ms": {k: round(x, 2) for k, x in acc.items()}, "calls": dict(calls)}
        print(step, json.dumps(res), flush=True)
        del v


if __name__ == "__main__":
    main()
