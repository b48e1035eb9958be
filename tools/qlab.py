"""K4 / K1+K2 kernel lab: time each stats pass per column type on the GPU.

    PYTHONPATH=. python tools/qlab.py [--rows 100000000] [--cols 64]
"""
import argparse
import json
import time

import torch

from shifu_amd.algos import quantile as Q
from shifu_amd.algos.stats import batch_histograms


def gen(kind, C, n, dev):
    g = torch.Generator(device=dev).manual_seed(3)
    v = torch.empty(C, n, dtype=torch.float64, device=dev).normal_(generator=g)
    if kind == "lognormal":
        v.mul_(2.0).exp_()
    elif kind == "int":
        v.mul_(3.0).floor_()
    elif kind == "dec2":
        v.mul_(100.0).round_().div_(100.0)
    return v


def timed(fn, reps=3):
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return min(ts) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--cols", type=int, default=64)
    a = ap.parse_args()
    dev = torch.device("cuda")
    y = (torch.rand(a.rows, device=dev) < 0.3).float()
    w = torch.ones(a.rows, dtype=torch.float64, device=dev)
    out = {}
    for kind in ("normal", "lognormal", "int", "dec2"):
        v = gen(kind, a.cols, a.rows, dev)
        res = {}
        for sm in (0, 1):
            e = Q.QuantileEngine(a.cols, 10, sm, False, False, device=dev)
            res[f"qprep_sel{sm}"] = timed(lambda: e.pass_a(v, y, w), 1)
            e.finish_a()
            res[f"qhist_sel{sm}"] = timed(lambda: e.pass_b(v, y, w), 1)
            st = e.finish_b()
            res[f"levels_sel{sm}"] = e.level
            lv = 1
            while st == "B":
                res[f"qhist_l{lv + 1}_sel{sm}"] = timed(lambda: e.pass_b(v, y, w), 1)
                st = e.finish_b()
                lv += 1
            if st == "C":
                res[f"qgather_sel{sm}"] = timed(lambda: e.pass_c(v, y, w), 1)
                res[f"gathered_sel{sm}"] = int(e.local_lens.sum())
            res[f"finish_sel{sm}"] = timed(lambda: e.finish(), 1)
        b, _ = Q.column_cuts(v, y, w, 10, "EqualPositive", True)
        res["column_stats"] = timed(lambda: batch_histograms(v, y, w, b, True))
        res["full_column_cuts"] = timed(lambda: Q.column_cuts(v, y, w, 10, "EqualPositive", True), 1)
        out[kind] = res
        print(kind, json.dumps(res), flush=True)
        del v
    gb = a.rows * a.cols * 8 / 1e9
    print(json.dumps({"batch_gb": gb, "results_ms": out}))


if __name__ == "__main__":
    main()
