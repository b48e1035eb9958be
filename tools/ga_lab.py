"""Timing of one voted-varsel generation (algos/ga_varsel.PopulationTrainer) at the reference's GA
defaults: 500 seeds x 300 of F candidate columns, 10 hidden units, on synthetic rows.

    python tools/ga_lab.py [--rows 200000] [--cols 1600] [--epochs 10]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=200000)
    ap.add_argument("--cols", type=int, default=1600)
    ap.add_argument("--seeds", type=int, default=500)
    ap.add_argument("--expect", type=int, default=300)
    ap.add_argument("--hidden", type=int, default=10)
    ap.add_argument("--epochs", type=int, default=10)
    a = ap.parse_args()
    from shifu_amd.algos.ga_varsel import PopulationData, PopulationTrainer
    g = np.random.default_rng(0)
    X = g.normal(size=(a.rows, a.cols)).astype(np.float32)
    y = (X[:, 0] + X[:, 1] > 0).astype(np.float32)
    w = np.ones(a.rows, np.float32)
    valid = g.random(a.rows) < 0.2
    masks = np.zeros((a.seeds, a.cols), bool)
    for p in range(a.seeds):
        masks[p, g.choice(a.cols, a.expect, replace=False)] = True
    t0 = time.perf_counter()
    data = PopulationData(X, y, w, valid, "cuda")
    torch.cuda.synchronize()
    t_stage = time.perf_counter() - t0
    tr = PopulationTrainer(data, masks, a.hidden, "sigmoid", 0.1, torch.Generator().manual_seed(1))
    tr.train(1)                                        # warm-up (workspaces, code objects)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr = PopulationTrainer(data, masks, a.hidden, "sigmoid", 0.1, torch.Generator().manual_seed(1))
    errs = tr.train(a.epochs)
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    ntr = int((~valid).sum())
    flops = a.epochs * 2 * 2 * ntr * tr.kx * tr.PH + 2 * int(valid.sum()) * tr.kx * tr.PH
    print(json.dumps({"rows": a.rows, "cols": a.cols, "seeds": a.seeds, "expect": a.expect, "hidden": a.hidden,
                      "epochs": a.epochs, "stage_s": round(t_stage, 3), "generation_s": round(t, 4),
                      "epoch_ms": round(1e3 * t / a.epochs, 3), "dense_gemm_tflops": round(flops / t / 1e12, 1),
                      "best_err": float(errs.min())}))


if __name__ == "__main__":
    main()
