"""RF tree parallelism A/B: trees grown one at a time vs in forest batches (SHIFU_RF_BATCH).

    python tools/bench_rf.py --rows 20000000 --cols 200 --trees 8 --depth 7
"""
import argparse
import json
import os
import time

import torch

from shifu_amd.models.gbdt import TreeConfig, TreeTrainer, synthetic_binned


def run(data, batch, a):
    os.environ["SHIFU_RF_BATCH"] = str(batch)
    cfg = TreeConfig("RF", tree_num=a.trees, max_depth=a.depth, impurity="gini", sample_with_replacement=True,
                     feature_subset_strategy=a.fss, seed=1)
    tr = TreeTrainer(cfg, data)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.train()
    torch.cuda.synchronize()
    return time.perf_counter() - t0, tr


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=20_000_000)
    ap.add_argument("--cols", type=int, default=200)
    ap.add_argument("--trees", type=int, default=8)
    ap.add_argument("--depth", type=int, default=7)
    ap.add_argument("--fss", default="SQRT")
    a = ap.parse_args()
    data = synthetic_binned(a.rows, a.cols, "cuda", seed=3)
    run(data, a.trees, a)                               # warm-up (kernels, allocator)
    out = {}
    for b in (1, a.trees):
        s, tr = run(data, b, a)
        out[f"batch{b}"] = {"s": s, "trees_per_s": a.trees / s, "train_error": tr.train_errors[-1]}
    print(json.dumps({"rows": a.rows, "cols": a.cols, "trees": a.trees, "depth": a.depth, **out}))


if __name__ == "__main__":
    main()
