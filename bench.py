#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): rows/sec (whole node) of Shifu NN training,
MLP 1000-500-200-1 binary classifier, bf16, 100M rows x 1000 cols per MI355X.

One step = one full training iteration of the reference's NN algorithm
(``J/core/dtrain/nn/AbstractNNWorker.java:521-588`` + ``NNMaster.java:207-319``): forward +
backward over every resident row of the local shard, one RCCL all-reduce of the fp32
gradient (+ error scalars), and the replicated RPROP update - nothing skipped.

Weak scaling: every rank owns ``--rows`` rows (synthetic, generated on device, random-init
weights).  ``value`` = total rows processed per second over all ranks.

    python bench.py --gpus 1 --steps 5 --warmup 2
    torchrun --nproc-per-node 8 bench.py --gpus 8 ...
    python bench.py --model gbdt    # GBDT rounds/sec (500 trees depth 7, 256 bins) config
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

# Derived reference throughput (CHANGES.txt:268): 20M rows x 200 epochs in
# 45 min on the Hadoop cluster = 1.48M row-epochs/s whole cluster (1600 inputs).
BASELINE_MLP_ROWS_PER_S = 20e6 * 200 / 2700.0
METRIC = "rows/sec (whole node) MLP train + GBDT rounds/sec on 1B-row×1k-col tabular"


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def make_synthetic(rows, n_in, k0, device, seed):
    """bf16 rows [rows, k0]: N(0,1) features, bias column = 1, zero padding; labels from a
    random hidden linear rule so the task is learnable."""
    g = torch.Generator(device=device).manual_seed(seed)
    x = torch.empty(rows, k0, dtype=torch.bfloat16, device=device)
    y = torch.empty(rows, 1, dtype=torch.float32, device=device)
    wt = torch.randn(n_in, 1, generator=g, device=device, dtype=torch.float32).to(torch.bfloat16)
    step = 1 << 22
    for r0 in range(0, rows, step):
        r1 = min(rows, r0 + step)
        blk = x[r0:r1]
        blk[:, :n_in].normal_(generator=g)
        blk[:, n_in] = 1
        blk[:, n_in + 1:] = 0
        y[r0:r1] = (blk[:, :n_in] @ wt > 0).float()
    return x, y


def bench_mlp(a, dev, info):
    from shifu_amd.models.nn import MLPSpec, MLPTrainer, TrainData
    from shifu_amd.parallel import dist
    spec = MLPSpec(n_in=a.cols, hidden=[500, 200], acts=["sigmoid", "sigmoid"], n_out=1)
    tr = MLPTrainer(spec, device=dev, propagation=a.propagation, learning_rate=0.1, seed=7,
                    chunk_rows=a.chunk_rows)
    t0 = time.time()
    if dev.type == "cuda":
        x, y = make_synthetic(a.rows, a.cols, spec.layer_kpad[0], dev, 1234 + info.rank)
    else:
        g = torch.Generator().manual_seed(1234 + info.rank)
        xr = torch.randn(a.rows, a.cols, generator=g)
        y = (xr[:, :1] > 0).float()
        x = tr.prepare(xr, y).x
    data = TrainData(x, y, None, a.rows)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    log(f"[bench] data ready: {a.rows} rows x {a.cols} cols/rank ({x.numel() * x.element_size() / 1e9:.1f} GB) "
        f"in {time.time() - t0:.1f}s")
    n_global = float(a.rows * info.world_size)
    for i in range(a.warmup):
        e = tr.step(data, num_train_global=n_global)
        log(f"[bench] warmup {i} train error {e:.6f}")

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()
    dist.barrier(); sync()
    t0 = time.perf_counter()
    errs = []
    for i in range(a.steps):
        errs.append(tr.step(data, num_train_global=n_global))
    sync(); dist.barrier()
    dt = time.perf_counter() - t0
    log(f"[bench] train errors {['%.6f' % e for e in errs]}")
    flops_row = 2 * (a.cols * 500 + 500 * 200 + 200) * 2 + 2 * 500 * 200   # fwd+wgrad all, dgrad layer2
    return dt, errs, flops_row


def bench_gbdt(a, dev, info):
    from shifu_amd.models.gbdt import bench_rounds
    return bench_rounds(a, dev, info)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default="mlp", choices=["mlp", "gbdt"])
    ap.add_argument("--rows", type=int, default=None, help="rows per GPU (default 100M on GPU)")
    ap.add_argument("--cols", type=int, default=1000)
    ap.add_argument("--chunk-rows", type=int, default=1 << 20)
    ap.add_argument("--propagation", default="R")
    a = ap.parse_args()

    from shifu_amd.parallel import dist
    info = dist.init_from_env()
    gpu = torch.cuda.is_available()
    dev = torch.device("cuda", torch.cuda.current_device()) if gpu else torch.device("cpu")
    if a.rows is None:
        a.rows = 100_000_000 if gpu else 20_000
    if a.model == "gbdt":
        res = bench_gbdt(a, dev, info)
        out = res
    else:
        dt, errs, flops_row = bench_mlp(a, dev, info)
        dt_t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce_(dt_t, "max")
        dt = float(dt_t.item())
        ms = dt / a.steps * 1e3
        total_rows = a.rows * info.world_size
        value = total_rows * a.steps / dt
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "rows/s",
            "n_gpus": info.world_size,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": value / BASELINE_MLP_ROWS_PER_S,
            "dtype": "bf16",
            "data": "synthetic (N(0,1) features, labels from a hidden linear rule), random-init weights",
            "config": {"model": "MLP 1000-500-200-1 (sigmoid, RPROP, squared loss, full-batch epoch)",
                       "global_batch": total_rows, "seq_len": None, "n_cols": a.cols,
                       "rows_per_gpu": a.rows, "parallelism": f"dp{info.world_size}"},
            "achieved_tflops": value * flops_row / 1e12,
            "baseline_note": "baseline = 1.48M rows/s derived from CHANGES.txt:268 (SURVEY §6)",
            "final_train_error": errs[-1] if errs else None,
        }
    if info.rank == 0:
        print(json.dumps(out), flush=True)
    dist.shutdown()


if __name__ == "__main__":
    main()
