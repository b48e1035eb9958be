"""Per-op device time of one EvalPerformance pass (algos/evaluation.performance) at the eval bench
shape (100M scored rows, integer scores with heavy ties, weights): torch.profiler table sorted
by device time, plus the wall time of the pass.

    python tools/eval_lab.py [--rows 100000000] [--top 25]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    import torch
    from shifu_amd.algos import evaluation as E
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(11)
    n = a.rows
    z = torch.randn(n, generator=g, device=dev, dtype=torch.float64)
    y = (torch.rand(n, generator=g, device=dev, dtype=torch.float64) < torch.sigmoid(1.5 * z - 1.0)).double()
    score = torch.round(1000.0 * torch.sigmoid(z))
    w = 0.5 + torch.rand(n, generator=g, device=dev, dtype=torch.float64)
    E.performance(score, y, w, 10, max_score=1000.0, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    E.performance(score, y, w, 10, max_score=1000.0, device=dev)
    torch.cuda.synchronize()
    print(f"performance wall: {time.perf_counter() - t0:.3f}s", flush=True)
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        E.performance(score, y, w, 10, max_score=1000.0, device=dev)
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=a.top), flush=True)
    print(prof.key_averages().table(sort_by="cpu_time_total", row_limit=a.top), flush=True)


if __name__ == "__main__":
    main()
