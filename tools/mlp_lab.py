"""Per-kernel time of one MLP training chunk at the bench shape (1000-500-200-1, sigmoid,
2M-row chunk, one lane), measured with HIP events around every native call of
``MLPTrainer._chunk_hip``; prints one JSON line (ms per kernel name and call index, total).

    python tools/mlp_lab.py [--rows 2097152] [--iters 5] [--env KEY=VAL ...]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1 << 21)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--env", nargs="*", default=[])
    ap.add_argument("--tune", nargs="*", default=[],
                    help="GEMM tune settings applied per run, e.g. 12:0 12:1 (key 12: ring forward, 14: ring dgrad)")
    ap.add_argument("--big", type=int, nargs="*", default=[0],
                    help="shifu_gemm_set_big per run (0 auto, 3 8-phase whenever M >= 64K and N >= 256, 4 128x128)")
    ap.add_argument("--stages", type=int, nargs="*", default=[1],
                    help="shifu_gemm_set_stages per run (LDS stages of the 128x128 tile kernels: 1 or 2)")
    ap.add_argument("--dbg", type=int, nargs="*", default=[0],
                    help="GEMM lab ablation bits per run (1: no head err atomics, 2: main loops only, 4: head "
                         "stages 1-2 only, 8: no head / 8-phase tile stores, 16: head w_out without loads)")
    a = ap.parse_args()
    for kv in a.env:
        k, v = kv.split("=", 1)
        os.environ[k] = v
    import torch
    from shifu_amd.models import nn as NN
    from shifu_amd.ops import _native as nat
    dev = torch.device("cuda")
    spec = NN.MLPSpec(n_in=1000, hidden=[500, 200], acts=["sigmoid", "sigmoid"], n_out=1)
    tr = NN.MLPTrainer(spec, device=dev, propagation="R", learning_rate=0.1, seed=7, chunk_rows=a.rows)
    g = torch.Generator(device=dev).manual_seed(5)
    k0 = spec.layer_kpad[0]
    x = torch.empty(a.rows, k0, dtype=torch.bfloat16, device=dev)
    x[:, :1000].normal_(generator=g)
    x[:, 1000] = 1
    x[:, 1001:] = 0
    y = (torch.rand(a.rows, 1, generator=g, device=dev) > 0.5).float()
    data = NN.TrainData(x, y, None, a.rows)
    wb, wt = tr._weights_bf16()
    real = nat.call_hip
    rec = []

    def timed(name, *args):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r = real(name, *args)
        e1.record()
        rec.append((name, e0, e1))
        return r
    tr.grad.zero_()
    tr._final_chunk = True
    tr._chunk_hip(data, 0, a.rows, wb, wt)              # warm-up (workspace, code objects)
    torch.cuda.synchronize()
    for tune in (a.tune or [None]):
        if tune is not None:
            k, v = (int(x) for x in tune.split(":"))
            nat.call_hip("shifu_gemm_set_tune", k, v)
        for big in a.big:
            nat.call_hip("shifu_gemm_set_big", big)
            for stg in a.stages:
                nat.call_hip("shifu_gemm_set_stages", stg)
                for dbg in a.dbg:
                    nat.call_hip("shifu_gemm_set_tune", 9, dbg)
                    run(a, tr, data, wb, wt, timed, real, rec, f"{dbg} tune {tune} big {big} stages {stg}", nat, torch)
    nat.call_hip("shifu_gemm_set_stages", 1)
    nat.call_hip("shifu_gemm_set_tune", 9, 0)


def run(a, tr, data, wb, wt, timed, real, rec, dbg, nat, torch):
    nat.call_hip = timed
    try:
        tot = {}
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        wall = 0.0
        for _ in range(a.iters):
            rec.clear()
            e0.record()
            tr._chunk_hip(data, 0, a.rows, wb, wt)
            e1.record()
            torch.cuda.synchronize()
            wall += e0.elapsed_time(e1)
            for i, (name, s0, s1) in enumerate(rec):
                key = f"{i:02d}_{name}"
                tot[key] = tot.get(key, 0.0) + s0.elapsed_time(s1)
    finally:
        nat.call_hip = real
    out = {k: round(v / a.iters, 4) for k, v in sorted(tot.items())}
    out["chunk_ms"] = round(wall / a.iters, 4)
    out["rows"] = a.rows
    out["rows_per_s_one_lane"] = round(a.rows / (wall / a.iters) * 1e3 / 1e6, 1)
    out["env"] = a.env
    out["dbg"] = dbg
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
