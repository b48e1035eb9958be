"""Phase timing of the fused MLP row-block kernel (ops/csrc/mlp_fused.hip) at the bench shape:
s_memtime stamps per block (GEMM1, epilogue 1, GEMM2, head, GEMM3 halves, tail) averaged over
the chunk's blocks, plus the kernel's HIP-event time.  One JSON line.

    python tools/fused_lab.py [--rows 2097152] [--iters 3]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1 << 21)
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    os.environ["SHIFU_FUSED_MLP"] = "1"
    import torch
    from shifu_amd.models import nn as NN
    from shifu_amd.ops import _native as nat
    dev = torch.device("cuda")
    spec = NN.MLPSpec(n_in=1000, hidden=[500, 200], acts=["sigmoid", "sigmoid"], n_out=1)
    tr = NN.MLPTrainer(spec, device=dev, propagation="R", learning_rate=0.1, seed=7, chunk_rows=a.rows)
    assert tr.fused2
    g = torch.Generator(device=dev).manual_seed(5)
    k0 = spec.layer_kpad[0]
    x = torch.empty(a.rows, k0, dtype=torch.bfloat16, device=dev)
    x[:, :1000].normal_(generator=g)
    x[:, 1000] = 1
    x[:, 1001:] = 0
    y = (torch.rand(a.rows, 1, generator=g, device=dev) > 0.5).float()
    data = NN.TrainData(x, y, None, a.rows)
    tr._weights_bf16()
    tiles = -(-a.rows // 128)
    st = torch.zeros(tiles * 8, dtype=torch.int64, device=dev)
    real = nat.call_hip
    times = []

    def timed(name, *args):
        if name != "shifu_mlp_fused2":
            return real(name, *args)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r = real(name, *args)
        e1.record()
        times.append((e0, e1))
        return r
    tr._final_chunk = True
    tr._chunk_hip(data, 0, a.rows, None, None)
    torch.cuda.synchronize()
    nat.call_hip = timed
    out = {}
    try:
        for mode in ("plain", "stamps"):
            nat.hip().shifu_mlp_fused2_set_stamps(st.data_ptr() if mode == "stamps" else None)
            times.clear()
            for _ in range(a.iters):
                tr._chunk_hip(data, 0, a.rows, None, None)
            torch.cuda.synchronize()
            out[f"kernel_ms_{mode}"] = round(sorted(e0.elapsed_time(e1) for e0, e1 in times)[len(times) // 2], 4)
    finally:
        nat.call_hip = real
        nat.hip().shifu_mlp_fused2_set_stamps(None)
    s = st.view(tiles, 8).cpu().double()
    d = s[:, 1:] - s[:, :-1]
    names = ["gemm1", "epi1", "gemm2", "head", "gemm3_h0", "gemm3_h1", "tail"]
    out["cycles_per_block"] = {n: round(float(d[:, i].mean()), 0) for i, n in enumerate(names)}
    tot = float((s[:, 7] - s[:, 0]).mean())
    out["cycles_per_block_total"] = round(tot, 0)
    out["blocks"] = tiles
    out["implied_ghz"] = round(tot * tiles / 256 / (out["kernel_ms_stamps"] * 1e6), 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
