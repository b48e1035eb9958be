"""Lab for the ring-pipelined TN wgrad (ops/csrc/gemm_ring.hip) at the MLP bench shapes:
correctness vs an fp32 torch reference (incl. an M % 32 tail), bitwise reproducibility, and
interleaved timing against the 128^2 wgrad kernel.

    python tools/ring_lab.py [--rows 2097152] [--rounds 3]
"""
import argparse
import json

import torch

from shifu_amd.ops import _native as nat


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def ring(D, X, G, Nv, ws):
    M, Kx = X.shape[0], X.shape[1]
    nat.call_hip("shifu_wgrad_ring", D, D.shape[1], X, X.shape[1], G, G.shape[1], M, Nv, Kx, ws, ws.numel() * 4,
                 nat.stream_of(X))


def old(D, X, G, Nv):
    M, Kx = X.shape[0], X.shape[1]
    ntiles = -(-Nv // 128) * (Kx // 128)
    spl = max(1, min(M // 256, 1024 // max(1, ntiles)))
    nat.call_hip("shifu_wgrad_tn", D, D.shape[1], X, X.shape[1], G, G.shape[1], M, Nv, Kx, spl, nat.stream_of(X))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1 << 21)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda")
    bf = torch.bfloat16
    res = {}
    # ---- correctness (small M with a tail), both layer shapes
    for name, (ldd, Nv, Kx) in {"l0": (512, 500, 1024), "l1": (256, 200, 512), "odd": (64, 30, 320)}.items():
        M = 65536 + 17
        D = (torch.rand(M, ldd, device=dev) * 2 - 1).to(bf)
        D[:, Nv:] = 0
        X = (torch.rand(M, Kx, device=dev) * 2 - 1).to(bf)
        ref = D[:, :Nv].float().t() @ X.float()
        ws = torch.empty(nat.hip().shifu_wgrad_ring_ws(M, Nv, Kx) // 4 + 4, device=dev)
        G = torch.full((Nv, Kx), 0.5, device=dev)
        ring(D, X, G, Nv, ws)
        G2 = torch.full((Nv, Kx), 0.5, device=dev)
        ring(D, X, G2, Nv, ws)
        torch.cuda.synchronize()
        err = ((G - 0.5) - ref).abs().max().item() / ref.abs().max().item()
        res[f"check_{name}"] = {"max_rel_err": err, "bitwise_repro": bool(torch.equal(G, G2))}
    # ---- timing at the bench chunk
    M = a.rows
    X = (torch.rand(M, 1024, device=dev) * 2 - 1).to(bf)
    D1 = (torch.rand(M, 512, device=dev) * 2 - 1).to(bf)
    H1 = (torch.rand(M, 512, device=dev) * 2 - 1).to(bf)
    D2 = (torch.rand(M, 256, device=dev) * 2 - 1).to(bf)
    G0 = torch.zeros(500, 1024, device=dev)
    G1 = torch.zeros(200, 512, device=dev)
    ws = torch.empty(max(nat.hip().shifu_wgrad_ring_ws(M, 500, 1024), nat.hip().shifu_wgrad_ring_ws(M, 200, 512)) // 4,
                     device=dev)
    fl0, fl1 = 2.0 * M * 512 * 1024, 2.0 * M * 256 * 512
    cases = {
        "wgrad0_old": (lambda: old(D1, X, G0, 500), fl0), "wgrad0_ring": (lambda: ring(D1, X, G0, 500, ws), fl0),
        "wgrad1_old": (lambda: old(D2, H1, G1, 200), fl1), "wgrad1_ring": (lambda: ring(D2, H1, G1, 200, ws), fl1),
    }
    for r in range(a.rounds):
        for k, (fn, fl) in cases.items():
            ms = timeit(fn)
            res.setdefault(k, []).append([round(ms, 4), round(fl / ms / 1e9, 1)])
    print(json.dumps(res))


if __name__ == "__main__":
    main()
