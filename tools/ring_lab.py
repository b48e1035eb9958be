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


def ring_ld(D, X, G, Nv, ws):          # variant: DMA issued in the LD segment
    nat.call_hip("shifu_ring_set_dmamma", 0)
    ring(D, X, G, Nv, ws)
    nat.call_hip("shifu_ring_set_dmamma", 1)


def ring32(D, X, G, Nv, ws):           # variant: 32x32x16 MFMA
    nat.call_hip("shifu_ring_set_mf", 32)
    ring(D, X, G, Nv, ws)
    nat.call_hip("shifu_ring_set_mf", 16)


def old(D, X, G, Nv):
    M, Kx = X.shape[0], X.shape[1]
    ntiles = -(-Nv // 128) * (Kx // 128)
    spl = max(1, min(M // 256, 1024 // max(1, ntiles)))
    nat.call_hip("shifu_wgrad_tn", D, D.shape[1], X, X.shape[1], G, G.shape[1], M, Nv, Kx, spl, nat.stream_of(X))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1 << 21)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", nargs="*", default=None, help="timed cases to run (PMC passes)")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--stamp", action="store_true", help="segment timestamps of the TN ring (diagnostic)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    bf = torch.bfloat16
    res = {}
    # ---- correctness (small M with a tail), both layer shapes
    checks = {} if a.no_check else {"l0": (512, 500, 1024), "l1": (256, 200, 512), "odd": (64, 30, 320)}
    for name, (ldd, Nv, Kx) in checks.items():
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
    # ---- NT forward ring: correctness (M not a multiple of 256, sigmoid + bias column + padding)
    M = 70000 if not a.no_check else 256
    X = (torch.rand(M, 1024, device=dev) * 2 - 1).to(bf)
    W = ((torch.rand(500, 1024, device=dev) * 2 - 1) * 0.05).to(bf)
    H = torch.full((M, 512), 7.0, device=dev, dtype=bf)
    nat.call_hip("shifu_gemm_ring_nt", X, 1024, W, 1024, 500, H, 512, M, 512, 1024, 0, 0, 500, 1, nat.stream_of(X))
    ref = torch.zeros(M, 512, device=dev)
    ref[:, :500] = torch.sigmoid(X.float() @ W.float().t())
    ref[:, 500] = 1
    torch.cuda.synchronize()
    res["check_nt_fwd"] = {"max_abs_err": (H.float() - ref).abs().max().item()}
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
    W1 = ((torch.rand(500, 1024, device=dev) * 2 - 1) * 0.05).to(bf)
    H1o = torch.empty(M, 512, device=dev, dtype=bf)
    st = nat.stream_of(X)
    flf = 2.0 * M * 512 * 1024

    def fwd_old():
        nat.call_hip("shifu_gemm_nt", X, 1024, W1, 1024, 500, H1o, 512, None, 0, None, 0, None, 0, M, 512, 1024, 0,
                     0, 500, 1, 0.0, st)

    def fwd_ring():
        nat.call_hip("shifu_gemm_ring_nt", X, 1024, W1, 1024, 500, H1o, 512, M, 512, 1024, 0, 0, 500, 1, st)

    def fwd_ring_store():
        nat.call_hip("shifu_gemm_ring_nt", X, 1024, W1, 1024, 500, H1o, 512, M, 512, 1024, 2, 2, 500, 0, st)

    cases = {
        "fwd1_old": (fwd_old, flf), "fwd1_ring": (fwd_ring, flf), "fwd1_ring_storeonly": (fwd_ring_store, flf),
        "wgrad0_old": (lambda: old(D1, X, G0, 500), fl0), "wgrad0_ring": (lambda: ring(D1, X, G0, 500, ws), fl0),
        "wgrad1_old": (lambda: old(D2, H1, G1, 200), fl1), "wgrad1_ring": (lambda: ring(D2, H1, G1, 200, ws), fl1),
        "wgrad0_ring_dmald": (lambda: ring_ld(D1, X, G0, 500, ws), fl0),
        "wgrad0_ring32": (lambda: ring32(D1, X, G0, 500, ws), fl0),
    }
    for r in range(a.rounds):
        for k, (fn, fl) in cases.items():
            if a.only and k not in a.only:
                continue
            ms = timeit(fn)
            res.setdefault(k, []).append([round(ms, 4), round(fl / ms / 1e9, 1)])
    if a.stamp:              # diagnostic STAMP build of the TN ring: mean cycles per step per segment
        for mf in (16, 32):
            buf = torch.zeros(256 * 8 * 8, dtype=torch.int64, device=dev)
            nat.call_hip("shifu_ring_set_mf", mf)
            nat.call_hip("shifu_ring_set_stamp", buf)
            ring(D1, X, G0, 500, ws)
            torch.cuda.synchronize()
            nat.call_hip("shifu_ring_set_stamp", None)
            b = buf.view(256, 8, 8).double().cpu()
            names = ["dma", "reads", "waits", "ld_bar", "mfma", "mma_bar"]
            for half, sl in (("lead", slice(0, 4)), ("lag", slice(4, 8))):
                v = b[:, sl, :6].sum(dim=(0, 1)) / b[:, sl, 6].sum()
                res[f"stamp{mf}_{half}_cycles_per_step"] = {n: round(float(x), 1) for n, x in zip(names, v)}
        nat.call_hip("shifu_ring_set_mf", 16)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
