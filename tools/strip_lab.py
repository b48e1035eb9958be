"""Forward-engine lab: the row-strip engine (gemm_strip_nt.hip, tune key 14) against the persistent
ring (gemm_ring_nt.hip, tune key 12) -- bitwise equality on the bench shape and tail shapes, then
interleaved timing rounds in one process (median / min ms per call), and the strip engine's LAB
ablations (dbg 1: no epilogue, 4: no MFMAs, 5: neither).  One JSON line per measurement.

    python tools/strip_lab.py [--rows 2097152] [--iters 10] [--rounds 3]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1 << 21)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--dbg", type=int, nargs="*", default=[1, 4, 5])
    a = ap.parse_args()
    import torch
    from shifu_amd.ops import _native as nat
    dev = torch.device("cuda")
    st = nat.stream_of(torch.empty(1, device=dev))

    def run(engine, A, B, C, M, K, N, nb, nv, act, dbg=-1):
        nat.call_hip("shifu_gemm_set_tune", 12, 1 if engine == "ring" else 0)
        nat.call_hip("shifu_gemm_set_tune", 14, 1 if engine == "strip" else 0)
        nat.call_hip("shifu_strip_nt_set_lab", dbg)
        nat.call_hip("shifu_gemm_nt", A, K, B, K, nb, C, N, None, 0, None, 0, None, 0, M, N, K, 0, act, nv, 1, 0.0, st)

    # correctness: bitwise vs the ring (same k order), plus an fp32 check on the tail shapes
    shapes = [(a.rows, 1024, 512, 500, 500, 0), (70033, 256, 512, 512, 512, 3), (65836, 128, 264, 260, 260, 0),
              (65536 + 300, 384, 384, 256, 256, 2), (131072, 512, 1024, 1000, 1000, 7)]
    g = torch.Generator(device=dev).manual_seed(5)
    for M, K, N, nb, nv, act in shapes:
        A = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        B = (torch.randn(nb, K, device=dev, generator=g) * 0.05).to(torch.bfloat16)
        out = {}
        for eng in ("ring", "strip"):
            C = torch.full((M, N), 7.0, dtype=torch.bfloat16, device=dev)
            run(eng, A, B, C, M, K, N, nb, nv, act)
            torch.cuda.synchronize()
            out[eng] = C
        same = bool(torch.equal(out["ring"], out["strip"]))
        nbad = int((out["ring"] != out["strip"]).sum())
        dmax = float((out["ring"].float() - out["strip"].float()).abs().max())
        print(json.dumps({"check": "bitwise_vs_ring", "M": M, "K": K, "N": N, "NB": nb, "act": act, "equal": same,
                          "mismatches": nbad, "max_abs_diff": dmax}), flush=True)
        del A, B, out
    torch.cuda.empty_cache()

    M, K, N, nv = a.rows, 1024, 512, 500
    A = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    B = (torch.randn(nv, K, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    C = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.iters)]
    flop = 2.0 * M * K * nv

    def timed(eng, dbg=-1):
        run(eng, A, B, C, M, K, N, nv, nv, 0, dbg)
        torch.cuda.synchronize()
        for i in range(a.iters):
            ev[2 * i].record()
            run(eng, A, B, C, M, K, N, nv, nv, 0, dbg)
            ev[2 * i + 1].record()
        torch.cuda.synchronize()
        ts = sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(a.iters))
        return ts[len(ts) // 2], ts[0]

    variants = [("ring", -1), ("strip", -1), ("strip_lab0", 0)] + [(f"strip_lab_dbg{d}", d) for d in a.dbg]
    for rnd in range(a.rounds):
        for name, dbg in variants:
            eng = "ring" if name == "ring" else "strip"
            med, mn = timed(eng, dbg)
            print(json.dumps({"variant": name, "round": rnd, "ms_median": round(med, 4), "ms_min": round(mn, 4),
                              "tflops_median": round(flop / med / 1e9, 1), "M": M, "K": K, "N": N}), flush=True)
    nat.call_hip("shifu_strip_nt_set_lab", -1)


if __name__ == "__main__":
    main()
