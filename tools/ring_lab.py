"""Forward-GEMM lab at the bench's first layer (2M-row chunk x 1024 -> 512, sigmoid + bias column):
times the persistent ring forward (gemm_ring_nt.hip) against the 8-phase kernel, its LAB build
with ablation bits, and the LAB build's per-wave segment cycle sums (s_memtime stamps).  One JSON
line per variant.

    python tools/ring_lab.py [--rows 2097152] [--k 1024] [--n 512] [--iters 10] [--dbg 1 2 4 8]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SEGS = ["epilogue", "frag_reads", "waits", "ld_barrier", "mma", "mma_barrier"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1 << 21)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--nv", type=int, default=500)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--dbg", type=int, nargs="*", default=[1, 2, 4, 8, 5])
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--variants", type=int, nargs="*", default=[0, 1, 2],
                    help="schedule variants (shifu_ring_nt_set_variant) timed in production and LAB builds")
    ap.add_argument("--stamp-dbg", type=int, nargs="*", default=[], help="extra LAB ablation bits for stamp runs")
    ap.add_argument("--no-lab", action="store_true", help="production builds only (PMC runs), no stamps")
    a = ap.parse_args()
    import torch
    from shifu_amd.ops import _native as nat
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(3)
    M, K, N = a.rows, a.k, a.n
    A = torch.empty(M, K, dtype=torch.bfloat16, device=dev)
    A.normal_(generator=g)
    B = (torch.randn(N, K, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    C = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    st = nat.stream_of(A)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.iters)]

    def launch():
        r = nat.call_hip("shifu_gemm_nt", A, K, B, K, a.nv, C, N, None, 0, None, 0, None, 0,
                         M, N, K, 0, 0, a.nv, 1, 0.0, st)
        assert r == 0, r

    def timed():
        launch()
        torch.cuda.synchronize()
        for i in range(a.iters):
            ev[2 * i].record()
            launch()
            ev[2 * i + 1].record()
        torch.cuda.synchronize()
        ts = sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(a.iters))
        return ts[len(ts) // 2], ts[0]

    flop = 2.0 * M * K * a.nv
    variants = [("8phase", 0, -1, 0)]
    for v in a.variants:
        variants += [(f"ring_v{v}", 1, -1, v)]
        if not a.no_lab:
            variants += [(f"ring_v{v}_lab_dbg0", 1, 0, v)] + [(f"ring_v{v}_lab_dbg{d}", 1, d, v) for d in a.dbg]
    for rnd in range(a.rounds):
        for name, ring, dbg, var in variants:
            nat.call_hip("shifu_gemm_set_tune", 12, ring)
            nat.call_hip("shifu_ring_nt_set_variant", var)
            nat.call_hip("shifu_ring_nt_set_lab", dbg, None)
            med, mn = timed()
            print(json.dumps({"variant": name, "round": rnd, "ms_median": round(med, 4), "ms_min": round(mn, 4),
                              "tflops_median": round(flop / med / 1e9, 1), "M": M, "K": K, "N": N}), flush=True)
    for var in ([] if a.no_lab else a.variants):
        for dbg in [0] + a.stamp_dbg:
            stamp_run(a, nat, torch, dev, launch, var, dbg)


def stamp_run(a, nat, torch, dev, launch, var, dbg=0):
    """Stamps of the LAB build (dbg 0): per wave group, mean cycles per segment and k-step."""
    nat.call_hip("shifu_gemm_set_tune", 12, 1)
    nat.call_hip("shifu_ring_nt_set_variant", var)
    stamps = torch.zeros(256 * 8 * 8, dtype=torch.int64, device=dev)
    nat.call_hip("shifu_ring_nt_set_lab", dbg, stamps)
    launch()
    torch.cuda.synchronize()
    nat.call_hip("shifu_ring_nt_set_lab", -1, None)
    nat.call_hip("shifu_ring_nt_set_variant", 0)
    nat.call_hip("shifu_gemm_set_tune", 12, 0)
    s = stamps.view(-1, 8, 8).double().cpu()
    s = s[s[:, 0, 6] > 0]
    out = {"variant": f"stamps_v{var}_dbg{dbg}", "blocks": int(s.shape[0])}
    for grp, sl in (("lead", slice(0, 4)), ("lag", slice(4, 8))):
        seg = s[:, sl, :6].mean(dim=(0, 1))
        tot = float(seg.sum())
        steps = float(s[:, sl, 6].mean())
        out[grp] = {k: round(float(v) / steps, 1) for k, v in zip(SEGS, seg)}
        out[grp]["cycles_per_step"] = round(tot / steps, 1)
        out[grp]["share"] = {k: round(float(v) / tot, 3) for k, v in zip(SEGS, seg)}
    hw = s[:, :, 7].long() & 0xffffffff
    out["simd_of_wave"] = [sorted(set(((hw[:, w] >> 4) & 3).tolist())) for w in range(8)]
    out["waves_per_simd_blk0"] = [int(((hw[0] >> 4) & 3).eq(k).sum()) for k in range(4)]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
