"""Micro-benchmark of the MLP HIP kernels at the bench shapes (1000-500-200-1, 1M-row chunk):
forward GEMMs, dgrad, wgrad and the output kernel, timed with HIP events; prints TF/s."""
import argparse
import json

import torch

from shifu_amd.models.nn import ACT_IDS
from shifu_amd.ops import _native as nat


def timeit(fn, iters):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1 << 20)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--stages", type=int, default=1)
    ap.add_argument("--big", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=0)
    ap.add_argument("--act", default="sigmoid")
    ap.add_argument("--only", nargs="*", default=None)
    ap.add_argument("--ab", type=lambda t: (t.split("=")[0], int(t.split("=")[1])), nargs="*",
                    help="interleaved A/B settings, e.g. interleave=0 interleave=1 out_waves=4096 out_waves=16384")
    ap.add_argument("--tune", type=lambda t: tuple(int(x) for x in t.split("=")), nargs="*")
    ap.add_argument("--out-waves", type=int, default=0)
    a = ap.parse_args()
    nat.call_hip("shifu_gemm_set_stages", a.stages)
    nat.call_hip("shifu_gemm_set_big", a.big)
    M = a.rows
    dev = torch.device("cuda")
    bf = torch.bfloat16
    X = torch.randn(M, 1024, device=dev).to(bf)
    W1 = (torch.randn(500, 1024, device=dev) * 0.03).to(bf)
    H1 = torch.empty(M, 512, device=dev, dtype=bf)
    W2 = (torch.randn(200, 512, device=dev) * 0.05).to(bf)
    H2 = torch.empty(M, 256, device=dev, dtype=bf)
    W2t = (torch.randn(512, 256, device=dev) * 0.05).to(bf)
    D2 = torch.randn(M, 256, device=dev).to(bf)
    D1 = torch.empty(M, 512, device=dev, dtype=bf)
    G1 = torch.zeros(500, 1024, device=dev)
    G2 = torch.zeros(200, 512, device=dev)
    st = nat.stream_of(X)
    tanh = ACT_IDS[a.act]
    res = {}

    def fwd1():
        nat.call_hip("shifu_gemm_nt", X, 1024, W1, 1024, 500, H1, 512, None, 0, None, 0, None, 0, M, 512, 1024, 0,
                     tanh, 500, 1, 0.0, st)

    def fwd2():
        nat.call_hip("shifu_gemm_nt", H1, 512, W2, 512, 200, H2, 256, None, 0, None, 0, None, 0, M, 256, 512, 0,
                     tanh, 200, 1, 0.0, st)

    def dgrad():
        nat.call_hip("shifu_gemm_nt", D2, 256, W2t, 256, 512, D1, 512, None, 0, H1, 512, None, 0, M, 512, 256, 1,
                     tanh, 500, 0, 0.0, st)

    def spl(hidden, kpad):       # same split rule as MLPTrainer._chunk_hip
        ntiles = -(-hidden // 128) * (kpad // 128)
        return max(1, min(M // 256, 1024 // max(1, ntiles)))

    def wgrad1():
        nat.call_hip("shifu_wgrad_tn", D1, 512, X, 1024, G1, 1024, M, 500, 1024, spl(500, 1024), st)

    def wgrad2():
        nat.call_hip("shifu_wgrad_tn", D2, 256, H1, 512, G2, 512, M, 200, 512, spl(200, 512), st)

    Cs = torch.empty(M, 512, device=dev, dtype=bf)

    def pure():                 # plain GEMM (store epilogue) at the forward-1 shape
        nat.call_hip("shifu_gemm_nt", X, 1024, W1, 1024, 500, Cs, 512, None, 0, None, 0, None, 0, M, 512, 1024, 2,
                     2, 500, 0, 0.0, st)

    W1p = torch.zeros(512, 1024, device=dev, dtype=bf)
    W1p[:500] = W1

    def blaslt():               # hipBLASLt through torch at the same shape (library reference)
        torch.mm(X, W1p.t(), out=Cs)

    G3 = torch.zeros(1, 256, device=dev)
    Y = torch.rand(M, 1, device=dev)
    W3 = (torch.randn(1, 256, device=dev) * 0.05)
    err = torch.zeros(2, device=dev, dtype=torch.float64)

    def output():
        nat.call_hip("shifu_mlp_output", H2, 256, None, 0, W3, Y, 1, None, D2, 256, G3, err, None, 0,
                     M, 256, 200, 1, ACT_IDS["sigmoid"], tanh, 0, 0.0, 0.0, st)

    for k, v in (a.tune or []):
        nat.call_hip("shifu_gemm_set_tune", k, v)
    if a.out_waves:
        nat.call_hip("shifu_mlp_set_out_waves", a.out_waves)
    # A/B rounds inside one process (interleaved): knob settings from --ab
    for rnd in range(a.rounds):
        for setting in (a.ab or [None]):
            if setting is not None:
                kind, val = setting
                if kind in ("interleave", "interleave8"):   # wgrad row-split layout (big 0 / big 3)
                    nat.call_hip("shifu_gemm_set_big", 3 if kind == "interleave8" else 0)
                    nat.call_hip("shifu_gemm_set_tune", 2, val)
                    for nm, f in (("wgrad1", wgrad1), ("wgrad2", wgrad2)):
                        ms = timeit(f, a.iters)
                        res.setdefault(f"{nm}_{kind}{val}", []).append(round(ms, 4))
                    nat.call_hip("shifu_gemm_set_tune", 2, 0)
                    nat.call_hip("shifu_gemm_set_big", a.big)
                elif kind == "out_waves":
                    nat.call_hip("shifu_mlp_set_out_waves", val)
                    ms = timeit(output, a.iters)
                    res.setdefault(f"output_w{val}", []).append(round(ms, 4))
    todo = (("output", output, 0),
                            ("pure_gemm", pure, 2 * M * 512 * 1024), ("torch_mm", blaslt, 2 * M * 512 * 1024),
                            ("fwd1", fwd1, 2 * M * 512 * 1024), ("fwd2", fwd2, 2 * M * 256 * 512),
                            ("dgrad1", dgrad, 2 * M * 512 * 256), ("wgrad1", wgrad1, 2 * M * 512 * 1024),
                            ("wgrad2", wgrad2, 2 * M * 256 * 512))
    for name, fn, flops in todo:
        if a.only and name not in a.only:
            continue
        ms = timeit(fn, a.iters)
        res[name] = {"ms": round(ms, 4), "tflops": round(flops / ms / 1e9, 1)}
        if name == "dgrad1":
            res[name]["hbm_gbs"] = round((M * 256 * 2 + 2 * M * 512 * 2) / ms / 1e6, 1)
        if name == "output":
            res[name]["hbm_gbs"] = round((2 * M * 256 * 2 + M * 4) / ms / 1e6, 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
