"""hipBLASLt (through torch) at the MLP bench GEMM shapes, random operands: the library bar the
hand-written kernels are measured against (2M-row chunk, 1000-500-200-1 padded to 1024/512/256).

    python tools/blaslt_probe.py [--rows 2097152]
"""
import argparse
import json

import torch


def timeit(fn, iters=10):
    for _ in range(3):
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
    ap.add_argument("--rows", type=int, default=1 << 21)
    a = ap.parse_args()
    M = a.rows
    bf = torch.bfloat16
    dev = torch.device("cuda")
    X = (torch.rand(M, 1024, device=dev) * 2 - 1).to(bf)
    D1 = (torch.rand(M, 512, device=dev) * 2 - 1).to(bf)
    W1 = (torch.rand(512, 1024, device=dev) * 2 - 1).to(bf)
    H1 = torch.empty(M, 512, device=dev, dtype=bf)
    res = {}
    fl = 2.0 * M * 512 * 1024
    ms = timeit(lambda: torch.mm(X, W1.t(), out=H1))
    res["fwd1_nt_bf16out"] = {"ms": round(ms, 4), "tflops": round(fl / ms / 1e9, 1)}
    G = torch.empty(512, 1024, device=dev, dtype=bf)
    ms = timeit(lambda: torch.mm(D1.t(), X, out=G))
    res["wgrad0_tn_bf16out"] = {"ms": round(ms, 4), "tflops": round(fl / ms / 1e9, 1)}
    try:
        ms = timeit(lambda: torch.mm(D1.t(), X, out_dtype=torch.float32))
        res["wgrad0_tn_f32out"] = {"ms": round(ms, 4), "tflops": round(fl / ms / 1e9, 1)}
    except Exception as e:  # out_dtype not supported by this torch build
        res["wgrad0_tn_f32out"] = f"unsupported: {type(e).__name__}: {str(e)[:120]}"
    D2 = (torch.rand(M, 256, device=dev) * 2 - 1).to(bf)
    W2t = (torch.rand(512, 256, device=dev) * 2 - 1).to(bf)
    fl2 = 2.0 * M * 512 * 256
    ms = timeit(lambda: torch.mm(D2, W2t.t(), out=H1))
    res["dgrad1_nt"] = {"ms": round(ms, 4), "tflops": round(fl2 / ms / 1e9, 1)}
    G2 = torch.empty(256, 512, device=dev, dtype=bf)
    ms = timeit(lambda: torch.mm(D2.t(), H1, out=G2))
    res["wgrad1_tn"] = {"ms": round(ms, 4), "tflops": round(fl2 / ms / 1e9, 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
