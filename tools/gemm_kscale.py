"""Per-tile fixed cost of the 8-phase NT GEMM: time C = A B^T at M = 1M, N = 512 for K = 256..4096
(store and activation epilogues) and fit t(K) = a + b K; a = prologue + epilogue per launch."""
import json

import torch

from shifu_amd.ops import _native as nat


def t(fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it


M, N = 1 << 20, 512
res = {}
for K in (256, 512, 1024, 2048, 4096):
    A = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N, K, device="cuda") * 0.1 - 0.05).to(torch.bfloat16)
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    st = nat.stream_of(A)
    r = {}
    for var, tag in ((3, "8ph"),):
        nat.call_hip("shifu_gemm_set_big", var)
        for name, epi, act in (("store", 2, 2), ("sigmoid", 0, 0)):
            ms = t(lambda: nat.call_hip("shifu_gemm_nt", A, K, B, K, 500, C, N, None, 0, None, 0, None, 0, M, N, K,
                                        epi, act, 500, 1, 0.0, st))
            r[f"{name}_{tag}"] = {"ms": round(ms, 4), "tflops": round(2.0 * M * N * K / ms / 1e9)}
    nat.call_hip("shifu_gemm_set_big", 0)
    ms = t(lambda: torch.matmul(A, B.t(), out=C))
    r["hipblaslt"] = {"ms": round(ms, 4), "tflops": round(2.0 * M * N * K / ms / 1e9)}
    res[K] = r
    print(K, json.dumps(r), flush=True)
    del A, B, C
ks = sorted(res)
for name in ("store_8ph", "sigmoid_8ph", "hipblaslt"):
    xs = [float(k) for k in ks]
    ys = [res[k][name]["ms"] for k in ks]
    n = len(xs)
    mx, my = sum(xs) / n, sum(ys) / n
    b = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
    a = my - b * mx
    res[f"fit_{name}"] = {"fixed_ms": round(a, 4), "ms_per_1k_K": round(b * 1024, 4),
                          "mainloop_tflops": round(2.0 * M * N * 1024 / (b * 1024) / 1e9)}
print(json.dumps(res))
