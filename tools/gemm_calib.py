"""Calibrate the NT GEMM variants on square and MLP shapes (EPI_STORE, random operands) against
torch.matmul (hipBLASLt) on the same data; prints TF/s per (shape, variant)."""
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


res = {}
for (M, N, K) in [(4096, 4096, 4096), (8192, 8192, 8192), (1 << 20, 512, 1024), (1 << 20, 256, 512)]:
    A = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    st = nat.stream_of(A)
    fl = 2.0 * M * N * K
    r = {}
    for v in (0, 3, 4):       # auto / 8-phase / 128x128
        nat.call_hip("shifu_gemm_set_big", v)
        ms = t(lambda: nat.call_hip("shifu_gemm_nt", A, K, B, K, N, C, N, None, 0, None, 0, None, 0, M, N, K, 2,
                                    2, N, 0, 0.0, st))
        r[f"v{v}"] = round(fl / ms / 1e9)
    nat.call_hip("shifu_gemm_set_big", 0)
    ms = t(lambda: torch.matmul(A, B.t(), out=C))
    r["hipblaslt"] = round(fl / ms / 1e9)
    res[f"{M}x{N}x{K}"] = r
print(json.dumps(res))
