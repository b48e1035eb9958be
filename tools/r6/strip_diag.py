"""Locate strip-vs-ring mismatches on the shapes that differ (row / column tiles, in-tile offsets)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from shifu_amd.ops import _native as nat

dev = torch.device("cuda")
st = nat.stream_of(torch.empty(1, device=dev))


def run(engine, A, B, C, M, K, N, nb, nv, act):
    nat.call_hip("shifu_gemm_set_tune", 12, 1 if engine == "ring" else 0)
    nat.call_hip("shifu_gemm_set_tune", 14, 1 if engine == "strip" else 0)
    nat.call_hip("shifu_gemm_nt", A, K, B, K, nb, C, N, None, 0, None, 0, None, 0, M, N, K, 0, act, nv, 1, 0.0, st)


for (M, K, N, nb, nv, act) in [(131072, 512, 1024, 1000, 1000, 7), (131072, 512, 1024, 1000, 1000, 0),
                               (131072, 512, 1024, 1024, 1024, 0), (131072, 512, 512, 500, 500, 0),
                               (131072, 1024, 1024, 1000, 1000, 0), (262144, 512, 1024, 1000, 1000, 0)]:
    g = torch.Generator(device=dev).manual_seed(5)
    A = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    B = (torch.randn(nb, K, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    out = {}
    for eng in ("ring", "strip", "strip2"):
        C = torch.full((M, N), 7.0, dtype=torch.bfloat16, device=dev)
        run("strip" if eng == "strip2" else eng, A, B, C, M, K, N, nb, nv, act)
        torch.cuda.synchronize()
        out[eng] = C
    bad = (out["ring"] != out["strip"]).nonzero()
    rep = {"M": M, "K": K, "N": N, "NB": nb, "act": act, "mismatches": int(bad.shape[0]),
           "strip_repeat_equal": bool(torch.equal(out["strip"], out["strip2"]))}
    if bad.shape[0]:
        r, c = bad[:, 0], bad[:, 1]
        rep.update(row_tiles=sorted(set((r // 256).tolist()))[:20], col_tiles=sorted(set((c // 256).tolist())),
                   row_in_tile=[int((r % 256).min()), int((r % 256).max())], col_in_tile=[int((c % 256).min()), int((c % 256).max())],
                   rows_unique=int(torch.unique(r).numel()), cols_unique=int(torch.unique(c).numel()),
                   max_abs=float((out["ring"].float() - out["strip"].float()).abs().max()))
    print(json.dumps(rep), flush=True)
