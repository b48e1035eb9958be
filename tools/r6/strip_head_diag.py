"""shifu_strip_head against an fp32 torch reference of the same math (bf16 operands), piece by piece:
head deltas D2, layer-below deltas DZ1, output-wgrad column sums, error sums.  One JSON line per
quantity: max |diff|, reference scale, fraction of exact-zero outputs.

    python tools/r6/strip_head_diag.py [--rows 70077] [--k1 512] [--nv 200] [--nv1 500]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=70077)
    ap.add_argument("--k1", type=int, default=512)
    ap.add_argument("--nv", type=int, default=200)
    ap.add_argument("--nv1", type=int, default=500)
    ap.add_argument("--act", type=int, default=0, help="0 sigmoid, 1 tanh (both layers)")
    ap.add_argument("--repeat", type=int, default=0, help="extra launches compared bitwise with the first")
    a = ap.parse_args()
    import torch
    from shifu_amd.ops import _native as nat
    if os.environ.get("SH_LIB"):                      # a lab build of gemm_strip_head.hip alone
        import ctypes
        lib = ctypes.CDLL(os.environ["SH_LIB"])
        nat._bind(lib, {k: nat.HIP_SIGNATURES[k] for k in
                        ("shifu_strip_head", "shifu_strip_head_rows", "shifu_strip_head_set_dbg_rows")})
        nat._hip = lib
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(3)
    M, K1, nv, nv1 = a.rows, a.k1, a.nv, a.nv1
    H = torch.rand(M, K1, generator=g, device=dev)
    H[:, nv1] = 1.0
    H[:, nv1 + 1:] = 0.0
    H = H.bfloat16()
    W = ((torch.rand(nv, K1, generator=g, device=dev) - 0.5) * 0.2).bfloat16()
    W[:, nv1 + 1:] = 0
    WT = torch.zeros(K1, 256, dtype=torch.bfloat16, device=dev)
    WT[:, :nv] = W.t()
    Wo = ((torch.rand(256, generator=g, device=dev) - 0.5) * 0.5)
    Wo[nv + 1:] = 0
    Y = (torch.rand(M, generator=g, device=dev) > 0.5).float()
    D = torch.full((M, 256), 7.0, dtype=torch.bfloat16, device=dev)
    DZ = torch.full((M, K1), 7.0, dtype=torch.bfloat16, device=dev)
    T = nat.hip().shifu_strip_head_rows(M)
    dbg = torch.full((M, 3), float("nan"), device=dev)
    nat.call_hip("shifu_strip_head_set_dbg_rows", dbg)
    gws = torch.zeros(T, 256, device=dev)
    ers = torch.zeros(T, 2, dtype=torch.float64, device=dev)
    err = torch.zeros(2, dtype=torch.float64, device=dev)
    st = nat.stream_of(H)
    nat.call_hip("shifu_strip_head", H, K1, W, K1, nv, WT, 256, D, 256, DZ, K1, M, K1, nv, nv1, Wo, 256, Y, None,
                 gws, ers, err, a.act, a.act, 0, 0, 0.0, 0.0, 0.0, st)
    torch.cuda.synchronize()
    # reference (squared loss, sigmoid everywhere, no flat spot)
    z2 = H.float() @ W.float().t()                                  # [M, nv]
    a2 = torch.zeros(M, 256, device=dev)
    f = torch.sigmoid if a.act == 0 else torch.tanh
    fd = (lambda v: v * (1 - v)) if a.act == 0 else (lambda v: 1 - v * v)
    a2[:, :nv] = f(z2)
    a2[:, nv] = 1.0
    a2 = a2.bfloat16().float()
    zo = a2 @ Wo
    ao = torch.sigmoid(zo)
    e = Y - ao
    dl = ao * (1 - ao) * e
    d2 = dl[:, None] * Wo[None, :] * fd(a2)
    d2[:, nv:] = 0
    d2b = d2.bfloat16()
    z1 = (d2b.float() @ WT.float().t()).bfloat16().float()
    dz = z1 * fd(H.float())
    dz[:, nv1:] = 0
    gw = (dl[:, None] * a2).sum(0)
    res = {}

    def rep(name, got, ref):
        d = (got.float() - ref.float()).abs()
        res[name] = {"max_abs_diff": float(d.max()), "ref_absmax": float(ref.abs().max()),
                     "frac_zero_got": float((got == 0).float().mean()), "frac_7_got": float((got == 7).float().mean())}
        if d.dim() == 2:
            tol = 0.02 * float(ref.abs().max()) + 1e-6
            bad = d > tol
            res[name]["n_bad"] = int(bad.sum())
            if int(bad.sum()):
                r, c = torch.nonzero(bad, as_tuple=True)
                res[name]["bad_rows_minmax"] = [int(r.min()), int(r.max())]
                res[name]["bad_row_mod256_hist"] = torch.bincount(r % 256 // 32, minlength=8).tolist()
                res[name]["bad_col_hist32"] = torch.bincount(c // 32, minlength=(got.shape[1] + 31) // 32).tolist()
                res[name]["bad_col_mod32_hist"] = torch.bincount(c % 32, minlength=32).tolist()
                bt = torch.unique(r // 256)
                res[name]["bad_tiles"] = bt.tolist()[:40]
                res[name]["n_bad_tiles"] = int(bt.numel())
                i = int(torch.argmax(d.flatten()))
                res[name]["argmax"] = [i // d.shape[1], i % d.shape[1]]
        print(json.dumps({name: res[name]}), flush=True)
    nat.call_hip("shifu_strip_head_set_dbg_rows", None)
    for i, (nm, ref) in enumerate((("zo", zo), ("y", Y), ("dl", dl))):
        d = (dbg[:, i] - ref).abs()
        bad = d > 1e-3 * float(ref.abs().max()) + 1e-6
        out = {"n_bad": int(bad.sum()), "max": float(d.max())}
        if int(bad.sum()):
            r = torch.nonzero(bad)[:, 0]
            out["bad_tiles"] = torch.unique(r // 256).tolist()[:20]
            out["first_bad"] = [int(r[0]), float(dbg[r[0], i]), float(ref[r[0]])]
            out["bad_mod256_hist"] = torch.bincount(r % 256 // 16, minlength=16).tolist()
        print(json.dumps({"row_" + nm: out}), flush=True)
    rep("D2", D, d2b)
    rep("DZ1", DZ, dz.bfloat16())
    rep("gw", gws.sum(0), gw)
    print(json.dumps({"err": [float(err[0]), float(err[1])], "ref_err": [float((e * e).sum()), float(M)],
                      "slab_rows": T}), flush=True)
    if a.repeat:
        D0, Z0, g0 = D.clone(), DZ.clone(), gws.clone()
        nrep = []
        for _ in range(a.repeat):
            D.fill_(7.0); DZ.fill_(7.0)
            nat.call_hip("shifu_strip_head", H, K1, W, K1, nv, WT, 256, D, 256, DZ, K1, M, K1, nv, nv1, Wo, 256, Y,
                         None, gws, ers, err, a.act, a.act, 0, 0, 0.0, 0.0, 0.0, st)
            torch.cuda.synchronize()
            bd = (D != D0).nonzero()
            bz = (DZ != Z0).nonzero()
            nrep.append({"D2_diff": int(bd.shape[0]), "DZ_diff": int(bz.shape[0]), "gw_equal": bool(torch.equal(gws, g0)),
                         "DZ_diff_tiles": torch.unique(bz[:, 0] // 256).tolist()[:10] if bz.shape[0] else [],
                         "DZ_diff_cols": torch.unique(bz[:, 1] // 64).tolist() if bz.shape[0] else []})
        print(json.dumps({"repeat": nrep}), flush=True)
    # first rows in detail
    print(json.dumps({"D2_row0_got": [float(v) for v in D[0, :8]], "D2_row0_ref": [float(v) for v in d2b[0, :8]],
                      "DZ_row0_got": [float(v) for v in DZ[0, :8]], "DZ_row0_ref": [float(v) for v in dz[0, :8]]}))


if __name__ == "__main__":
    main()
