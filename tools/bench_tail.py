"""Times the fused MLP tail kernel (ops/csrc/mlp_tail.hip) at the bench shape (1M rows,
h1 = 512 padded, h2 = 256 padded, n_out = 1) against the unfused kernels it replaces."""
import json

import torch

from shifu_amd.ops import _native as nat


def timeit(fn, iters=10):
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
    M = 1 << 20
    dev = "cuda"
    bf = torch.bfloat16
    H1 = torch.rand(M, 512, device=dev).to(bf)
    W2 = (torch.randn(200, 512, device=dev) * 0.05).to(bf)
    Wout = torch.randn(1, 256, device=dev) * 0.1
    Y = (torch.rand(M, 1, device=dev) > 0.5).float()
    D2 = torch.empty(M, 256, device=dev, dtype=bf)
    D1 = torch.empty(M, 512, device=dev, dtype=bf)
    H2 = torch.empty(M, 256, device=dev, dtype=bf)
    W2t = (torch.randn(512, 256, device=dev) * 0.05).to(bf)
    GW = torch.zeros(1, 256, device=dev)
    err = torch.zeros(2, dtype=torch.float64, device=dev)
    st = nat.stream_of(H1)
    res = {}

    def tail(bwd, blocks=0):
        def f():
            nat.call_hip("shifu_mlp_tail", H1, 512, W2, 200, 512, 0, 0.1, Wout, 256, Y, 1, None, 1, 0, 0, 0.1,
                         D2, 256, GW, err, bwd, W2t, 256, D1, 512, 0, 500, 0.1, M, blocks, st)
        return f

    def unfused():
        nat.call_hip("shifu_gemm_nt", H1, 512, W2, 512, 200, H2, 256, None, 0, None, 0, None, 0, M, 256, 512, 0,
                     0, 200, 1, 0.1, st)
        nat.call_hip("shifu_mlp_output", H2, 256, None, 0, Wout, Y, 1, None, D2, 256, GW, err, None, 0, M, 256,
                     201, 1, 0, 0, 0, 0.1, 0.1, st)
        nat.call_hip("shifu_gemm_nt", D2, 256, W2t, 256, 512, D1, 512, None, 0, H1, 512, None, 0, M, 512, 256, 1,
                     0, 500, 0, 0.1, st)

    res["tail_fwd_only"] = timeit(tail(0))
    res["tail_full"] = timeit(tail(1))
    res["tail_full_128blk"] = timeit(tail(1, 128))
    res["tail_full_1024blk"] = timeit(tail(1, 1024))
    res["unfused_3_kernels"] = timeit(unfused)
    print(json.dumps({k: round(v, 4) for k, v in res.items()}))


if __name__ == "__main__":
    main()
