"""Split-bf16 fp32-accurate GEMM (ops/gemm_ops.py) and the default fp32 NN scoring path.

CPU: the split operands' exact bf16 product reproduces x @ W^T + b to fp32 accuracy (the
construction the HIP GEMM consumes).  GPU: the own-kernel path (split kernel + EPI_F32 GEMM with
the accurate activation epilogue) against an fp64 numpy oracle, and against the vendor fp32 GEMM.
"""
import numpy as np
import pytest
import torch

from shifu_amd.ops.gemm_ops import SplitWeights, linear_fp32, split_bf16


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max())


def test_split_parts_reconstruct_fp32():
    g = torch.Generator().manual_seed(0)
    v = torch.randn(10000, generator=g) * torch.exp(torch.randn(10000, generator=g) * 4)
    hi, mid, lo = split_bf16(v, 3)
    assert torch.equal(hi.double() + mid.double() + lo.double(), v.double())


@pytest.mark.parametrize("terms,tol", [(3, 3e-5), (6, 3e-7)])
def test_split_operands_cpu_product(terms, tol):
    g = torch.Generator().manual_seed(1)
    x = torch.randn(300, 77, generator=g)
    W = torch.randn(19, 77, generator=g) * 0.3
    b = torch.randn(19, generator=g)
    sw = SplitWeights(W, b, terms=terms)
    A = sw.operand(x)
    assert A.shape == (300, sw.kp) and sw.kp % 64 == 0
    got = (A.double() @ sw.B.double().t())                 # exact products of the bf16 parts
    ref = x.double() @ W.double().t() + b.double()
    assert _rel(got, ref) < tol


def test_linear_fp32_cpu_is_torch_oracle():
    x = torch.randn(10, 6)
    W = torch.randn(3, 6)
    b = torch.randn(3)
    assert torch.allclose(linear_fp32(x, W, b, act=0), torch.sigmoid(x @ W.t() + b))


@pytest.mark.gpu
@pytest.mark.parametrize("M,K,N,act", [(70000 + 13, 1000, 500, 0), (4099, 75, 33, 1), (1000, 200, 1, 0),
                                       (513, 130, 70, 5), (2048, 64, 8, 2)])
def test_linear_fp32_gpu_matches_fp64(M, K, N, act):
    from shifu_amd.models.nn import ACT_IDS, act_fwd
    g = torch.Generator().manual_seed(M)
    x = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) / K ** 0.5
    b = torch.randn(N, generator=g) * 0.1
    y = linear_fp32(x.cuda(), W.cuda(), b.cuda(), act=act)
    torch.cuda.synchronize()
    name = {v: k for k, v in ACT_IDS.items()}[act]
    ref = act_fwd(name, x.double() @ W.double().t() + b.double())
    assert y.shape == (M, N)
    err = (y.double().cpu() - ref).abs().max().item()
    assert err < 2e-6 * max(1.0, ref.abs().max().item()), err


@pytest.mark.gpu
def test_split_kernel_matches_torch_split():
    """shifu_split_bf16_rows (vector and scalar paths, strided rows) == the torch split."""
    g = torch.Generator().manual_seed(3)
    for K, ld in ((64, 64), (75, 80), (200, 208)):
        xs = torch.randn(1000, ld, generator=g).cuda()
        x = xs[:, :K]
        sw = SplitWeights(torch.randn(5, K).cuda(), torch.randn(5).cuda(), terms=6)
        A = sw.operand(x).clone()
        xp = split_bf16(x, 3)
        for t, (xi, _) in enumerate(sw.pairs):
            assert torch.equal(A[:, t * K:(t + 1) * K], xp[xi])
        assert torch.equal(A[:, sw.kb:sw.kb + 6].float().cpu(),
                           torch.tensor([1.0, 1, 0, 1, 0, 0]).expand(1000, 6))


@pytest.mark.gpu
def test_nn_scoring_fp32_own_kernels_vs_fp64():
    """Default fp32 NN scoring (own split-bf16 GEMM) agrees with an fp64 oracle to ~1e-6 and with
    the vendor fp32 GEMM path; chunk boundaries and an input-subset net included."""
    from shifu_amd.formats.nn_format import NNNetwork
    from shifu_amd.scoring.model_runner import nn_forward
    rng = np.random.default_rng(4)
    sizes = [300, 120, 40, 2]
    acts = ["tanh", "sigmoid", "sigmoid"]
    net = NNNetwork(sizes, acts, [rng.normal(size=(sizes[i + 1], sizes[i] + 1)) * 0.2 for i in range(3)])
    X = rng.normal(size=(50000, 300)).astype(np.float32)
    a = nn_forward(net, X, torch.device("cuda"), chunk=16384, precision="fp32")
    t = nn_forward(net, X, torch.device("cuda"), chunk=16384, precision="fp32_torch")
    r = X.astype(np.float64)
    for l, W in enumerate(net.weights):
        z = r @ W[:, :-1].T + W[:, -1]
        r = np.tanh(z) if acts[l] == "tanh" else 1 / (1 + np.exp(-z))
    assert a.shape == r.shape == (50000, 2)
    assert np.abs(a - r).max() < 1e-6
    assert np.abs(a - t).max() < 5e-6
