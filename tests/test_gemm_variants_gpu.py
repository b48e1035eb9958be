"""Every NT GEMM code path (auto dispatch, 256x256 8-phase forced, 128x128 register-staged forced)
against a torch fp32 reference, for the forward (act), dgrad (dact) and store epilogues."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("variant", [0, 3, 4])
@pytest.mark.parametrize("epi", ["act", "dact", "store"])
@pytest.mark.parametrize("K", [320, 1024])
def test_gemm_nt_variants(variant, epi, K):
    from shifu_amd.ops import _native as nat
    torch.manual_seed(0)
    M, N, NB, nv = 70000 + 37, 512, 500, 500
    dev = "cuda"
    A = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
    B = (torch.randn(NB, K, device=dev) * 0.05).to(torch.bfloat16)
    H = torch.rand(M, N, device=dev).to(torch.bfloat16)
    C = torch.full((M, N), 7.0, device=dev).to(torch.bfloat16)
    nat.call_hip("shifu_gemm_set_big", variant)
    try:
        st = nat.stream_of(A)
        e = {"act": 0, "dact": 1, "store": 2}[epi]
        nat.call_hip("shifu_gemm_nt", A, K, B, K, NB, C, N, None, 0, H if epi == "dact" else None, N, None, 0,
                     M, N, K, e, 1, nv, 1, 0.0, st)
        torch.cuda.synchronize()
    finally:
        nat.call_hip("shifu_gemm_set_big", 0)
    z = A.float() @ B.float().t()                       # [M, NB]
    ref = torch.zeros(M, N, device=dev)
    if epi == "act":
        ref[:, :nv] = torch.tanh(z[:, :nv])
        ref[:, nv] = 1.0
    elif epi == "dact":
        h = H.float()[:, :nv]
        ref[:, :nv] = z[:, :nv] * (1 - h * h)
    else:
        ref[:, :NB] = z
    torch.testing.assert_close(C.float(), ref, rtol=2e-2, atol=2e-2)
