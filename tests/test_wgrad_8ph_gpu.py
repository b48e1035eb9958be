"""8-phase TN wgrad kernel (gemm_kernels.hip: wgrad_8ph_kernel) vs torch fp32 on bf16 inputs:
row counts with a tail (M % 64 != 0, handled by the 128x128 kernel), output widths that do not
fill a 256 tile, input widths that are not multiples of 256, accumulation into a nonzero G; contiguous and interleaved row splits."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("Nv,ldd,Kx", [(500, 512, 1024), (200, 256, 512), (130, 192, 384)])
@pytest.mark.parametrize("variant", [3, 4])
@pytest.mark.parametrize("interleave", [0, 1])
def test_wgrad_8ph_matches_torch(Nv, ldd, Kx, variant, interleave):
    from shifu_amd.ops import _native as nat
    torch.manual_seed(0)
    M = 70000 + 37
    dev = "cuda"
    D = (torch.randn(M, ldd, device=dev) * 0.1).to(torch.bfloat16)
    X = torch.randn(M, Kx, device=dev).to(torch.bfloat16)
    G0 = torch.randn(Nv, Kx, device=dev)
    G = G0.clone()
    nat.call_hip("shifu_gemm_set_big", variant)
    nat.call_hip("shifu_gemm_set_tune", 2, interleave)     # interleaved 64-row split steps
    try:
        nat.call_hip("shifu_wgrad_tn", D, ldd, X, Kx, G, Kx, M, Nv, Kx, 64, nat.stream_of(D))
        torch.cuda.synchronize()
    finally:
        nat.call_hip("shifu_gemm_set_big", 0)
        nat.call_hip("shifu_gemm_set_tune", 2, 1)
    ref = G0 + D[:, :Nv].float().t() @ X.float()
    torch.testing.assert_close(G, ref, rtol=2e-3, atol=2e-2)
