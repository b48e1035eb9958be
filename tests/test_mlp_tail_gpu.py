"""Fused MLP tail kernel (ops/csrc/mlp_tail.hip) vs the unfused HIP kernels and the fp32 oracle:
same gradients, errors and last-hidden deltas for one/two/three hidden layers, several output
widths and all three losses, with a row count that is not a multiple of the 128-row tile."""
import pytest
import torch

from shifu_amd.models.nn import MLPSpec, MLPTrainer

pytestmark = pytest.mark.gpu


def _grads(spec, x, y, s, fused, loss_seed=5, chunk=4096):
    tr = MLPTrainer(spec, device="cuda", seed=loss_seed, chunk_rows=chunk)
    tr.fused_tail = fused and tr._tail_supported()
    d = tr.prepare(x, y, s)
    tr.grad.zero_()
    tr.err_acc.zero_()
    tr.accumulate_gradients(d)
    torch.cuda.synchronize()
    return tr, tr.grad.cpu().clone(), tr.err_acc.cpu().clone()


@pytest.mark.parametrize("hidden,acts,n_out,loss", [
    ([64], ["sigmoid"], 1, "squared"),
    ([96, 40], ["tanh", "sigmoid"], 1, "squared"),
    ([300, 200], ["sigmoid", "sigmoid"], 1, "log"),
    ([130, 70, 33], ["relu", "tanh", "sigmoid"], 3, "absolute"),
    ([500, 200], ["sigmoid", "sigmoid"], 2, "squared"),
])
def test_fused_tail_matches_unfused(hidden, acts, n_out, loss):
    spec = MLPSpec(n_in=123, hidden=hidden, acts=acts, n_out=n_out, loss=loss)
    g = torch.Generator().manual_seed(1)
    n = 10000 + 77
    x = torch.randn(n, spec.n_in, generator=g)
    y = (torch.rand(n, n_out, generator=g) > 0.5).float()
    s = torch.rand(n, generator=g) + 0.5
    tf, gf, ef = _grads(spec, x, y, s, True)
    assert tf.fused_tail, "fused tail kernel not selected for an eligible net"
    tu, gu, eu = _grads(spec, x, y, s, False)
    rel = (gf - gu).norm() / gu.norm()
    assert rel < 1e-2, float(rel)
    for vf, vu in zip(tf.params.views(gf), tu.params.views(gu)):
        r = (vf - vu).norm() / vu.norm().clamp(min=1e-12)
        assert r < 2e-2, float(r)
    assert abs(float(ef[0]) - float(eu[0])) <= 1e-4 * abs(float(eu[0])) + 1e-6
    assert abs(float(ef[1]) - float(eu[1])) <= 1e-6 * abs(float(eu[1]))


def test_fused_tail_vs_cpu_oracle_bench_shape():
    spec = MLPSpec(n_in=1000, hidden=[500, 200], acts=["sigmoid", "sigmoid"], n_out=1)
    g = torch.Generator().manual_seed(3)
    n = 6000 + 5
    x = torch.randn(n, spec.n_in, generator=g).bfloat16().float()
    y = (torch.rand(n, 1, generator=g) > 0.5).float()
    cpu = MLPTrainer(spec, device="cpu", seed=9, chunk_rows=2000)
    cpu.params.flat.copy_(cpu.params.flat.bfloat16().float())
    gpu = MLPTrainer(spec, device="cuda", seed=9, chunk_rows=4096)
    gpu.fused_tail = gpu._tail_supported()
    assert gpu.fused_tail
    gpu.params.flat.copy_(cpu.params.flat.cuda())
    dc, dg = cpu.prepare(x, y), gpu.prepare(x, y)
    cpu.grad.zero_(); cpu.err_acc.zero_(); cpu.accumulate_gradients(dc)
    gpu.grad.zero_(); gpu.err_acc.zero_(); gpu.accumulate_gradients(dg)
    torch.cuda.synchronize()
    gc, gg = cpu.grad, gpu.grad.cpu()
    assert (gc - gg).norm() / gc.norm() < 3e-2
    for vc, vg in zip(cpu.params.views(gc), gpu.params.views(gg)):
        assert (vc - vg).norm() / vc.norm().clamp(min=1e-12) < 5e-2
    assert abs(float(cpu.err_acc[0]) - float(gpu.err_acc[0].cpu())) / float(cpu.err_acc[0]) < 1e-2
