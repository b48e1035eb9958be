"""GPU MLP shapes beyond the register-resident output kernel (last hidden >= 512 wide, more than
8 outputs): the any-shape output kernel (mlp_kernels.hip mlp_output_wide_kernel) + the TN wgrad,
against the fp32 CPU trainer on the same bf16-rounded inputs and weights.

The reference builds any width and any number of output nodes (J/core/dtrain/DTrainUtils.java:
303-386; NATIVE multi-class has one sigmoid output per tag, ModelConfig.java:381-384)."""
import numpy as np
import pytest
import torch

from shifu_amd.models.nn import MLPSpec, MLPTrainer

pytestmark = pytest.mark.gpu

SHAPES = [
    ([1000], ["sigmoid"], 1),                  # one wide layer
    ([700, 600], ["tanh", "relu"], 1),         # two wide layers
    ([64], ["sigmoid"], 12),                   # 12-class NATIVE (one output per tag)
    ([300, 520], ["sigmoid", "ptanh"], 10),    # stored-derivative activation under a wide head
]


def _data(spec, n, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, spec.n_in, generator=g).bfloat16().float()
    if spec.n_out == 1:
        y = (x[:, :3].sum(1, keepdim=True) > 0).float()
    else:                                       # one-hot tags from a hidden linear rule
        cls = (x[:, : spec.n_out] * torch.linspace(1, 2, spec.n_out)).argmax(1)
        y = torch.nn.functional.one_hot(cls, spec.n_out).float()
    s = torch.rand(n, generator=g) + 0.5
    return x, y, s


def _pair(spec, seed=5):
    cpu = MLPTrainer(spec, device="cpu", seed=seed, chunk_rows=1000, propagation="R")
    gpu = MLPTrainer(spec, device="cuda", seed=seed, chunk_rows=1024, propagation="R")
    cpu.params.flat.copy_(cpu.params.flat.bfloat16().float())
    gpu.params.flat.copy_(cpu.params.flat.cuda())
    return cpu, gpu


@pytest.mark.parametrize("hidden,acts,n_out", SHAPES)
def test_wide_shapes_first_gradient_and_rprop_epochs(hidden, acts, n_out):
    spec = MLPSpec(n_in=90, hidden=hidden, acts=acts, n_out=n_out)
    cpu, gpu = _pair(spec)
    assert gpu.wide_out == (spec.layer_kpad[-1] > 512 or n_out > 8)
    assert not gpu.fused_head
    x, y, s = _data(spec, 3000)
    dc, dg = cpu.prepare(x, y, s), gpu.prepare(x, y, s)
    # first gradient
    cpu.grad.zero_(); cpu.err_acc.zero_(); cpu.accumulate_gradients(dc)
    gpu.grad.zero_(); gpu.err_acc.zero_(); gpu.accumulate_gradients(dg)
    torch.cuda.synchronize()
    gc, gg = cpu.grad, gpu.grad.cpu()
    assert float((gc - gg).norm() / gc.norm()) < 3e-2
    for vc, vg in zip(cpu.params.views(gc), gpu.params.views(gg)):
        assert float((vc - vg).norm() / vc.norm().clamp(min=1e-12)) < 5e-2
    assert abs(float(cpu.err_acc[0]) - float(gpu.err_acc[0])) / float(cpu.err_acc[0]) < 1e-2
    assert abs(float(cpu.err_acc[1]) - float(gpu.err_acc[1])) < 1e-2
    # 4 RPROP epochs, each from the GPU trainer's current weights and optimizer state (the CPU
    # trainer is re-synced before every epoch, so bf16 rounding cannot compound through a chaotic
    # RPROP trajectory): same training error, same update direction on every weight whose
    # gradient is not lost in bf16 rounding
    for epoch in range(4):
        cpu.params.flat.copy_(gpu.params.flat.cpu())
        for k in ("s0", "s1", "s2"):
            getattr(cpu.opt, k).copy_(getattr(gpu.opt, k).cpu())
        cpu.opt.iteration, cpu.opt.lr = gpu.opt.iteration, gpu.opt.lr
        w0 = cpu.params.flat.clone()
        ec, eg = cpu.step(dc), gpu.step(dg)
        assert abs(eg - ec) / ec < 1e-2, (epoch, eg, ec)
        gc, gg = cpu.grad, gpu.grad.cpu()
        assert float((gc - gg).norm() / gc.norm()) < 3e-2, epoch
        big = gc.abs() > 0.05 * gc.abs().max()
        assert bool(big.any())
        dcpu, dgpu = (cpu.params.flat - w0)[big], (gpu.params.flat.cpu() - w0)[big]
        agree = float((torch.sign(dcpu) == torch.sign(dgpu)).float().mean())
        assert agree > 0.995, (epoch, agree)


@pytest.mark.parametrize("hidden,acts,n_out", SHAPES[:3])
def test_wide_shapes_predict_matches_cpu(hidden, acts, n_out):
    spec = MLPSpec(n_in=90, hidden=hidden, acts=acts, n_out=n_out)
    cpu, gpu = _pair(spec, seed=8)
    x, y, s = _data(spec, 2500, seed=1)
    pc = cpu.predict_rows(cpu.prepare(x, y, s).x)
    pg = gpu.predict_rows(gpu.prepare(x, y, s).x).cpu()
    assert pg.shape == (2500, n_out)
    assert float((pc - pg).abs().max()) < 2e-2


def test_tensorflow_alg_wide_layer_tracks_autograd():
    """TENSORFLOW algorithm on the MLP engine with a 1000-wide hidden layer."""
    from shifu_amd.models.dnn_sgd import train_dnn, train_dnn_autograd
    g = np.random.default_rng(4)
    X = torch.from_numpy(g.normal(size=(3000, 40)).astype(np.float32)).bfloat16().float().numpy()
    y = (X[:, 0] - X[:, 3] > 0).astype(np.float32)
    w = np.ones(3000, np.float32)
    valid = g.random(3000) < 0.2
    p = {"NumHiddenNodes": [1000], "ActivationFunc": ["tanh"], "LearningRate": 0.002, "WeightInitializer": "xavier",
         "MiniBatchs": 500, "TF.optimizer": "adam", "TF.loss": "log"}
    m1, h1 = train_dnn(X, y, w, valid, p, 3, torch.device("cuda"), seed=2)
    m2, h2 = train_dnn_autograd(X, y, w, valid, p, 3, torch.device("cpu"), seed=2)
    v1, v2 = [v for _, _, v in h1], [v for _, _, v in h2]
    np.testing.assert_allclose(v1, v2, rtol=0.05)
    np.testing.assert_allclose([t for _, t, _ in h1], [t for _, t, _ in h2], rtol=0.05)


@pytest.mark.parametrize("hidden,acts,n_out,loss", [([96, 40], ["tanh", "sigmoid"], 3, "squared"),
                                                    ([200], ["ptanh"], 1, "log"),
                                                    ([64], ["relu"], 8, "absolute")])
def test_wide_output_kernel_matches_register_kernel(hidden, acts, n_out, loss, monkeypatch):
    """Where both output kernels apply (last hidden <= 511, <= 8 outputs), the any-shape kernel
    (forced by SHIFU_WIDE_OUTPUT=1) gives the register kernel's errors and gradients; the output
    wgrad differs only by its bf16 delta operand."""
    spec = MLPSpec(n_in=70, hidden=hidden, acts=acts, n_out=n_out, loss=loss)
    a = MLPTrainer(spec, device="cuda", seed=4, chunk_rows=4096)
    monkeypatch.setenv("SHIFU_WIDE_OUTPUT", "1")
    b = MLPTrainer(spec, device="cuda", seed=4, chunk_rows=4096)
    assert b.wide_out and not a.wide_out
    b.params.flat.copy_(a.params.flat)
    x, y, s = _data(spec, 9000, seed=2)
    da, db = a.prepare(x, y, s), b.prepare(x, y, s)
    for t, d in ((a, da), (b, db)):
        t.grad.zero_(); t.err_acc.zero_(); t.accumulate_gradients(d)
    torch.cuda.synchronize()
    assert abs(float(a.err_acc[0]) - float(b.err_acc[0])) / float(a.err_acc[0]) < 1e-5
    assert abs(float(a.err_acc[1]) - float(b.err_acc[1])) / float(a.err_acc[1]) < 1e-9
    for va, vb in zip(a.params.views(a.grad), b.params.views(b.grad)):
        assert float((va - vb).norm() / va.norm().clamp(min=1e-12)) < 1e-2
    pa, pb = a.predict_rows(da.x), b.predict_rows(db.x)
    assert float((pa - pb).abs().max()) < 1e-5
