"""HIP MLP kernels vs the fp32 PyTorch oracle (same bf16-rounded inputs)."""
import pytest
import torch

from shifu_amd.models.nn import MLPSpec, MLPTrainer, TrainData

pytestmark = pytest.mark.gpu
STRIP_DEFAULT = 1          # gemm_kernels.hip g_strip_nt (tune key 14) as built


def _mk(spec, n, seed=0, loss="squared"):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, spec.n_in, generator=g).bfloat16().float()
    y = (torch.rand(n, spec.n_out, generator=g) > 0.5).float()
    s = torch.rand(n, generator=g) + 0.5
    return x, y, s


@pytest.mark.parametrize("hidden,acts", [([64], ["sigmoid"]), ([96, 40], ["tanh", "sigmoid"]),
                                         ([130, 70, 33], ["relu", "swish", "sigmoid"])])
def test_gradients_match_cpu_oracle(hidden, acts):
    spec = MLPSpec(n_in=75, hidden=hidden, acts=acts, n_out=1)
    n = 3000
    x, y, s = _mk(spec, n)
    cpu = MLPTrainer(spec, device="cpu", seed=5, chunk_rows=1000)
    gpu = MLPTrainer(spec, device="cuda", seed=5, chunk_rows=1024)
    # make the oracle use exactly the bf16-rounded weights of the GPU path
    cpu.params.flat.copy_(cpu.params.flat.bfloat16().float())
    gpu.params.flat.copy_(cpu.params.flat.cuda())
    dc, dg = cpu.prepare(x, y, s), gpu.prepare(x, y, s)
    cpu.grad.zero_(); cpu.err_acc.zero_(); cpu.accumulate_gradients(dc)
    gpu.grad.zero_(); gpu.err_acc.zero_(); gpu.accumulate_gradients(dg)
    torch.cuda.synchronize()
    gc, gg = cpu.grad, gpu.grad.cpu()
    rel = (gc - gg).norm() / gc.norm()
    assert rel < 3e-2, float(rel)
    for vc, vg in zip(cpu.params.views(gc), gpu.params.views(gg)):
        r = (vc - vg).norm() / vc.norm().clamp(min=1e-12)
        assert r < 5e-2, float(r)
    assert abs(float(cpu.err_acc[0]) - float(gpu.err_acc[0].cpu())) / float(cpu.err_acc[0]) < 1e-2
    assert abs(float(cpu.err_acc[1]) - float(gpu.err_acc[1].cpu())) < 1e-2


def test_gemm_nt_epilogue_exact_small():
    """Identity-weight check with an ASYMMETRIC B: catches a transposed C write."""
    from shifu_amd.ops import _native as nat
    M, K, NB = 300, 128, 70
    a = (torch.arange(M * K, dtype=torch.float32).reshape(M, K) % 7 - 3).bfloat16().cuda()
    b = (torch.arange(NB * K, dtype=torch.float32).reshape(NB, K) % 5 - 2).bfloat16().cuda()
    N = 128
    c = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    nat.call_hip("shifu_gemm_nt", a.data_ptr(), K, b.data_ptr(), K, NB, c.data_ptr(), N, None, 0, None, 0,
                 None, 0, M, N, K, 2, 2, NB, 0, 0.0, nat.stream_of(a))
    ref = a.float() @ b.float().t()
    torch.cuda.synchronize()
    assert torch.allclose(c[:, :NB].float(), ref.bfloat16().float(), atol=0.5)
    assert torch.all(c[:, NB:] == 0)


def test_wgrad_tn_matches_torch():
    from shifu_amd.ops import _native as nat
    M, Nv, Kx = 5000, 150, 256
    g = torch.Generator(device="cuda").manual_seed(0)
    d = torch.randn(M, 256, generator=g, device="cuda").bfloat16()
    d[:, Nv:] = 0
    x = torch.randn(M, Kx, generator=g, device="cuda").bfloat16()
    G = torch.zeros(Nv, Kx, device="cuda")
    nat.call_hip("shifu_wgrad_tn", d.data_ptr(), 256, x.data_ptr(), Kx, G.data_ptr(), Kx, M, Nv, Kx, 7,
                 nat.stream_of(d))
    ref = d[:, :Nv].float().t() @ x.float()
    torch.cuda.synchronize()
    assert torch.allclose(G, ref, atol=1e-2, rtol=1e-3), float((G - ref).abs().max())


def test_training_converges_on_gpu():
    spec = MLPSpec(n_in=40, hidden=[64, 32], acts=["sigmoid", "sigmoid"], n_out=1)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(20000, 40, generator=g)
    y = (x[:, :3].sum(1, keepdim=True) > 0).float()
    tr = MLPTrainer(spec, device="cuda", seed=3, propagation="R", chunk_rows=8192)
    data = tr.prepare(x, y)
    errs = [tr.step(data) for _ in range(25)]
    assert errs[-1] < 0.5 * errs[0], errs
    p = tr.predict_rows(data.x).cpu()
    acc = ((p > 0.5).float() == y).float().mean()
    assert acc > 0.9, float(acc)


def test_optimizer_kernel_matches_cpu():
    from shifu_amd.models.nn import Optimizer
    torch.manual_seed(0)
    for rule in ["R", "B", "Q", "M", "ADAM", "ADAGRAD", "RMSPROP", "MOMENTUM", "NESTEROV"]:
        oc = Optimizer(1000, "cpu", rule, learning_rate=0.05, learning_decay=0.1)
        og = Optimizer(1000, "cuda", rule, learning_rate=0.05, learning_decay=0.1)
        wc = torch.randn(1000)
        wg = wc.clone().cuda()
        for _ in range(4):
            gr = torch.randn(1000)
            oc.step(wc, gr, 100)
            og.step(wg, gr.cuda(), 100)
        torch.cuda.synchronize()
        assert torch.allclose(wc, wg.cpu(), atol=1e-4, rtol=1e-4), rule


@pytest.mark.parametrize("hidden,acts,loss", [([300, 200], ["sigmoid", "sigmoid"], "squared"),
                                              ([96, 130], ["relu", "tanh"], "log"),
                                              ([64], ["sigmoid"], "absolute")])
def test_fused_head_matches_unfused(hidden, acts, loss, monkeypatch):
    """gemm_head_8ph_kernel (last hidden forward + output layer + loss + deltas + output wgrad in
    one epilogue) against the unfused GEMM + mlp_output_kernel path: same gradients / errors."""
    spec = MLPSpec(n_in=120, hidden=hidden, acts=acts, n_out=1, loss=loss)
    n = 70000 + 77                       # >= 65536 rows per chunk: the fused head is used
    x, y, s = _mk(spec, n, seed=3)
    monkeypatch.setenv("SHIFU_FUSED_HEAD", "1")
    a = MLPTrainer(spec, device="cuda", seed=9, chunk_rows=1 << 20)
    monkeypatch.setenv("SHIFU_FUSED_HEAD", "0")
    b = MLPTrainer(spec, device="cuda", seed=9, chunk_rows=1 << 20)
    assert a.fused_head and not b.fused_head
    b.params.flat.copy_(a.params.flat)
    da, db = a.prepare(x, y, s), b.prepare(x, y, s)
    for t, d in ((a, da), (b, db)):
        t.grad.zero_(); t.err_acc.zero_(); t.accumulate_gradients(d)
    torch.cuda.synchronize()
    for va, vb in zip(a.params.views(a.grad), b.params.views(b.grad)):
        r = (va - vb).norm() / vb.norm().clamp(min=1e-12)
        assert r < 1e-2, float(r)
    assert abs(float(a.err_acc[0]) - float(b.err_acc[0])) / float(b.err_acc[0]) < 1e-4
    assert abs(float(a.err_acc[1]) - float(b.err_acc[1])) / float(b.err_acc[1]) < 1e-6


@pytest.mark.parametrize("hidden,acts,loss,n", [
    ([500, 200], ["sigmoid", "sigmoid"], "squared", 70000 + 77),     # the bench's head + layer-1 dgrad
    ([500, 150], ["tanh", "tanh"], "log", 65536 + 1000),             # a partial last tile, two tiles on a few blocks
    ([400, 250], ["relu", "relu"], "absolute", 300000 + 5),          # several tiles per block
])
def test_strip_head_matches_head_plus_dgrad(hidden, acts, loss, n, monkeypatch):
    """gemm_strip_head.hip (head forward + output + loss + head deltas + output wgrad + the layer
    below's dgrad in one persistent kernel, the head deltas kept in registers as the dgrad operand)
    against the 8-phase head kernel + the dgrad tile kernel: same gradients / errors (k order inside
    the MFMA blocks differs: not bitwise), and bitwise reproducible run to run."""
    spec = MLPSpec(n_in=120, hidden=hidden, acts=acts, n_out=1, loss=loss)
    x, y, s = _mk(spec, n, seed=4)
    monkeypatch.setenv("SHIFU_STRIP_HEAD", "1")
    a = MLPTrainer(spec, device="cuda", seed=11, chunk_rows=1 << 20)
    monkeypatch.setenv("SHIFU_STRIP_HEAD", "0")
    b = MLPTrainer(spec, device="cuda", seed=11, chunk_rows=1 << 20)
    assert a.strip_head and b.fused_head and not b.strip_head
    # a 256-wide layer below (K1 = 256) keeps the head + dgrad kernels (gemm_strip_head.hip)
    assert not MLPTrainer(MLPSpec(n_in=120, hidden=[255, 150], acts=acts, n_out=1), device="cuda").strip_head
    b.params.flat.copy_(a.params.flat)
    da, db = a.prepare(x, y, s), b.prepare(x, y, s)
    for t, d in ((a, da), (b, db)):
        t.grad.zero_(); t.err_acc.zero_(); t.accumulate_gradients(d)
    torch.cuda.synchronize()
    g1, e1 = a.grad.clone(), a.err_acc.clone()
    for va, vb in zip(a.params.views(a.grad), b.params.views(b.grad)):
        r = (va - vb).norm() / vb.norm().clamp(min=1e-12)
        assert r < 1e-2, float(r)
    assert abs(float(a.err_acc[0]) - float(b.err_acc[0])) / float(b.err_acc[0]) < 1e-4
    assert abs(float(a.err_acc[1]) - float(b.err_acc[1])) / float(b.err_acc[1]) < 1e-6
    a.grad.zero_(); a.err_acc.zero_(); a.accumulate_gradients(da)
    torch.cuda.synchronize()
    # gradients bitwise; the error sums are per-wave double atomics (equal up to summation order)
    assert torch.equal(a.grad, g1) and torch.allclose(a.err_acc, e1, rtol=1e-12, atol=0)


@pytest.mark.parametrize("M,K,N,NB,nv,epi,act", [
    ((1 << 20) + 77, 1024, 512, 500, 500, 0, 0),       # the bench's first layer (sigmoid + bias column)
    (70000 + 33, 256, 512, 512, 512, 0, 1),           # K = 8 steps per tile, tanh, no partial columns
    (65536 + 300, 128, 264, 260, 260, 2, 2),          # store z, partial last column tile (N % 256 != 0)
    (65536, 384, 384, 256, 256, 0, 0),                # a column tile entirely past the weight rows (n0 >= NB)
])
def test_ring_forward_matches_8phase_and_oracle(M, K, N, NB, nv, epi, act):
    """The persistent ring forward (gemm_ring_nt.hip, tune key 12) against the 8-phase / 128x128
    kernels it replaces (same k order: bitwise equal where the 8-phase kernel runs) and an fp32
    oracle of the same bf16 inputs: activations, the bias column, zero padding, rows >= M untouched."""
    from shifu_amd.ops import _native as nat
    g = torch.Generator(device="cuda").manual_seed(M % 97)
    A = (torch.randn(M + 64, K, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    B = (torch.randn(NB, K, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    outs = []
    for ring in (0, 1):
        C = torch.full((M + 64, N), 7.0, device="cuda", dtype=torch.bfloat16)
        nat.call_hip("shifu_gemm_set_tune", 12, ring)
        try:
            nat.call_hip("shifu_gemm_nt", A, K, B, K, NB, C, N, None, 0, None, 0, None, 0,
                         M, N, K, epi, act, nv, 1, 0.0, nat.stream_of(A))
            torch.cuda.synchronize()
        finally:
            nat.call_hip("shifu_gemm_set_tune", 12, 1)       # the default
        outs.append(C)
    old, new = outs
    assert torch.all(new[M:] == 7.0), "rows >= M written"
    z = A[:M].float() @ B.float().t()
    ref = {0: torch.sigmoid, 1: torch.tanh, 2: lambda v: v}[act](z)
    assert (new[:M, :min(nv, NB)].float() - ref[:, :min(nv, NB)]).abs().max().item() < 2e-2
    if epi == 0 and nv < N:
        assert torch.all(new[:M, nv] == 1.0) and torch.all(new[:M, nv + 1:] == 0)
    else:
        assert torch.all(new[:M, NB:] == 0)
    if K >= 512 and N >= 512:                         # the 8-phase kernel's shapes: identical bits
        assert torch.equal(old.view(torch.int16), new.view(torch.int16))
    else:
        assert (old.float() - new.float()).abs().max().item() < 2e-2


@pytest.mark.parametrize("M,K,N,NB,nv,act", [
    ((1 << 21), 1024, 512, 500, 500, 0),               # the bench's first layer (sigmoid + bias column)
    ((1 << 20) + 77, 1024, 512, 500, 500, 0),           # a partial last row tile
    (70000 + 33, 256, 512, 512, 512, 3),                # K = 4 steps per tile, relu, no partial columns
    (65536 + 300, 128, 264, 260, 260, 0),               # partial last column tile (N % 256 != 0)
    (65536, 384, 384, 256, 256, 2),                     # a column tile entirely past the weight rows
    (131072, 512, 1024, 1000, 1000, 7),                 # four column tiles, log activation
])
def test_strip_forward_bitwise_equals_ring(M, K, N, NB, nv, act):
    """The row-strip forward (gemm_strip_nt.hip, tune key 14: A fragments global -> VGPR, B by
    LDS-DMA in 64-deep k-steps) against the ring engine: the same k order per accumulator, so the
    outputs are identical bits, rows >= M untouched."""
    from shifu_amd.ops import _native as nat
    g = torch.Generator(device="cuda").manual_seed(M % 89)
    A = (torch.randn(M + 64, K, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    B = (torch.randn(NB, K, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    outs = []
    for strip in (0, 1):
        C = torch.full((M + 64, N), 7.0, device="cuda", dtype=torch.bfloat16)
        nat.call_hip("shifu_gemm_set_tune", 14, strip)
        try:
            nat.call_hip("shifu_gemm_nt", A, K, B, K, NB, C, N, None, 0, None, 0, None, 0,
                         M, N, K, 0, act, nv, 1, 0.0, nat.stream_of(A))
            torch.cuda.synchronize()
        finally:
            nat.call_hip("shifu_gemm_set_tune", 14, STRIP_DEFAULT)
        outs.append(C)
    ring, strip = outs
    assert torch.all(strip[M:] == 7.0), "rows >= M written"
    if act in (0, 2, 3):
        assert torch.equal(ring.view(torch.int16), strip.view(torch.int16))
    else:       # __logf / v_log_f32 codegen may differ by an fp32 ulp between the two kernels
        d = (ring.float() - strip.float()).abs()
        assert float(d.max()) <= 2 ** -7 * max(1.0, float(ring.float().abs().max()))
        assert int((d > 0).sum()) < 1e-3 * d.numel()


def test_bench_configuration_tracks_fp32_oracle():
    """The exact bench trainer configuration (bench.py: n_in 1000, hidden 500/200 sigmoid, RPROP,
    chunks >= 2^17 rows) so the persistent ring forward, the fused head, the ring wgrad (incl. the M % 32
    tail) and dgrad all run, for 8 full-batch epochs against the fp32 torch oracle on the same
    bf16-rounded rows and weights: the training-error trajectory agrees within 1e-2 relative and
    the final weights stay close."""
    spec = MLPSpec(n_in=1000, hidden=[500, 200], acts=["sigmoid", "sigmoid"], n_out=1)
    n = (1 << 17) + 77
    g = torch.Generator().manual_seed(11)
    x = torch.randn(n, spec.n_in, generator=g).bfloat16().float()
    wt = torch.randn(spec.n_in, 1, generator=g)
    y = ((x @ wt) > 0).float()
    cpu = MLPTrainer(spec, device="cpu", seed=7, chunk_rows=1 << 17)
    gpu = MLPTrainer(spec, device="cuda", seed=7, chunk_rows=1 << 17)
    assert gpu.fused_head and gpu.wgrad_ring
    cpu.params.flat.copy_(cpu.params.flat.bfloat16().float())
    gpu.params.flat.copy_(cpu.params.flat.cuda())
    dc, dg = cpu.prepare(x, y), gpu.prepare(x, y)
    # first full-batch gradient, layer by layer (RPROP only uses gradient signs afterwards, so
    # weights of near-zero gradients legitimately drift apart between bf16 and fp32 runs)
    cpu.grad.zero_(); cpu.err_acc.zero_(); cpu.accumulate_gradients(dc)
    gpu.grad.zero_(); gpu.err_acc.zero_(); gpu.accumulate_gradients(dg)
    torch.cuda.synchronize()
    for vc, vg in zip(cpu.params.views(cpu.grad), gpu.params.views(gpu.grad.cpu())):
        r = (vc - vg).norm() / vc.norm().clamp(min=1e-12)
        assert r < 3e-2, float(r)
    ec, eg = [], []
    for _ in range(8):
        ec.append(cpu.step(dc))
        eg.append(gpu.step(dg))
    torch.cuda.synchronize()
    for a, b in zip(ec, eg):
        assert abs(a - b) / a < 1e-2, (ec, eg)


@pytest.mark.parametrize("ring", [1, 0])
def test_pipeline_configuration_tracks_fp32_oracle(ring):
    """The text pipeline's default NN (bench.py --model pipeline: 1603 inputs, one tanh layer of
    50, RPROP) on chunks of 2^17 rows, with the ring forward on and off: first gradient and the
    error trajectory against the fp32 CPU trainer on the same bf16-rounded data."""
    from shifu_amd.ops import _native as nat
    spec = MLPSpec(n_in=1603, hidden=[50], acts=["tanh"], n_out=1)
    n = (1 << 17) + 77
    g = torch.Generator().manual_seed(5)
    x = torch.randn(n, spec.n_in, generator=g).bfloat16().float()
    wt = torch.randn(spec.n_in, 1, generator=g)
    y = ((x @ wt) > 0).float()
    nat.call_hip("shifu_gemm_set_tune", 12, ring)
    try:
        cpu = MLPTrainer(spec, device="cpu", seed=7, chunk_rows=1 << 17)
        gpu = MLPTrainer(spec, device="cuda", seed=7, chunk_rows=1 << 17)
        cpu.params.flat.copy_(cpu.params.flat.bfloat16().float())
        gpu.params.flat.copy_(cpu.params.flat.cuda())
        dc, dg = cpu.prepare(x, y), gpu.prepare(x, y)
        cpu.grad.zero_(); cpu.err_acc.zero_(); cpu.accumulate_gradients(dc)
        gpu.grad.zero_(); gpu.err_acc.zero_(); gpu.accumulate_gradients(dg)
        torch.cuda.synchronize()
        for vc, vg in zip(cpu.params.views(cpu.grad), gpu.params.views(gpu.grad.cpu())):
            r = (vc - vg).norm() / vc.norm().clamp(min=1e-12)
            assert r < 3e-2, float(r)
        ec, eg = [], []
        for _ in range(4):
            ec.append(cpu.step(dc))
            eg.append(gpu.step(dg))
        torch.cuda.synchronize()
    finally:
        nat.call_hip("shifu_gemm_set_tune", 12, 1)
    for a, b in zip(ec, eg):
        assert abs(a - b) / a < 1e-2, (ec, eg)


def test_ring_wgrad_bitwise_reproducible():
    """The ring wgrad reduces split partials in a fixed order: two runs are bit-identical."""
    from shifu_amd.ops import _native as nat
    M, Nv, Kx = 300_000 + 13, 500, 1024
    D = torch.randn(M, 512, device="cuda").bfloat16()
    D[:, Nv:] = 0
    X = torch.randn(M, Kx, device="cuda").bfloat16()
    ws = torch.empty(nat.hip().shifu_wgrad_ring_ws(M, Nv, Kx) // 4, device="cuda")
    outs = []
    for _ in range(2):
        G = torch.zeros(Nv, Kx, device="cuda")
        nat.call_hip("shifu_wgrad_ring", D, 512, X, Kx, G, Kx, M, Nv, Kx, ws, ws.numel() * 4, nat.stream_of(X))
        outs.append(G)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    ref = D[:, :Nv].float().t() @ X.float()
    assert ((outs[0] - ref).abs().max() / ref.abs().max()).item() < 1e-4


def test_two_chunk_lanes_match_one_lane(monkeypatch):
    """Chunks alternating over two HIP streams (own workspaces, second gradient buffer summed at
    the end) give the single-stream gradients and errors (up to float summation order: the output
    layer's gradient and the short tail chunk's wgrad use float atomics in either mode)."""
    spec = MLPSpec(n_in=300, hidden=[256, 90], acts=["sigmoid", "sigmoid"], n_out=1)
    x, y, s = _mk(spec, 5 * 65536 + 77, seed=11)
    grads, errs = {}, {}
    for lanes in ("1", "2", "2"):
        monkeypatch.setenv("SHIFU_CHUNK_LANES", lanes)
        t = MLPTrainer(spec, device="cuda", seed=3, chunk_rows=65536)
        d = t.prepare(x, y, s)
        t.grad.zero_(); t.err_acc.zero_(); t.accumulate_gradients(d)
        torch.cuda.synchronize()
        if lanes in grads:
            assert float((grads[lanes] - t.grad).norm() / t.grad.norm()) < 1e-5
        grads[lanes], errs[lanes] = t.grad.clone(), t.err_acc.clone()
    g1, g2 = grads["1"], grads["2"]
    assert float((g1 - g2).norm() / g1.norm()) < 1e-5
    torch.testing.assert_close(errs["2"], errs["1"], rtol=1e-9, atol=1e-9)


def test_bench_configuration_gradient_bitwise_reproducible():
    """The bench trainer path (ring forward, fused head, ring wgrad, dgrad; full chunks) gives
    bit-identical gradients run to run: the head's output-layer wgrad goes through per-tile
    partials + a fixed-order reduction (colsum_fixed) instead of float atomics."""
    spec = MLPSpec(n_in=1000, hidden=[500, 200], acts=["sigmoid", "sigmoid"], n_out=1)
    n = 2 << 17
    g = torch.Generator().manual_seed(5)
    x = torch.randn(n, spec.n_in, generator=g)
    y = (x[:, :1] > 0).float()
    t = MLPTrainer(spec, device="cuda", seed=7, chunk_rows=1 << 17)
    assert t.fused_head and t.wgrad_ring
    d = t.prepare(x, y)
    grads = []
    for _ in range(2):
        t.grad.zero_(); t.err_acc.zero_(); t.accumulate_gradients(d)
        torch.cuda.synchronize()
        grads.append(t.grad.clone())
    assert torch.equal(grads[0], grads[1])
    assert float(grads[0].abs().sum()) > 0


def test_nn_scoring_bf16_close_to_fp32():
    """shifu.eval.nnPrecision=bf16: scoring on the trainer's MFMA kernels agrees with the fp32
    scoring path to bf16 accuracy (incl. an input-subset net and a swish layer)."""
    import numpy as np
    import torch
    from shifu_amd.formats.nn_format import NNNetwork
    from shifu_amd.scoring.model_runner import nn_forward
    rng = np.random.default_rng(4)
    sizes = [70, 40, 12, 2]
    net = NNNetwork(sizes, ["tanh", "swish", "sigmoid"],
                    [rng.normal(size=(sizes[i + 1], sizes[i] + 1)) * 0.3 for i in range(3)])
    X = rng.normal(size=(20000, 70)).astype(np.float32)
    a = nn_forward(net, X, torch.device("cuda"), precision="fp32")
    b = nn_forward(net, X, torch.device("cuda"), precision="bf16")
    assert a.shape == b.shape == (20000, 2)
    assert np.abs(a - b).max() <= 2e-2




def test_strip_head_falls_back_on_4m_row_chunks():
    """A 4M-row chunk puts the strip head's H1 / DZ1 operands past 32-bit buffer offsets at
    K1 = 512: the trainer takes the 8-phase head + dgrad kernels for that chunk (the launcher used
    to surface as an error) and the gradients match 1M-row chunks (strip head) up to summation
    order."""
    spec = MLPSpec(n_in=60, hidden=[500, 200], acts=["sigmoid", "sigmoid"], n_out=1)
    n = (1 << 22) + 4096
    x, y, s = _mk(spec, n, seed=9)
    big = MLPTrainer(spec, device="cuda", seed=3, chunk_rows=1 << 22)
    small = MLPTrainer(spec, device="cuda", seed=3, chunk_rows=1 << 20)
    assert big.strip_head and small.strip_head
    small.params.flat.copy_(big.params.flat)
    for t in (big, small):
        d = t.prepare(x, y, s)
        t.grad.zero_(); t.err_acc.zero_(); t.accumulate_gradients(d)
    torch.cuda.synchronize()
    for va, vb in zip(big.params.views(big.grad), small.params.views(small.grad)):
        r = (va - vb).norm() / vb.norm().clamp(min=1e-12)
        assert r < 1e-2, float(r)
    assert abs(float(big.err_acc[0]) - float(small.err_acc[0])) / float(small.err_acc[0]) < 1e-4
