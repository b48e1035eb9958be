"""WDL training against a numpy port of the reference's per-row WideAndDeep.forward / backward
(J/core/dtrain/wdl/WideAndDeep.java:163-232 and the layers' backward: DenseLayer.java:188-205,
WideFieldLayer.java:97-109, WideDenseLayer.java:96-104, EmbedFieldLayer.java:107-117, the
activations) plus the master's GradientDescent.update on the summed gradients
(WDLMaster.java:159-186, GradientDescent.java:44-63); the world-4 gloo run equals one process;
the CPU row stream keeps host memory bounded."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

SIZES, EMB, D = [4, 6, 3], [0, 2], 3
HIDDEN, ACTS = [5, 4], ["sigmoid", "tanh"]
ND = 3


def _data(n, seed=0):
    g = np.random.default_rng(seed)
    dense = g.normal(size=(n, ND)).astype(np.float32)
    cats = np.stack([g.integers(0, s + 1, n) for s in SIZES], 1)           # s = missing category
    y = ((dense[:, 0] + (cats[:, 1] % 2) - 0.5 + 0.3 * g.normal(size=n)) > 0).astype(np.float32)
    w = (g.random(n) + 0.5).astype(np.float32)
    return dense, cats, y, w


def _net(seed=3):
    from shifu_amd.models.wdl import WideDeepNet
    torch.manual_seed(seed)
    net = WideDeepNet(ND, SIZES, EMB, D, HIDDEN, ACTS)
    with torch.no_grad():
        for t in net.wide_tables:
            t.normal_(0, 0.1)
        net.wide_dense.normal_(0, 0.1)
        net.bias.fill_(0.05)
    return net


class RefWDL:
    """numpy (float64) port of the reference's per-row math; weights as the Java objects hold them
    (DenseLayer weights [in][out] + bias[out])."""

    def __init__(self, net):
        c = lambda t: t.detach().double().numpy().copy()   # noqa: E731
        self.wt = [c(t) for t in net.wide_tables]
        self.wd = c(net.wide_dense)
        self.b = float(net.bias.detach()[0])
        self.emb = [c(e) for e in net.embeds]
        self.W = [c(L[:, :-1]).T.copy() for L in net.layers]
        self.bW = [c(L[:, -1]) for L in net.layers]
        self.F = c(net.final[:, :-1]).T.copy()
        self.bF = c(net.final[:, -1])

    @staticmethod
    def act(name, z):
        return 1 / (1 + np.exp(-z)) if name == "sigmoid" else np.tanh(z)

    @staticmethod
    def dact(name, out):                     # Activation.backward from the forward output
        return out * (1 - out) if name == "sigmoid" else 1 - out * out

    def epoch(self, dense, cats, y, sig, lr, l2):
        g_wt = [np.zeros_like(t) for t in self.wt]
        g_wd, g_b = np.zeros_like(self.wd), 0.0
        g_emb = [np.zeros_like(e) for e in self.emb]
        g_W = [np.zeros_like(W) for W in self.W]
        g_bW = [np.zeros_like(b) for b in self.bW]
        g_F, g_bF = np.zeros_like(self.F), np.zeros_like(self.bF)
        err = 0.0
        for r in range(len(y)):
            x, ci = dense[r].astype(np.float64), cats[r]
            wide = sum(t[ci[f]] for f, t in enumerate(self.wt)) + x @ self.wd + self.b
            inp = np.concatenate([x] + [self.emb[k][ci[f]] for k, f in enumerate(EMB)])
            ins, outs = [], []
            a = inp
            for W, b, nm in zip(self.W, self.bW, ACTS):
                ins.append(a)
                a = self.act(nm, a @ W + b)
                outs.append(a)
            deep = float(a @ self.F[:, 0] + self.bF[0])
            p = 1 / (1 + np.exp(-(wide + deep)))
            err += sig[r] * (p - y[r]) ** 2
            g = (p - y[r]) * p * (1 - p) * sig[r]              # WideAndDeep.backward
            for f, t in enumerate(self.wt):                     # WideFieldLayer: value 1 + per-row L2
                g_wt[f][ci[f]] += g + l2 * t[ci[f]]
            g_wd += x * g + l2 * self.wd                        # WideDenseLayer
            g_b += g                                            # BiasLayer (summed: see WDLTrainer doc)
            g_F[:, 0] += a * g + l2 * self.F[:, 0]              # final DenseLayer
            g_bF += g
            back = self.F[:, 0] * g
            for l in range(len(self.W) - 1, -1, -1):
                back = back * self.dact(ACTS[l], outs[l])       # activation backward
                g_W[l] += np.outer(ins[l], back) + l2 * self.W[l]
                g_bW[l] += back
                back = self.W[l] @ back
            for k, f in enumerate(EMB):                         # EmbedFieldLayer: no L2
                g_emb[k][ci[f]] += back[ND + k * D: ND + (k + 1) * D]
        # GradientDescent.update on the summed gradients: w -= lr * g
        for t, gt in zip(self.wt, g_wt):
            t -= lr * gt
        self.wd -= lr * g_wd
        self.b -= lr * g_b
        for e, ge in zip(self.emb, g_emb):
            e -= lr * ge
        for W, gw, b, gb in zip(self.W, g_W, self.bW, g_bW):
            W -= lr * gw
            b -= lr * gb
        self.F -= lr * g_F
        self.bF -= lr * g_bF
        return err / len(y)

    def compare(self, net, rtol=2e-4, atol=2e-6):
        c = lambda t: t.detach().double().cpu().numpy()   # noqa: E731
        for t, q in zip(self.wt, net.wide_tables):
            np.testing.assert_allclose(c(q), t, rtol=rtol, atol=atol)
        np.testing.assert_allclose(c(net.wide_dense), self.wd, rtol=rtol, atol=atol)
        np.testing.assert_allclose(float(net.bias.detach()[0]), self.b, rtol=rtol, atol=atol)
        for e, q in zip(self.emb, net.embeds):
            np.testing.assert_allclose(c(q), e, rtol=rtol, atol=atol)
        for W, b, L in zip(self.W, self.bW, net.layers):
            np.testing.assert_allclose(c(L[:, :-1]).T, W, rtol=rtol, atol=atol)
            np.testing.assert_allclose(c(L[:, -1]), b, rtol=rtol, atol=atol)
        np.testing.assert_allclose(c(net.final[:, :-1]).T, self.F, rtol=rtol, atol=atol)
        np.testing.assert_allclose(c(net.final[:, -1]), self.bF, rtol=rtol, atol=atol)


def _rows(dense, cats, device="cpu", chunk=64):
    from shifu_amd.models.wdl import WDLRows
    X = np.concatenate([dense, cats.astype(np.float32)], 1)
    return WDLRows(X, list(range(ND)), list(range(ND, ND + len(SIZES))), device, chunk_rows=chunk)


@pytest.mark.parametrize("l2", [0.0, 1e-3])
def test_wdl_trainer_equals_reference_port(l2):
    from shifu_amd.models.wdl import WDLTrainer
    dense, cats, y, w = _data(240)
    net = _net()
    ref = RefWDL(net)
    tr = WDLTrainer(net, "cpu", lr=0.02, l2=l2)
    rows = _rows(dense, cats)
    s_va = np.zeros_like(w)
    for ep in range(3):
        e_ref = ref.epoch(dense, cats, y, w, 0.02, l2)
        terr, verr = tr.epoch(rows, y, w, s_va, float(len(y)), 0.0)
        assert abs(terr - e_ref) < 1e-5 * max(1.0, e_ref), (ep, terr, e_ref)
        assert np.isnan(verr)
        ref.compare(tr.net)


def test_wdl_validation_split_and_bagging_weights():
    """Validation rows take no part in the gradient; their error uses the epoch's weights."""
    from shifu_amd.models.wdl import WDLTrainer
    dense, cats, y, w = _data(300, seed=4)
    valid = np.arange(300) % 5 == 0
    net = _net(5)
    ref = RefWDL(net)
    tr = WDLTrainer(net, "cpu", lr=0.01, l2=0.0)
    s_tr = np.where(valid, 0.0, w).astype(np.float32)
    s_va = np.where(valid, w, 0.0).astype(np.float32)
    for _ in range(3):
        ref_v = RefWDL.__new__(RefWDL)
        ref_v.__dict__ = {k: (v.copy() if isinstance(v, np.ndarray) else ([a.copy() for a in v] if isinstance(v, list) else v))
                          for k, v in ref.__dict__.items()}
        ev = ref_v.epoch(dense[valid], cats[valid], y[valid], w[valid], 0.0, 0.0) * valid.sum()
        et = ref.epoch(dense[~valid], cats[~valid], y[~valid], w[~valid], 0.01, 0.0)
        terr, verr = tr.epoch(_rows(dense, cats), y, s_tr, s_va, float((~valid).sum()), float(valid.sum()))
        assert abs(terr - et) < 1e-5 and abs(verr - ev / valid.sum()) < 1e-5
    ref.compare(tr.net)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_train(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), SHIFU_FORCE_CPU="1")
    from shifu_amd.models.wdl import WDLTrainer
    from shifu_amd.parallel import dist
    dist.init_from_env()
    dense, cats, y, w = _data(1000, seed=7)
    lo, hi = 1000 * rank // world, 1000 * (rank + 1) // world
    tr = WDLTrainer(_net(9), "cpu", lr=0.002, l2=1e-4)
    hist = [tr.epoch(_rows(dense[lo:hi], cats[lo:hi]), y[lo:hi], w[lo:hi], np.zeros(hi - lo, np.float32),
                     float(hi - lo), 0.0)[0] for _ in range(4)]
    if rank == 0:
        np.save(out, np.concatenate([tr.flat.numpy(), hist]))
    dist.shutdown()


def test_wdl_world4_equals_one_process(tmp_path):
    outs = {}
    for world in (1, 4):
        out = str(tmp_path / f"w{world}.npy")
        mp.start_processes(_rank_train, args=(world, _port(), out), nprocs=world, join=True, start_method="spawn")
        outs[world] = np.load(out)
    np.testing.assert_allclose(outs[4], outs[1], rtol=1e-5, atol=1e-7)


_RSS = r"""
import numpy as np, os, sys, json
sys.path.insert(0, {repo!r})
def anon():
    for l in open("/proc/self/status"):
        if l.startswith("RssAnon:"):
            return int(l.split()[1])
X = np.load({path!r}, mmap_mode="r")
n = X.shape[0]
y = (np.asarray(X[:, 0]) > 0).astype(np.float32)
w = np.ones(n, np.float32)
s_va = np.zeros(n, np.float32)
import torch
from shifu_amd.models.wdl import WDLRows, WDLTrainer, WideDeepNet
net = WideDeepNet(12, [9, 9, 9, 9], [0, 1], 4, [8], ["relu"])
base = anon()
rows = WDLRows(X, list(range(12)), list(range(12, 16)), "cpu", chunk_rows=1 << 16)
tr = WDLTrainer(net, "cpu", lr=1e-6)
for _ in range(2):
    tr.epoch(rows, y, w, s_va, float(n), 0.0)
print(json.dumps({{"growth_kb": anon() - base, "data_kb": X.nbytes // 1024}}))
"""


def test_wdl_cpu_stream_host_memory_bounded(tmp_path):
    """The rows stream from the memmap in chunks: anonymous memory grows by far less than the
    table (the previous trainer loaded the whole raw table into host memory and HBM)."""
    import json
    import subprocess
    import sys
    n = 3_000_000
    path = str(tmp_path / "x.npy")
    X = np.lib.format.open_memmap(path, mode="w+", dtype=np.float32, shape=(n, 16))
    g = np.random.default_rng(0)
    for a in range(0, n, 500_000):
        b = min(n, a + 500_000)
        X[a:b, :12] = g.normal(size=(b - a, 12))
        X[a:b, 12:] = g.integers(0, 10, (b - a, 4))
    X.flush()
    del X
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _RSS.format(repo=repo, path=path)], capture_output=True, text=True,
                       timeout=600, env=dict(os.environ, SHIFU_FORCE_CPU="1", OMP_NUM_THREADS="4"))
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["data_kb"] > 180_000
    assert out["growth_kb"] < 0.35 * out["data_kb"], out
