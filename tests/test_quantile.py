"""K4 exact quantile engine (algos/quantile.py): cuts equal binning.equal_population_boundaries /
equal_interval_boundaries (the host oracle, reference EqualPopulationBinning semantics) on
adversarial columns -- ties, NaN, +-inf, -0.0, constants, outliers that put most values in one
bucket, low-cardinality columns -- for every binning method, in one batch, in streamed row chunks,
and on the HIP kernels (gpu marker: bounds identical to the oracle, pass state identical to the
torch implementation)."""
import numpy as np
import pytest
import torch

from shifu_amd.algos import quantile as Q
from shifu_amd.algos.stats import _numeric_bounds, exact_distinct

METHODS = ("EqualPositive", "EqualNegtive", "EqualTotal", "WeightEqualPositive", "WeightEqualTotal",
           "EqualInterval")


def _columns(n, rng):
    cols = [rng.normal(size=n), rng.integers(0, 5, size=n).astype(float)]
    x = rng.integers(0, 7, size=n).astype(float)
    x[:3] = 1e12                                   # outliers: the bulk lands in one bucket
    cols.append(x)
    cols.append(np.exp(rng.normal(size=n) * 3))    # heavy tail
    x = rng.normal(size=n)
    x[rng.random(n) < 0.3] = np.nan
    x[:2] = np.inf
    x[2:4] = -np.inf
    cols.append(x)
    cols.append(np.round(rng.normal(size=n), 2))   # many ties
    cols.append(np.full(n, 3.0))
    cols.append(np.full(n, np.nan))
    x = rng.normal(size=n)
    x[x < 0] = 0.0
    x[:5] = -0.0
    cols.append(x)
    x = rng.integers(0, 12, size=n).astype(float) + (rng.random(n) < 0.01) * 1e-13   # near-ties
    cols.append(x)
    cols.append(1e300 * rng.normal(size=n))        # range overflows float64
    return np.stack(cols)


def _check(V, y, w, dev, nbins, chunk=None):
    n = V.shape[1]
    for method in METHODS:
        if chunk is None:
            b, _ = Q.column_cuts(torch.from_numpy(V.copy()).to(dev), torch.from_numpy(y).to(dev),
                                 torch.from_numpy(w).to(dev), nbins, method, True)
        else:
            sm = Q.sel_mode_for(method, True)
            eng = Q.QuantileEngine(V.shape[0], nbins, sm, method.startswith("Weight"), method == "EqualInterval",
                                   device=dev)
            chunks = [(torch.from_numpy(V[:, a:a + chunk].copy()).to(dev), torch.from_numpy(y[a:a + chunk]).to(dev),
                       torch.from_numpy(w[a:a + chunk]).to(dev)) for a in range(0, n, chunk)]
            Q.run_passes(eng, chunks)
            b, _ = eng.finish()
        for c in range(V.shape[0]):
            ref = _numeric_bounds(V[c].copy(), y, w, True, method, nbins)
            if chunk is not None and len(ref) <= 1:
                continue                           # the all-rows fallback is column_cuts' job
            assert b[c] == ref, (method, nbins, c, ref[:4], b[c][:4])


@pytest.mark.parametrize("n,nbins", [(60, 10), (3000, 10), (3000, 4), (20000, 64)])
def test_cuts_equal_host_oracle_cpu(n, nbins):
    rng = np.random.default_rng(n + nbins)
    V = _columns(n, rng)
    y = (rng.random(n) < 0.3).astype(np.float32)
    w = rng.integers(1, 5, size=n).astype(float)
    _check(V, y, w, "cpu", nbins)


def test_streamed_chunks_equal_oracle_cpu():
    rng = np.random.default_rng(7)
    n = 9000
    V = _columns(n, rng)
    y = (rng.random(n) < 0.4).astype(np.float32)
    w = rng.random(n) * 3                           # fractional weights (fixed point)
    _check(V, y, w, "cpu", 10, chunk=2500)


def test_distinct_counts_cpu():
    rng = np.random.default_rng(3)
    n = 20000
    V = _columns(n, rng)
    y = (rng.random(n) < 0.5).astype(np.float32)
    w = np.ones(n)
    _, d = Q.column_cuts(torch.from_numpy(V.copy()), torch.from_numpy(y), torch.from_numpy(w), 10, "EqualTotal", True)
    ex = exact_distinct(torch.from_numpy(V.copy()), 1.7976931348623157e308)
    for c in range(V.shape[0]):
        fin = V[c][np.isfinite(V[c])]
        u = np.unique(fin).size
        assert ex[c] == u
        assert abs(d[c] - u) <= max(2, 0.03 * u), (c, u, d[c])   # HLL p=14: ~0.8 % rel. error


@pytest.mark.gpu
@pytest.mark.parametrize("n,nbins", [(3000, 10), (200003, 10), (200003, 33)])
def test_cuts_equal_host_oracle_gpu(n, nbins):
    rng = np.random.default_rng(n + nbins)
    V = _columns(n, rng)
    y = (rng.random(n) < 0.3).astype(np.float32)
    w = rng.integers(1, 5, size=n).astype(float)
    _check(V, y, w, "cuda", nbins)
    _check(V, y, w, "cuda", nbins, chunk=50000)


@pytest.mark.gpu
def test_kernel_state_equals_torch_passes():
    """qprep/qhist/qgather state (keys, counts, weights, HLL registers) == the torch passes."""
    rng = np.random.default_rng(11)
    n = 100000
    V = _columns(n, rng)
    y = (rng.random(n) < 0.3).astype(np.float32)
    w = rng.random(n) * 2
    engs = {}
    for dev in ("cpu", "cuda"):
        e = Q.QuantileEngine(V.shape[0], 10, 1, True, False, device=dev)
        ch = [(torch.from_numpy(V.copy()).to(dev), torch.from_numpy(y).to(dev), torch.from_numpy(w).to(dev))]
        Q.run_passes(e, ch)
        engs[dev] = e
    a, b = engs["cpu"], engs["cuda"]
    assert torch.equal(a.mm, b.mm.cpu())
    assert torch.equal(a.scnt, b.scnt.cpu())
    assert torch.equal(a.hll, b.hll.cpu())
    for k in ("cnt", "wq", "kmn", "kmx", "akmn", "akmx"):
        assert torch.equal(getattr(a, k), getattr(b, k).cpu()), k
    assert a.slots == b.slots
    ga = a.gv[: int(a.local_lens.sum())].cpu().sort().values
    gb = b.gv[: int(b.local_lens.sum())].cpu().sort().values
    assert torch.equal(ga, gb)
    assert a.finish() == b.finish()


@pytest.mark.parametrize("cap,budget", [(4, 1 << 30), (64, 1 << 30), (1 << 20, 50)])
def test_refinement_levels_equal_oracle_cpu(monkeypatch, cap, budget):
    """A tiny per-bucket gather cap (or a tiny per-batch gather budget) forces the multi-valued
    target buckets through windowed refinement (and AMBIG columns through the outside-value
    bookkeeping) -- cuts stay exact."""
    monkeypatch.setattr(Q, "GATHER_CAP", cap)
    monkeypatch.setattr(Q, "GATHER_BUDGET", budget)
    rng = np.random.default_rng(cap)
    n = 4000
    V = _columns(n, rng)
    y = (rng.random(n) < 0.3).astype(np.float32)
    w = rng.integers(1, 5, size=n).astype(float)
    _check(V, y, w, "cpu", 10)
    _check(V, y, w, "cpu", 10, chunk=1500)


@pytest.mark.gpu
def test_refinement_levels_equal_oracle_gpu(monkeypatch):
    monkeypatch.setattr(Q, "GATHER_CAP", 64)
    rng = np.random.default_rng(5)
    n = 50000
    V = _columns(n, rng)
    y = (rng.random(n) < 0.3).astype(np.float32)
    w = rng.integers(1, 5, size=n).astype(float)
    _check(V, y, w, "cuda", 10)
    _check(V, y, w, "cuda", 10, chunk=20000)


def test_pack_bits_matches_numpy():
    from shifu_amd.ops.stats_ops import pack_bits
    rng = np.random.default_rng(0)
    for n in (1, 31, 32, 33, 1000):
        m = rng.random(n) < 0.4
        words = pack_bits(torch.from_numpy(m)).numpy().view(np.uint32)
        ref = np.packbits(np.concatenate([m, np.zeros((-n) % 32, bool)]), bitorder="little").view("<u4")
        assert np.array_equal(words, ref)


@pytest.mark.gpu
def test_pack_sel_kernel_matches_cpu():
    from shifu_amd.ops.stats_ops import pack_sel
    rng = np.random.default_rng(1)
    for n in (1, 31, 63, 64, 65, 1000, 100003):
        y = torch.from_numpy((rng.random(n) < 0.4).astype(np.float32))
        for mode in (1, 2):
            a = pack_sel(y, mode).numpy()
            b = pack_sel(y.cuda(), mode).cpu().numpy()[: a.size]
            assert np.array_equal(a, b), (n, mode)


@pytest.mark.gpu
def test_stats_lanes_equal_sequential():
    """Column batches run two at a time on separate HIP streams (algos/stats.run_lanes, host
    threads) give exactly the sequential cuts, distinct counts and bin histograms."""
    from shifu_amd.algos.stats import batch_histograms, run_lanes
    rng = np.random.default_rng(5)
    n = 150_001
    dev = torch.device("cuda")
    batches = [torch.as_tensor(_columns(n, rng), device=dev) for _ in range(3)]
    y = torch.as_tensor((rng.random(n) < 0.3).astype(np.float32), device=dev)
    w = torch.as_tensor(rng.integers(1, 5, size=n).astype(float), device=dev)

    def fn(v):
        bounds, distinct = Q.column_cuts(v, y, w, 10, "EqualPositive", True)
        return bounds, distinct, batch_histograms(v, y, w, bounds, True)

    seq = run_lanes(fn, batches, dev, lanes=1)
    par = run_lanes(fn, batches, dev, lanes=2)
    for (b1, d1, h1), (b2, d2, h2) in zip(seq, par):
        assert [list(b) for b in b1] == [list(b) for b in b2]
        assert list(d1) == list(d2)
        for r1, r2 in zip(h1, h2):
            for a1, a2 in zip(r1, r2):
                np.testing.assert_array_equal(np.asarray(a1), np.asarray(a2))
