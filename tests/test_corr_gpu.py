"""K15 correlation sums on the int8 MFMA (ops/csrc/corr_kernels.hip digit planes +
gemm_kernels.hip corr_i8_kernel) against the fp64 torch oracle (the same CorrAccumulator with
method="fp64": four fp64 addmm per chunk on the CPU).

The data exercise every exactness hazard: chunks that straddle the 64K-row GEMM chunk, F not a
multiple of the 256 tile (symmetric upper-tile mirroring), missing and +inf cells, a constant
column, an all-missing column, a tiny-variance column on a large mean (shift), a heavy-tailed
(lognormal) column whose chunk maximum is far above its typical value, an integer-valued column."""
import numpy as np
import pytest
import torch

from shifu_amd.algos.stats import CorrAccumulator, pearson_correlation

pytestmark = pytest.mark.gpu


def _data(n, F, seed):
    rng = np.random.default_rng(seed)
    z = rng.standard_normal((n, F + 1))
    x = z[:, 1:] + 0.6 * z[:, :-1]
    x[:, 3] = x[:, 3] * 1e-3 + 1e4
    x[:, 5] = np.exp(2.0 * rng.standard_normal(n))
    x[:, 7] = 2.5
    x[:, 9] = np.nan
    x[:, 11] = np.round(x[:, 11] * 3.0)
    x[rng.random((n, F)) < 0.05] = np.nan
    x[rng.random((n, F)) < 0.001] = np.inf
    return x


def _shift(X):
    fin = np.isfinite(X)
    cnt = fin.sum(0)
    return np.where(cnt > 0, np.where(fin, X, 0.0).sum(0) / np.maximum(cnt, 1), 0.0)


def _run(X, shift, method, slices=None, step=70_000):
    F = X.shape[1]
    acc = CorrAccumulator(F, "cuda" if method == "i8" else "cpu", shift=shift, method=method, slices=slices)
    for r0 in range(0, len(X), step):
        acc.update(X[r0:r0 + step])
    sums = acc.raw_sums().cpu().clone()
    return sums, acc.finalize(0)


@pytest.mark.parametrize("F", [300, 40])
def test_corr_i8_matches_fp64_oracle(F):
    n = 150_000
    X = _data(n, F, F)
    shift = _shift(X)
    s8, c8 = _run(X, shift, "i8")
    s64, c64 = _run(X, shift, "fp64")
    # pair counts are exact integers
    assert torch.equal(s8[0], s64[0])
    # every sum within 1e-12 of its worst-case magnitude (n * max|u_i|^a * max|u_j|^b): the digit
    # truncation (2^-43 of a column's chunk maximum per value) is random, so it stays far below
    fin = np.isfinite(X)
    mx = torch.from_numpy(np.where(fin, np.abs(np.where(fin, X, 0.0) - shift), 0.0).max(0))
    for k, sc in ((1, mx[:, None] * torch.ones(F)[None, :]), (2, (mx ** 2)[:, None] * torch.ones(F)[None, :]),
                  (3, mx[:, None] * mx[None, :])):
        assert ((s8[k] - s64[k]).abs() <= 1e-12 * n * sc + 1e-12).all(), k
    d = np.abs(c8 - c64)
    assert np.nanmax(d) <= 1e-9, float(np.nanmax(d))
    big = np.abs(c64) > 0.01
    assert np.max(d[big] / np.abs(c64[big])) <= 1e-9
    # structure: unit diagonal (where defined), symmetric, all-missing / constant columns read 0
    assert np.allclose(c8, c8.T, atol=1e-12)
    assert np.all(c8[9, np.arange(F) != 9] == 0.0)
    assert np.all(c8[7, np.arange(F) != 7] == 0.0)


def test_corr_i8_fewer_digits_degrade_gracefully():
    X = _data(70_000, 64, 3)
    shift = _shift(X)
    _, c4 = _run(X, shift, "i8", slices=4)
    _, c64 = _run(X, shift, "fp64")
    assert np.nanmax(np.abs(c4 - c64)) <= 1e-6


def test_pearson_correlation_gpu_default_is_i8_and_centres():
    X = _data(20_000, 33, 5)
    X[:, 0] += 1e6                                   # no explicit shift: first-chunk means are used
    c = pearson_correlation(X, device="cuda")
    _, ref = _run(X, _shift(X), "fp64")
    assert np.nanmax(np.abs(c - ref)) <= 1e-9
