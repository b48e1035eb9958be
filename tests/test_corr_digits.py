"""K15 digit-plane arithmetic, emulated in numpy on the CPU: the plane construction of
ops/csrc/corr_kernels.hip (per-column exponent, balanced base-128 digits of u / 2^ex and
u^2 / 2^ey) and the job table of ``corr_job_list`` (plane pairs, scale rows, weights) must
reproduce the fp64 sums of CorrAccumulator(method="fp64") -- so a GPU mismatch can only be the
kernels' indexing, not the scheme."""
import math

import numpy as np
import pytest

from shifu_amd.algos.stats import CorrAccumulator, corr_job_list


def _planes(X, shift, S):
    ok = np.isfinite(X)
    u = np.where(ok, X - shift, 0.0)
    mx = np.abs(u).max(0)
    E = np.array([math.frexp(m)[1] if m > 0 else 0 for m in mx])
    ex = np.where(mx > 0, E + 1, 0)
    ey = np.where(mx > 0, 2 * E + 1, 0)
    planes = [ok.astype(np.int64)]
    for v0, e in ((u, ex), (u * u, ey)):
        v = np.ldexp(v0, -e)
        for _ in range(S):
            t = v * 128.0
            q = np.rint(t)
            v = t - q
            assert np.abs(q).max() <= 64
            planes.append(q.astype(np.int64))
    xs = [planes[0]] + planes[1:1 + S] + planes[1 + S:]
    scale = np.stack([np.ones_like(mx), np.ldexp(1.0, ex), np.ldexp(1.0, ey)])
    return xs, scale


@pytest.mark.parametrize("S", [5, 6, 7])
def test_digit_jobs_reproduce_fp64_sums(S):
    rng = np.random.default_rng(S)
    n, F = 3000, 9
    X = rng.standard_normal((n, F)) * rng.uniform(0.01, 100, F) + rng.uniform(-1e3, 1e3, F)
    X[:, 2] = np.exp(2 * rng.standard_normal(n))
    X[rng.random((n, F)) < 0.05] = np.nan
    shift = np.nanmean(X, 0)
    planes, scale = _planes(X, shift, S)
    out = {}
    for name, pairs, ka, kb, wexp, sym in corr_job_list(S):
        acc = sum(planes[a].T @ planes[b] for a, b in pairs)          # exact int64
        assert np.abs(acc).max() < 2 ** 31 * n / 65536 or n <= 65536
        out[name] = acc.astype(np.float64) * np.ldexp(1.0, -wexp) * scale[ka][:, None] * scale[kb][None, :]
    n_ = out["n"]
    sx = sum(out[f"sx{s}"] for s in range(S))
    sxx = sum(out[f"sxx{s}"] for s in range(S))
    sxy = sum(out[f"sxy{d}"] for d in range(S))
    ref = CorrAccumulator(F, "cpu", shift=shift, method="fp64")
    ref.update(X)
    r = ref.raw_sums().numpy()
    assert np.array_equal(n_, r[0])
    tol = 2.0 ** (-7 * S) * 64 * n
    for got, want, k in ((sx, r[1], 1), (sxx, r[2], 2), (sxy, r[3], 3)):
        mx = np.abs(np.where(np.isfinite(X), X - shift, 0)).max(0)
        bound = tol * (mx[:, None] ** (2 if k == 2 else 1)) * (mx[None, :] if k == 3 else 1.0) + 1e-9 * np.abs(want)
        assert np.all(np.abs(got - want) <= bound), k
