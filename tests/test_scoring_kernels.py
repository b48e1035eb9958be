"""K13 tree-ensemble inference and K17/K18 keyed counts (``scoring_kernels.hip``) against the
fp64 torch / numpy oracles on the CPU."""
import numpy as np
import pytest
import torch

from shifu_amd.formats.tree_format import CATEGORICAL, CONTINUOUS, Node, Split, TreeModelFile, TreeRecord
from shifu_amd.scoring.tree_ensemble import TreeScorer

N_NUM, CATS = 12, {12: 7, 13: 40, 14: 3}      # numeric columns 0..11, categorical 12..14


def _random_model(n_trees=60, max_depth=7, algorithm="GBT", seed=0):
    rng = np.random.default_rng(seed)
    nid = [0]

    def grow(d):
        nid[0] += 1
        nd = Node(nid[0])
        if d == max_depth or (d > 1 and rng.random() < 0.2):
            nd.predict = float(rng.normal())
            return nd
        col = int(rng.integers(0, N_NUM + len(CATS)))
        if col < N_NUM:
            nd.split = Split(col, CONTINUOUS, threshold=float(rng.normal()))
        else:
            k = CATS[col]
            sub = {int(c) for c in rng.choice(k, size=int(rng.integers(1, k + 1)), replace=False)}
            nd.split = Split(col, CATEGORICAL, is_left=bool(rng.random() < 0.5), categories=sub)
        nd.left, nd.right = grow(d + 1), grow(d + 1)
        return nd

    bags = [[TreeRecord(t, 0, grow(0), float(rng.uniform(0.05, 0.3))) for t in range(n_trees)]]
    cols = list(range(N_NUM + len(CATS)))
    return TreeModelFile(algorithm, "squared", False, False, len(cols), {c: 0.0 for c in cols},
                         {c: f"c{c}" for c in cols}, {c: [f"v{j}" for j in range(k)] for c, k in CATS.items()},
                         {c: i for i, c in enumerate(cols)}, bags)


def _inputs(n, seed=1):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, N_NUM + len(CATS)))
    for j, (c, k) in enumerate(CATS.items()):
        X[:, N_NUM + j] = rng.integers(-1, k + 2, size=n)          # incl. unseen (k) and invalid codes
    X[rng.random(size=X.shape) < 0.01] = 0.0
    return torch.from_numpy(X)


def test_flat_ensemble_matches_record_walk():
    """The CPU torch path (the oracle of the HIP kernel) equals the per-row record walk
    (IndependentTreeModel semantics in TreeModelFile.score)."""
    m = _random_model(n_trees=8)
    X = _inputs(300)
    x = {c: X[:, i].numpy() for i, c in enumerate(sorted(m.names))}
    ref = m.score(x, 300)
    got = TreeScorer(m, device="cpu").score_bags(X)[:, 0]
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("coded", [True, False])
@pytest.mark.parametrize("algorithm,n,trees", [("GBT", 70_001, 60), ("RF", 5_000, 3), ("GBT", 257, 500)])
def test_tree_infer_kernel_matches_torch(algorithm, n, trees, coded, monkeypatch):
    from shifu_amd.ops import _native
    from shifu_amd.scoring import tree_ensemble
    _native.require_gpu_native()
    monkeypatch.setattr(tree_ensemble, "CODED_WALK", coded)
    m = _random_model(n_trees=trees, algorithm=algorithm, seed=n)
    X = _inputs(n, seed=trees)
    cpu, gpu = TreeScorer(m, device="cpu"), TreeScorer(m, device="cuda")
    Xd = X.cuda()
    np.testing.assert_array_equal(gpu.ens[0].leaves(Xd).cpu().numpy(), cpu.ens[0].leaves(X).numpy())
    np.testing.assert_allclose(gpu.score_bags(Xd), cpu.score_bags(X), rtol=1e-12, atol=1e-12)


@pytest.mark.gpu
def test_coded_walk_wide_inputs():
    """1000 numeric inputs (16 rows per block in LDS, 16 threads per row), NaN / +-inf inputs and
    thresholds shared by several nodes: the coded walk equals the fp64 torch walk."""
    from shifu_amd.formats.tree_format import CONTINUOUS, Node, Split, TreeModelFile, TreeRecord
    rng = np.random.default_rng(11)
    C = 1000
    shared = rng.normal(size=50)

    def grow(d):
        nd = Node(0)
        if d == 6:
            nd.predict = float(rng.normal())
            return nd
        nd.split = Split(int(rng.integers(0, C)), CONTINUOUS, threshold=float(rng.choice(shared)))
        nd.left, nd.right = grow(d + 1), grow(d + 1)
        return nd
    cols = list(range(C))
    m = TreeModelFile("GBT", "squared", False, False, C, {c: 0.0 for c in cols}, {c: f"c{c}" for c in cols}, {},
                      {c: c for c in cols}, [[TreeRecord(t, 0, grow(0), 0.1) for t in range(40)]])
    X = torch.from_numpy(rng.choice(np.concatenate([shared, rng.normal(size=50), [np.nan, np.inf, -np.inf]]),
                                    size=(3001, C)))
    cpu, gpu = TreeScorer(m, device="cpu"), TreeScorer(m, device="cuda")
    np.testing.assert_array_equal(gpu.ens[0].leaves(X.cuda()).cpu().numpy(), cpu.ens[0].leaves(X).numpy())
    np.testing.assert_allclose(gpu.score_bags(X.cuda()), cpu.score_bags(X), rtol=1e-12, atol=1e-12)


@pytest.mark.gpu
def test_keyed_hist_matches_bincount():
    from shifu_amd.ops.stats_ops import keyed_hist
    rng = np.random.default_rng(3)
    n = 300_007
    for K in (11, 5000):                       # LDS-private and global-atomic paths
        keys = rng.integers(-2, K + 3, size=(5, n))
        w = rng.normal(size=n) * 100.0
        cnt, ws = keyed_hist(torch.from_numpy(keys).cuda(), K, torch.from_numpy(w).cuda())
        for f in range(5):
            ok = (keys[f] >= 0) & (keys[f] < K)
            np.testing.assert_array_equal(cnt[f].cpu().numpy(), np.bincount(keys[f][ok], minlength=K))
            np.testing.assert_allclose(ws[f].cpu().numpy(), np.bincount(keys[f][ok], weights=w[ok], minlength=K),
                                       rtol=1e-9, atol=1e-6)
        # deterministic: fixed-point sums are order-independent
        cnt2, ws2 = keyed_hist(torch.from_numpy(keys).cuda(), K, torch.from_numpy(w).cuda())
        assert torch.equal(ws, ws2) and torch.equal(cnt, cnt2)
    # 1-D keys with 1-D weights -> one row
    k1 = torch.from_numpy(rng.integers(0, 9, size=n)).cuda()
    c1, w1 = keyed_hist(k1, 9, torch.ones(n, dtype=torch.float64, device="cuda"))
    assert c1.shape == (1, 9) and torch.equal(c1, w1)
