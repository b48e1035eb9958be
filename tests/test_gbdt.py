"""GBT/RF engine: CPU oracle semantics + HIP kernels vs the CPU oracle."""
import numpy as np
import pytest
import torch

from shifu_amd.models.gbdt import (BinnedData, Tree, TreeConfig, TreeTrainer, _gain_py,
                                   _strategy_count)


def _data(n=600, f=6, nb=12, seed=0, device="cpu", cat_cols=()):
    rng = np.random.default_rng(seed)
    codes = rng.integers(0, nb, size=(n, f))
    y = ((codes[:, 0] > nb // 2) ^ (codes[:, 1] < 3)).astype(np.float32)
    y = np.where(rng.random(n) < 0.05, 1 - y, y)
    nbins = np.full(f, nb)
    is_cat = np.zeros(f, np.uint8)
    for c in cat_cols:
        is_cat[c] = 1
    return BinnedData.from_codes(codes, y, nbins, is_cat, device=device), codes, y


def _best_split_bruteforce(codes, g, w, nb, min_inst, imp=0):
    best = (-1.0, None, None)
    for f in range(codes.shape[1]):
        for b in range(nb - 1):
            left = codes[:, f] <= b
            lw, rw = w[left].sum(), w[~left].sum()
            if lw <= min_inst or rw <= min_inst:
                continue
            ls, rs = (w * g)[left].sum(), (w * g)[~left].sum()
            gain = _gain_py(imp, lw, ls, rw, rs)
            if gain > best[0] + 1e-12:
                best = (gain, f, b)
    return best


@pytest.mark.parametrize("imp", ["variance", "friedmanmse", "entropy", "gini"])
def test_root_split_matches_bruteforce(imp):
    data, codes, y = _data()
    tr = TreeTrainer(TreeConfig("GBT", tree_num=1, max_depth=2, impurity=imp, feature_subset_strategy="ALL",
                                min_instances_per_node=5), data)
    tr.train()
    t = tr.trees[0]
    gain, f, b = _best_split_bruteforce(codes, y, np.ones(len(y)), 12, 5, {"variance": 0, "friedmanmse": 1,
                                                                           "entropy": 2, "gini": 3}[imp])
    assert t.feat[1] == f and t.thr[1] == b
    assert abs(t.gain[1] - gain) < 1e-4 * max(1, abs(gain))
    # leaf values are weighted means of the children
    left = codes[:, f] <= b
    assert abs(t.value[2] - y[left].mean()) < 1e-5
    assert abs(t.value[3] - y[~left].mean()) < 1e-5


def test_gbt_reduces_error_and_predict_consistent():
    data, codes, y = _data(n=2000, f=8)
    tr = TreeTrainer(TreeConfig("GBT", tree_num=8, max_depth=4, learning_rate=0.3,
                                feature_subset_strategy="ALL"), data)
    tr.train()
    assert tr.train_errors[-1] < tr.train_errors[0]
    p = tr.predict(data)
    assert torch.allclose(p, tr.pred, atol=1e-5)
    # tree partition consistency: host traversal of every tree reproduces predictions
    acc = np.zeros(len(y), np.float32)
    for i, t in enumerate(tr.trees):
        v = t.predict_bins(data.codes().numpy(), data.is_cat)
        acc = v if i == 0 else acc + t.weight * v
    assert np.allclose(acc, p.numpy(), atol=1e-5)


def test_rf_bagging_and_average():
    data, codes, y = _data(n=1500, f=6)
    tr = TreeTrainer(TreeConfig("RF", tree_num=5, max_depth=4, impurity="gini", sample_with_replacement=True,
                                feature_subset_strategy="HALF", seed=3), data)
    tr.train()
    p = tr.predict(data).numpy()
    assert ((p > 0.5) == (y > 0.5)).mean() > 0.8


def test_categorical_split_orders_by_mean():
    rng = np.random.default_rng(1)
    n = 3000
    cat = rng.integers(0, 8, n)
    # categories {1, 5, 6} are positive
    y = np.isin(cat, [1, 5, 6]).astype(np.float32)
    codes = np.stack([cat, rng.integers(0, 8, n)], 1)
    data = BinnedData.from_codes(codes, y, np.array([9, 8]), np.array([1, 0]))
    tr = TreeTrainer(TreeConfig("GBT", tree_num=1, max_depth=2, feature_subset_strategy="ALL"), data)
    tr.train()
    t = tr.trees[0]
    assert t.feat[1] == 0
    bits = t.cat_left[1][0]
    left = {c for c in range(9) if (bits >> c) & 1}
    # empty missing bin 8 sorts as Double.MIN_VALUE (after the zero-mean bins); first max wins
    assert left == {0, 2, 3, 4, 7}
    assert abs(tr.train_errors[0]) < 1e-6


def test_strategy_counts():
    assert _strategy_count("TWOTHIRDS", 30, 30, 10) == 20
    assert _strategy_count("HALF", 30, 30, 10) == 15
    assert _strategy_count("ALL", 30, 30, 10) == 30
    assert _strategy_count(0.5, 30, 30, 10) == 15
    assert _strategy_count("SQRT", 100, 100, 10) == 10


@pytest.mark.gpu
@pytest.mark.parametrize("imp", ["variance", "entropy"])
def test_gpu_trees_match_cpu(imp):
    data_c, codes, y = _data(n=20000, f=40, nb=64, seed=5, cat_cols=(3,))
    data_g = BinnedData.from_codes(codes, y, data_c.nbins, data_c.is_cat, device="cuda")
    cfg = dict(algorithm="GBT", tree_num=4, max_depth=5, learning_rate=0.2, impurity=imp,
               feature_subset_strategy="ALL")
    tc = TreeTrainer(TreeConfig(**cfg), data_c)
    tg = TreeTrainer(TreeConfig(**cfg), data_g)
    tc.train()
    tg.train()
    for a, b in zip(tc.trees, tg.trees):
        assert (a.feat == b.feat).all()
        assert (a.thr == b.thr).all()
        assert np.allclose(a.value, b.value, atol=1e-4)
    assert np.allclose(tc.pred.numpy(), tg.pred.cpu().numpy(), atol=1e-4)
    assert abs(tc.train_errors[-1] - tg.train_errors[-1]) < 1e-5


@pytest.mark.gpu
def test_gpu_many_items_and_feature_mask():
    from shifu_amd.models.gbdt import synthetic_binned
    data = synthetic_binned(300000, 100, "cuda", seed=2)
    tr = TreeTrainer(TreeConfig("GBT", tree_num=3, max_depth=7, feature_subset_strategy="TWOTHIRDS"), data)
    tr.train()
    assert tr.train_errors[-1] < tr.train_errors[0]
    host = data.codes().cpu().numpy()
    p = np.zeros(data.n, np.float32)
    for i, t in enumerate(tr.trees):
        v = t.predict_bins(host, data.is_cat)
        p = v if i == 0 else p + t.weight * v
    assert np.allclose(p, tr.pred.cpu().numpy(), atol=1e-4)


def test_max_leaves_budget():
    import numpy as np
    import torch
    from shifu_amd.models.gbdt import BinnedData, TreeConfig, TreeTrainer
    rng = np.random.default_rng(3)
    codes = rng.integers(0, 32, size=(3000, 8))
    y = (codes[:, 0] + codes[:, 1] * 0.5 + rng.normal(size=3000) * 3 > 24).astype(np.float32)
    d = BinnedData.from_codes(torch.from_numpy(codes), y, np.full(8, 32))
    for ml in (3, 7, 12):
        tt = TreeTrainer(TreeConfig("GBT", tree_num=2, max_depth=6, max_leaves=ml, feature_subset_strategy="ALL",
                                    min_instances_per_node=1), d)
        tt.train()
        for t in tt.trees:
            assert 2 <= len(t.leaves()) <= ml


def _rf_trees(data, batch, monkeypatch, **kw):
    monkeypatch.setenv("SHIFU_RF_BATCH", str(batch))
    cfg = dict(algorithm="RF", tree_num=5, max_depth=5, impurity="gini", sample_with_replacement=True,
               feature_subset_strategy="HALF", seed=11, max_leaves=kw.get("max_leaves", 0))
    tr = TreeTrainer(TreeConfig(**cfg), data)
    tr.train()
    return tr


def _same_trees(ta, tb, atol=0.0):
    assert len(ta.trees) == len(tb.trees)
    for a, b in zip(ta.trees, tb.trees):
        assert (a.feat == b.feat).all() and (a.thr == b.thr).all() and (a.exists == b.exists).all()
        assert np.allclose(a.value, b.value, atol=atol) and (a.cat_left == b.cat_left).all()


@pytest.mark.parametrize("max_leaves", [0, 9])
def test_rf_forest_batch_equals_sequential(monkeypatch, max_leaves):
    """F5 tree parallelism: RF trees grown together in one level loop (virtual positions
    tree*N + row, one histogram pass + one all-reduce per level for the whole batch) are the
    same trees as growing them one at a time."""
    data, _, _ = _data(n=1400, f=7, nb=10, seed=4, cat_cols=(2,))
    one = _rf_trees(data, 1, monkeypatch, max_leaves=max_leaves)
    four = _rf_trees(data, 4, monkeypatch, max_leaves=max_leaves)   # batches of 4 + 1
    _same_trees(one, four)
    assert np.allclose(one.pred.numpy(), four.pred.numpy())


def test_rf_forest_batch_checkpoint_keeps_pending(monkeypatch):
    data, _, _ = _data(n=900, f=5, nb=8, seed=6)
    ref = _rf_trees(data, 4, monkeypatch)
    monkeypatch.setenv("SHIFU_RF_BATCH", "4")
    cfg = dict(algorithm="RF", tree_num=5, max_depth=5, impurity="gini", sample_with_replacement=True,
               feature_subset_strategy="HALF", seed=11)
    a = TreeTrainer(TreeConfig(**cfg), data)
    a.train(2)                                  # 2 trees used, 2 grown ahead and pending
    st = a.state_dict()
    b = TreeTrainer(TreeConfig(**cfg), data)
    b.load_state_dict(st)
    b.train(3)
    _same_trees(ref, b)


@pytest.mark.gpu
def test_gpu_rf_forest_batch_matches_sequential(monkeypatch):
    """HIP path: batch of 3 (+2) RF trees == the same trees grown one by one on the GPU (the
    Poisson subsample weights come from the device generator, so the CPU oracle draws others)."""
    data_c, codes, y = _data(n=30000, f=40, nb=64, seed=8, cat_cols=(5,))
    data_g = BinnedData.from_codes(codes, y, data_c.nbins, data_c.is_cat, device="cuda")
    t1 = _rf_trees(data_g, 1, monkeypatch)
    t3 = _rf_trees(data_g, 3, monkeypatch)
    _same_trees(t1, t3, atol=1e-6)
    assert np.allclose(t1.pred.cpu().numpy(), t3.pred.cpu().numpy(), atol=1e-6)


def test_resume_reproduces_uninterrupted_sampled_run():
    """Row sub-sampling streams are a function of (seed, rank, tree index): 3 trees, a checkpoint
    round trip into a fresh trainer, 3 more trees == 6 trees straight.  (With DropoutRate > 0 the
    per-row skipped updates are not in the checkpoint -- predictions are replayed from the trees,
    as the reference's resumed workers do -- so that case is not bit-exact.)"""
    cfg = dict(algorithm="GBT", tree_num=6, max_depth=3, learning_rate=0.2, bagging_sample_rate=0.7,
               feature_subset_strategy="ALL", seed=5)
    data, _, _ = _data(n=1500, f=6)
    a = TreeTrainer(TreeConfig(**cfg), data)
    a.train(6)
    b = TreeTrainer(TreeConfig(**cfg), data)
    b.train(3)
    st = b.state_dict()
    c = TreeTrainer(TreeConfig(**cfg), data)
    c.load_state_dict(st)
    c.train(3)
    assert len(c.trees) == 6
    for ta, tc in zip(a.trees, c.trees):
        assert np.array_equal(ta.feat, tc.feat) and np.array_equal(ta.thr, tc.thr)
        np.testing.assert_allclose(ta.value, tc.value, rtol=1e-6)
    np.testing.assert_allclose(a.pred.numpy(), c.pred.numpy(), rtol=1e-5, atol=1e-6)


# ---- native multi-class RF (Entropy / Gini over C classes) + RF out-of-bag errors ------------------
def _mc_data(n=900, f=5, nb=10, C=3, seed=0, device="cpu", cat_cols=(1,)):
    rng = np.random.default_rng(seed)
    codes = rng.integers(0, nb, size=(n, f))
    y = np.where(codes[:, 0] < 3, 0, np.where(codes[:, 1] % 3 == 0, 1, 2)).astype(np.float32)
    y = np.where(rng.random(n) < 0.1, rng.integers(0, C, n), y).astype(np.float32)
    is_cat = np.zeros(f, np.uint8)
    for c in cat_cols:
        is_cat[c] = 1
    return BinnedData.from_codes(codes, y, np.full(f, nb), is_cat, device=device), codes, y


def _mc_imp(counts, imp):
    s = counts.sum()
    if s == 0:
        return 0.0
    p = counts / s
    if imp == "gini":
        return -float((p * p).sum())
    p = p[p > 0]
    return -float((p * np.log2(p)).sum())


def _mc_bruteforce(codes, y, C, nb, is_cat, imp, min_inst):
    """Impurity.java Entropy/Gini computeImpurity: categorical bins ordered by class-1 rate of
    (class 0 + class 1), numeric bins in order; best = max gain, first feature / bin on ties."""
    best = (-np.inf, None, None, None)
    for f in range(codes.shape[1]):
        st = np.zeros((nb, C))
        np.add.at(st, (codes[:, f], y.astype(int)), 1.0)
        order = list(range(nb))
        if is_cat[f]:
            den = st[:, 0] + st[:, 1]
            key = np.where(den != 0, st[:, 1] / np.where(den != 0, den, 1), 0.0)
            order = sorted(range(nb), key=lambda b: (key[b], b))
        tot = st.sum(0)
        base = _mc_imp(tot, imp)
        left = np.zeros(C)
        for i in range(nb - 1):
            left = left + st[order[i]]
            right = tot - left
            lw, rw = left.sum(), right.sum()
            if lw <= min_inst or rw <= min_inst:
                continue
            gain = base - lw / tot.sum() * _mc_imp(left, imp) - rw / tot.sum() * _mc_imp(right, imp)
            if gain > best[0] + 1e-12:
                best = (gain, f, i, (int(np.argmax(left)), int(np.argmax(right))))
    return best


@pytest.mark.parametrize("imp", ["entropy", "gini"])
def test_multiclass_root_split_matches_reference_rule(imp):
    data, codes, y = _mc_data()
    cfg = TreeConfig("RF", tree_num=1, max_depth=2, impurity=imp, feature_subset_strategy="ALL",
                     min_instances_per_node=5, n_classes=3)
    tr = TreeTrainer(cfg, data)
    t = tr.train(1)[0]
    gain, f, i, (cl, cr) = _mc_bruteforce(codes, y, 3, 10, data.is_cat, imp, 5)
    assert t.feat[1] == f
    assert abs(t.gain[1] - gain) < 1e-5
    assert (t.class_value[2], t.class_value[3]) == (cl, cr)
    assert t.classification and t.class_value[1] == np.argmax(np.bincount(y.astype(int), minlength=3))


def test_multiclass_rf_votes_learn_the_rule():
    data, codes, y = _mc_data(n=3000, seed=1)
    cfg = TreeConfig("RF", tree_num=6, max_depth=5, impurity="gini", feature_subset_strategy="ALL",
                     bagging_sample_rate=0.8, n_classes=3, seed=3)
    tr = TreeTrainer(cfg, data)
    tr.train()
    pred = tr.predict(data).numpy()
    assert (pred == y).mean() > 0.85
    assert set(np.unique(pred)) <= {0.0, 1.0, 2.0}


def test_rf_oob_errors_match_manual_accumulation():
    data, codes, y = _data(n=800, seed=4)
    cfg = TreeConfig("RF", tree_num=4, max_depth=3, impurity="variance", feature_subset_strategy="ALL",
                     bagging_sample_rate=0.6, sample_with_replacement=False, seed=2)
    tr = TreeTrainer(cfg, data)
    tr.train()
    num_in = den_in = num_oob = den_oob = 0.0
    for i, t in enumerate(tr.trees):
        tr._reseed_rows(i)
        sub, _ = tr._subsample()
        sub = sub.numpy()
        p = t.predict_bins(codes, data.is_cat).astype(np.float64)
        e = (p - y) ** 2
        num_in += (sub * e)[sub > 0].sum()
        den_in += sub[sub > 0].sum()
        num_oob += e[sub == 0].sum()
        den_oob += (sub == 0).sum()
    assert abs(tr.train_errors[-1] - num_in / den_in) < 1e-6
    assert abs(tr.valid_errors[-1] - num_oob / den_oob) < 1e-6
    assert abs(tr.oob_error - num_oob / den_oob) < 1e-6
    # resume replays the same cumulative sums
    st = tr.state_dict()
    tr2 = TreeTrainer(cfg, data)
    tr2.load_state_dict(st)
    assert abs(tr2.oob_error - tr.oob_error) < 1e-9


@pytest.mark.gpu
@pytest.mark.parametrize("imp", ["entropy", "gini"])
def test_multiclass_gpu_matches_cpu(imp):
    """Per-class histograms from the HIP kernel + the vectorized gain scan == the CPU oracle."""
    cfg = dict(algorithm="RF", tree_num=3, max_depth=4, impurity=imp, feature_subset_strategy="ALL",
               bagging_sample_rate=1.0, n_classes=3, seed=5)   # bags are device-RNG streams
    dc, codes, y = _mc_data(n=5000, seed=7)
    dg = BinnedData.from_codes(codes, y, dc.nbins, dc.is_cat, device="cuda")
    tc, tg = TreeTrainer(TreeConfig(**cfg), dc), TreeTrainer(TreeConfig(**cfg), dg)
    tc.train()
    tg.train()
    for a, b in zip(tc.trees, tg.trees):
        assert np.array_equal(a.feat, b.feat) and np.array_equal(a.thr, b.thr)
        assert np.array_equal(a.class_value, b.class_value)
    assert np.array_equal(tc.predict(dc).numpy(), tg.predict(dg).cpu().numpy())


@pytest.mark.gpu
@pytest.mark.parametrize("alg", ["GBT", "RF"])
def test_gpu_host_resident_bins_match_device(alg, monkeypatch):
    """Out-of-core trees: bins in pinned host memory read by the kernels in place grow the same
    trees and predictions as HBM-resident bins (RF also through the forest-batch path)."""
    monkeypatch.setenv("SHIFU_RF_BATCH", "2")
    data_c, codes, y = _data(n=20000, f=40, nb=64, seed=5, cat_cols=(3,))
    dd = BinnedData.from_codes(codes, y, data_c.nbins, data_c.is_cat, device="cuda")
    dh = BinnedData.host_resident(codes, y, data_c.nbins, data_c.is_cat, device="cuda")
    assert dh.bins.device.type == "cpu" and dh.bins.is_pinned() and dh.bins_dptr
    assert torch.equal(dh.bins, dd.bins.cpu())
    cfg = dict(algorithm=alg, tree_num=4, max_depth=5, learning_rate=0.2, feature_subset_strategy="ALL")
    if alg == "RF":
        cfg.update(bagging_sample_rate=0.8, feature_subset_strategy="HALF")
    ta, tb = TreeTrainer(TreeConfig(**cfg), dd), TreeTrainer(TreeConfig(**cfg), dh)
    ta.train()
    tb.train()
    for a, b in zip(ta.trees, tb.trees):
        assert (a.feat == b.feat).all() and (a.thr == b.thr).all()
        assert np.array_equal(a.value, b.value)
    assert torch.equal(ta.pred, tb.pred)


@pytest.mark.gpu
def test_gpu_quantised_splits_vs_fp64_oracle():
    """the int64 fixed-point histograms (w 16-bit, w*g 23-bit grid; root w*g 2^3
    coarser) against an UNQUANTISED fp64 oracle.  2M rows x 200 features, depth 5 GBT, 3 trees:
    for every split node, the exact fp64 best (feature, bin) over the rows that reach it (same
    variance gain, same min-instances rule, lowest feature / bin on ties) is compared with the
    GPU's choice.  Near-ties may flip; the chosen split must then lose < 1e-6 of the exact gain."""
    import torch
    from shifu_amd.models.gbdt import TreeConfig, TreeTrainer, synthetic_binned
    dev = torch.device("cuda")
    n, F = 2_000_000, 200
    data = synthetic_binned(n, F, dev, seed=17)
    cfg = TreeConfig("GBT", tree_num=3, max_depth=5, learning_rate=0.1, feature_subset_strategy="ALL",
                     min_instances_per_node=5)
    tr = TreeTrainer(cfg, data)
    codes = data.codes().long()                         # [n, F] on the device
    pred = torch.zeros(n, dtype=torch.float64, device=dev)
    y = data.y.double()
    w = torch.ones(n, dtype=torch.float64, device=dev)
    same = total = 0
    flips = []
    worst = 1.0
    for t in range(3):
        g = y if t == 0 else 2.0 * (y - pred)           # squared loss: output = -dL/dp = 2 (y - p)
        tr.train(1)
        tree = tr.trees[-1]
        node = torch.ones(n, dtype=torch.int64, device=dev)
        for depth in range(cfg.max_depth - 1):
            ids = torch.unique(node).tolist()
            for nid in ids:
                if nid >= len(tree.feat) or tree.feat[nid] < 0:
                    continue
                m = node == nid
                b = codes[m]
                gw = (w[m] * g[m])
                idx = (torch.arange(F, device=dev).unsqueeze(0) * 256 + b).reshape(-1)
                hw = torch.zeros(F * 256, dtype=torch.float64, device=dev).index_add_(
                    0, idx, w[m].unsqueeze(1).expand(-1, F).reshape(-1)).view(F, 256)
                hg = torch.zeros(F * 256, dtype=torch.float64, device=dev).index_add_(
                    0, idx, gw.unsqueeze(1).expand(-1, F).reshape(-1)).view(F, 256)
                pw, ps = hw.cumsum(1)[:, :255], hg.cumsum(1)[:, :255]
                tw, ts = hw.sum(1, keepdim=True), hg.sum(1, keepdim=True)
                rw, rs = tw - pw, ts - ps
                gain = (ps * ps / pw + rs * rs / rw - ts * ts / tw) / tw
                gain = torch.where((pw > cfg.min_instances_per_node) & (rw > cfg.min_instances_per_node), gain,
                                   torch.full_like(gain, -1.0))
                flat = gain.reshape(-1)
                best = float(flat.max())
                k = int(torch.nonzero(flat == best)[0])
                f_gpu, b_gpu = int(tree.feat[nid]), int(tree.thr[nid])
                total += 1
                if (k // 255, k % 255) == (f_gpu, b_gpu):
                    same += 1
                else:
                    # gain lost by the flip, relative to the node's own scale (sum g^2 / n):
                    # near-zero-gain nodes (a fitted residual) tie at any split
                    scale = float((gw * g[m]).sum() / m.sum())
                    loss = (best - float(gain[f_gpu, b_gpu])) / max(scale, 1e-300)
                    flips.append((t, nid, f_gpu, b_gpu, k // 255, k % 255, best, float(gain[f_gpu, b_gpu]), scale))
                    worst = min(worst, 1.0 - loss)
            go_left = torch.zeros(n, dtype=torch.bool, device=dev)
            for nid in ids:
                if nid < len(tree.feat) and tree.feat[nid] >= 0:
                    m = node == nid
                    go_left[m] = codes[m, int(tree.feat[nid])] <= int(tree.thr[nid])
            split = torch.tensor([nid < len(tree.feat) and tree.feat[nid] >= 0 for nid in range(int(node.max()) + 1)],
                                 device=dev)
            s = split[node]
            node = torch.where(s, 2 * node + (~go_left).long(), node)
        # GBT update as the trainer does (first tree weight 1, then learning rate)
        vals = torch.tensor(tree.value, dtype=torch.float64, device=dev)
        pred += (1.0 if t == 0 else cfg.learning_rate) * vals[node]
    print(f"quantised vs fp64 splits: {same}/{total} identical, worst relative gain loss of a flip "
          f"{1 - worst:.3e}; flips (tree, node, gpu f/b, exact f/b, best, chosen, scale): {flips[:8]}")
    assert total >= 20
    assert same / total >= 0.95
    assert worst > 1 - 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("n", [300001, 257])
def test_gpu_feature_tiled_root_matches_quad_records(n, monkeypatch):
    """The feature-tiled root copy ([G][NT][32][128]: tiled root histogram + partition reads) grows
    the same trees and predictions, bit for bit, as the quad-record root path (no copy), with a
    row count that leaves a partial last tile and a feature count that leaves a partial group."""
    import torch
    from shifu_amd.models import gbdt as gb
    from shifu_amd.models.gbdt import TreeConfig, TreeTrainer, synthetic_binned
    data = synthetic_binned(n, 100, "cuda", seed=4, labels="balanced")
    cfg = TreeConfig("GBT", tree_num=3, max_depth=6, learning_rate=0.1, feature_subset_strategy="ALL",
                     min_instances_per_node=2)
    runs = []
    for tiled in (True, False):
        monkeypatch.setattr(gb, "ROOT_G32", tiled)
        tr = TreeTrainer(cfg, data)
        tr.train()
        assert (getattr(tr, "_g32", None) is not None and tr._g32 is not False) == tiled
        runs.append(tr)
    a, b = runs
    for x, y in zip(a.trees, b.trees):
        assert (x.feat == y.feat).all() and (x.thr == y.thr).all()
        assert np.array_equal(x.value, y.value)
    assert torch.equal(a.pred, b.pred)


@pytest.mark.gpu
@pytest.mark.parametrize("w_rows,y_blocks", [(1000, 3), (1 << 16, 128)])
def test_gpu_leaf_window_update_matches_position_pass(w_rows, y_blocks, monkeypatch):
    """The final-level prediction update walked in row windows (per-node position sub-ranges found
    by binary search, XCD-ordered windows) gives the same trees and the same pred, bit for bit, as
    the position-ordered flag pass; a small window exercises many windows and empty sub-ranges."""
    import torch
    from shifu_amd.models import gbdt as gb
    from shifu_amd.models.gbdt import TreeConfig, TreeTrainer, synthetic_binned
    data = synthetic_binned(200003, 70, "cuda", seed=9, labels="balanced")
    cfg = TreeConfig("GBT", tree_num=3, max_depth=6, learning_rate=0.1, feature_subset_strategy="ALL",
                     min_instances_per_node=2)
    monkeypatch.setattr(gb, "LEAF_W", w_rows)
    monkeypatch.setattr(gb, "LEAF_Y", y_blocks)
    runs = []
    for win in (True, False):
        monkeypatch.setattr(gb, "LEAF_WINDOW", win)
        tr = TreeTrainer(cfg, data)
        tr.train()
        runs.append(tr)
    a, b = runs
    for x, y in zip(a.trees, b.trees):
        assert (x.feat == y.feat).all() and (x.thr == y.thr).all()
        assert np.array_equal(x.value, y.value)
    assert torch.equal(a.pred, b.pred)


@pytest.mark.gpu
@pytest.mark.parametrize("alg,f", [("GBT", 100), ("GBT", 70), ("RF", 45)])
def test_gpu_hist64_matches_group_items(alg, f, monkeypatch):
    """Below-root histograms from 64-feature half-record blocks (paired 32-feature items, a lone
    last group when the group count is odd, forest batches for RF) give the same trees and
    predictions, bit for bit, as the per-group kernel."""
    import torch
    from shifu_amd.models import gbdt as gb
    from shifu_amd.models.gbdt import TreeConfig, TreeTrainer, synthetic_binned
    monkeypatch.setenv("SHIFU_RF_BATCH", "2")
    monkeypatch.setattr(gb, "HIST64_MIN_NODE_ROWS", 0)        # every non-root level
    data = synthetic_binned(150001, f, "cuda", seed=11, labels="balanced")
    kw = dict(tree_num=3, max_depth=6, feature_subset_strategy="ALL", min_instances_per_node=2)
    if alg == "RF":
        kw.update(bagging_sample_rate=0.7, feature_subset_strategy="HALF")
    else:
        kw.update(learning_rate=0.1)
    runs = []
    for on in (True, False):
        monkeypatch.setattr(gb, "HIST64", on)
        tr = TreeTrainer(TreeConfig(alg, **kw), data)
        tr.train()
        runs.append(tr)
    a, b = runs
    for x, y in zip(a.trees, b.trees):
        assert (x.feat == y.feat).all() and (x.thr == y.thr).all()
        assert np.array_equal(x.value, y.value)
    assert torch.equal(a.pred, b.pred)


def test_group_pairs_matches_sorting_construction():
    """Half-record pairing of histogram items (O(n) scan) equals the pairing by sorting keys, for
    group counts with and without a lone last group."""
    from shifu_amd.models.gbdt import _group_pairs
    rng = np.random.default_rng(0)
    for G in (32, 31, 3, 1, 7):
        rows = []
        for node in range(5):
            for q in range((G + 3) // 4):
                for ch in range(int(rng.integers(1, 6))):
                    for sg in range(4):
                        if q * 4 + sg < G:
                            rows.append((node, ch * 1000 + node, ch * 1000 + 1000, q * 4 + sg))
        items = np.array(rows, np.int32)
        key = np.stack([items[:, 0], items[:, 1], items[:, 2], items[:, 3] >> 1], 1)
        uniq, inv = np.unique(key, axis=0, return_inverse=True)
        ref = np.full((len(uniq), 2), -1, np.int32)
        ref[inv.reshape(-1), items[:, 3] & 1] = np.arange(len(items), dtype=np.int32)
        got = _group_pairs(items)
        assert sorted(map(tuple, got.tolist())) == sorted(map(tuple, ref.tolist()))
        assert ((got[:, 0] < 0) | (items[np.maximum(got[:, 0], 0), 3] % 2 == 0)).all()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["gbt_balanced", "gbt_categorical", "rf_forest_poisson"])
def test_gpu_device_decisions_match_host_path(case, monkeypatch):
    """Split decisions made on the device ahead of the partition (shifu_gbdt_decide), node row
    ranges kept on the device and histogram items sized from estimated child sizes
    (shifu_gbdt_items_fix, empty chunks included) grow the same trees, categorical left sets and
    predictions, bit for bit, as the host-decision path with two syncs per level."""
    from shifu_amd.models import gbdt as gb
    from shifu_amd.models.gbdt import synthetic_binned
    monkeypatch.setenv("SHIFU_RF_BATCH", "3")
    if case == "gbt_categorical":
        _, codes, y = _data(n=40000, f=40, nb=64, seed=7, cat_cols=(1, 3, 17))
        nbins = np.full(40, 64)
        is_cat = np.zeros(40, np.uint8)
        is_cat[[1, 3, 17]] = 1
        data = BinnedData.from_codes(codes, y, nbins, is_cat, device="cuda")
        cfg = TreeConfig("GBT", tree_num=3, max_depth=6, learning_rate=0.2, feature_subset_strategy="ALL",
                         min_instances_per_node=2)
    elif case == "gbt_balanced":
        data = synthetic_binned(200003, 70, "cuda", seed=12, labels="balanced")
        cfg = TreeConfig("GBT", tree_num=3, max_depth=7, learning_rate=0.1, feature_subset_strategy="ALL",
                         min_instances_per_node=2)
    else:
        data = synthetic_binned(120001, 45, "cuda", seed=13, labels="balanced")
        cfg = TreeConfig("RF", tree_num=4, max_depth=6, feature_subset_strategy="HALF", min_instances_per_node=2,
                         bagging_sample_rate=0.6, sample_with_replacement=True, seed=5)
    runs = []
    # device decisions with the node-range lookup, with the per-position node array, host path
    for dev_dec, ranges in ((True, True), (True, False), (False, False)):
        monkeypatch.setattr(gb, "DEV_DECIDE", dev_dec)
        monkeypatch.setattr(gb, "RANGE_NODES", ranges)
        tr = TreeTrainer(cfg, data)
        assert tr._pipelined(1) == dev_dec
        tr.train()
        runs.append(tr)
    b = runs[-1]
    for a in runs[:-1]:
        assert a.hist_rows_total == b.hist_rows_total
        for x, y_ in zip(a.trees, b.trees):
            assert (x.feat == y_.feat).all() and (x.thr == y_.thr).all()
            assert np.array_equal(x.value, y_.value) and np.array_equal(x.wgt_cnt, y_.wgt_cnt)
            assert np.array_equal(np.asarray(x.cat_left), np.asarray(y_.cat_left))
        if case == "gbt_categorical":
            assert any((np.asarray(t.cat_left) != 0).any() for t in a.trees)
        assert torch.equal(a.pred, b.pred)
        # (the residual kernel's error sum uses float64 atomics: equal up to summation order)
        assert np.allclose(a.train_errors, b.train_errors, rtol=1e-9, atol=0)


def test_categorical_split_with_many_categories_partitions_rows():
    """A categorical split whose left set holds categories >= 8: every left category's rows go
    left (the host's left-set bits were once built with a uint8 shift that dropped them)."""
    rng = np.random.default_rng(4)
    n = 4000
    cat = rng.integers(0, 40, n)
    pos = np.array([9, 13, 22, 31, 38])
    y = np.isin(cat, pos).astype(np.float32)
    codes = np.stack([cat, rng.integers(0, 8, n)], 1)
    data = BinnedData.from_codes(codes, y, np.array([41, 8]), np.array([1, 0]))
    tr = TreeTrainer(TreeConfig("GBT", tree_num=1, max_depth=2, feature_subset_strategy="ALL"), data)
    tr.train()
    t = tr.trees[0]
    assert t.feat[1] == 0
    left = {c for c in range(41) if (int(t.cat_left[1][c >> 5]) >> (c & 31)) & 1}
    assert left == set(pos.tolist()) or left.isdisjoint(pos.tolist())
    assert abs(tr.train_errors[0]) < 1e-6


def test_estimated_items_cover_each_node_exactly_once():
    """Histogram items sized from estimated child sizes (TreeTrainer._make_items(est=True): rows
    (slot, chunk, n_chunks, group)) resolved against the real node ranges the way
    gbdt_items_fix_kernel does: every (node, group) covers its node's rows exactly once, whether
    the estimate is high, low or the node is empty."""
    from shifu_amd.models.gbdt import TreeTrainer, TreeConfig
    data, _, _ = _data(n=500, f=70)
    tr = TreeTrainer(TreeConfig("GBT", tree_num=1, max_depth=3, feature_subset_strategy="ALL"), data)
    tr._root_level = False
    real = [(0, 3_000_000), (3_000_000, 3_000_000), (3_000_000, 3_900_000), (5_000_000, 5_000_017)]
    est = [2_000_000, 40_000, 5_000_000, 1]
    nodes = [{"slot": s, "built": True, "m": e} for s, e in enumerate(est)]
    nodes.append({"slot": 4, "built": False, "m": 123})
    items, ni, max_items = tr._make_items(nodes, 4, est=True)
    assert items.shape[1] == 4 and len(items)
    G = tr.ngroups
    starts = np.array([r[0] for r in real] + [0])
    ends = np.array([r[1] for r in real] + [0])
    cover = {}
    for slot, ch, k, grp in items:                    # gbdt_items_fix_kernel
        s, m = starts[slot], max(0, ends[slot] - starts[slot])
        step = (m + k - 1) // k
        lo, hi = min(m, ch * step), min(m, min(m, ch * step) + step)
        cover.setdefault((slot, grp), []).append((s + lo, s + hi))
    for slot in range(4):
        for grp in range(G):
            segs = sorted(cover.get((slot, grp), []))
            tot = sum(h - l for l, h in segs)
            assert tot == ends[slot] - starts[slot], (slot, grp, tot)
            for (l0, h0), (l1, h1) in zip(segs, segs[1:]):
                assert h0 <= l1                        # no overlap
            ids = ni[slot, grp]
            assert sorted(int(i) for i in ids if i >= 0) == sorted(
                int(i) for i in np.flatnonzero((items[:, 0] == slot) & (items[:, 3] == grp)))
    assert (ni[4] < 0).all()                          # derived node: no items
