"""HIP stats / normalize / bin-code / LR / sensitivity kernels vs the fp64 CPU oracles."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

NORMS = ["ZSCALE", "OLD_ZSCALE", "WOE", "WEIGHT_WOE", "WOE_ZSCORE", "WEIGHT_WOE_ZSCALE", "HYBRID", "ONEHOT",
         "ZSCALE_ONEHOT", "ASIS_WOE", "ASIS_PR", "DISCRETE_ZSCORE", "ZSCALE_INDEX", "WOE_INDEX", "WOE_ZSCALE_INDEX"]


@pytest.fixture(scope="module")
def prepared(tmp_path_factory):
    from shifu_amd.steps.base import ModelSet
    from shifu_amd.utils.synthetic import make_model_set
    root = make_model_set(str(tmp_path_factory.mktemp("k")), "k", "NN", n_rows=5000)
    from shifu_amd.cli import main
    import os
    cwd = os.getcwd()
    os.chdir(root)
    try:
        assert main(["init"]) == 0
    finally:
        os.chdir(cwd)
    ms = ModelSet(root)
    cols = [c for c in ms.ccs if not c.is_target() and not c.is_meta() and not c.is_weight()]
    md = ms.load_raw(cols)
    return ms, cols, md


def test_column_stats_gpu_matches_cpu(prepared):
    import copy
    from shifu_amd.algos.stats import compute_column_stats
    ms, cols, md = prepared
    a = copy.deepcopy(ms.ccs)
    b = copy.deepcopy(ms.ccs)
    compute_column_stats(ms.mc, a, md, device="cpu")
    compute_column_stats(ms.mc, b, md, device="cuda")
    for ca, cb in zip(a, b):
        if ca.is_target() or ca.is_meta():
            continue
        assert ca.bin_boundary == cb.bin_boundary and ca.bin_category == cb.bin_category
        assert ca.bin_count_pos == cb.bin_count_pos and ca.bin_count_neg == cb.bin_count_neg, ca.name
        np.testing.assert_allclose(ca.bin_weighted_pos, cb.bin_weighted_pos, rtol=1e-9)
        for k in ("mean", "stdDev", "min", "max", "skewness", "kurtosis", "ks", "iv", "median", "distinctCount"):
            va, vb = ca.stats.get(k), cb.stats.get(k)
            if va is None:
                assert vb is None
            else:
                assert vb == pytest.approx(va, rel=1e-9, abs=1e-9), (ca.name, k)


@pytest.mark.parametrize("nt", NORMS)
def test_normalize_gpu_matches_cpu(prepared, nt):
    import copy
    from shifu_amd.algos.normalize import normalize_table, normalize_table_gpu
    from shifu_amd.algos.stats import compute_column_stats
    ms, cols, md = prepared
    ccs = copy.deepcopy(ms.ccs)
    compute_column_stats(ms.mc, ccs, md, device="cpu")
    c2 = [c for c in ccs if c.name in {x.name for x in cols}]
    X1, n1, _ = normalize_table(ms.mc, ccs, md.table, columns=c2, norm_type=nt)
    X2, n2, _ = normalize_table_gpu(ms.mc, ccs, md.table, columns=c2, norm_type=nt)
    assert n1 == n2
    np.testing.assert_allclose(X2, X1, rtol=1e-6, atol=1e-6)


def test_bin_codes_gpu_matches_cpu(prepared):
    import copy
    from shifu_amd.algos.normalize import tree_bin_codes, tree_bin_codes_gpu
    from shifu_amd.algos.stats import compute_column_stats
    ms, cols, md = prepared
    ccs = copy.deepcopy(ms.ccs)
    compute_column_stats(ms.mc, ccs, md, device="cpu")
    c2 = [c for c in ccs if c.name in {x.name for x in cols}]
    C1, nb1, ic1 = tree_bin_codes(ccs, md.table, c2)
    C2, nb2, ic2 = tree_bin_codes_gpu(ccs, md.table, c2)
    np.testing.assert_array_equal(C1, C2)
    np.testing.assert_array_equal(nb1, nb2)


@pytest.mark.parametrize("dtype,F", [(torch.float32, 37), (torch.float32, 1000), (torch.bfloat16, 1000)])
def test_lr_grad_kernel(dtype, F):
    from shifu_amd.ops import stats_ops
    g = torch.Generator().manual_seed(0)
    n = 20000
    fp = (F + 7) // 8 * 8
    xp = torch.zeros(n, fp, dtype=dtype, device="cuda")
    xp[:, :F] = torch.randn(n, F, generator=g).to("cuda", dtype)
    x = xp[:, :F]
    w = (torch.randn(F + 1, generator=g) * 0.05).cuda()
    y = (torch.rand(n, generator=g) > 0.5).float().cuda()
    s = torch.rand(n, generator=g).cuda()
    grad, err = stats_ops.lr_grad(x, w, y, s)
    xf = x.float().double()
    p = torch.sigmoid(xf @ w[:-1].double() + w[-1].double())
    e = y.double() - p
    d = e * (p * (1 - p) + 0.1) * s.double()
    ref = torch.cat([d @ xf, d.sum()[None]])
    torch.testing.assert_close(grad.double(), ref, rtol=2e-3, atol=2e-3)
    assert float(err) == pytest.approx(float((e * e).sum()), rel=1e-4)


@pytest.mark.parametrize("dtype,F", [(torch.float32, 2500), (torch.bfloat16, 5000)])
def test_lr_step_above_k9_limit_on_own_dot_kernels(dtype, F):
    """Feature counts above K9's limit: the LR step's score / gradient run on the own row / column
    dot kernels (no vendor GEMV), equal to the CPU trainer's step on the same data."""
    from shifu_amd.models.lr import LRTrainer
    g = torch.Generator().manual_seed(2)
    n = 9000
    x = torch.randn(n, F, generator=g).to(dtype).float()
    y = (torch.rand(n, generator=g) > 0.5).float()
    errs = {}
    ws = {}
    for dev in ("cpu", "cuda"):
        t = LRTrainer(F, device=dev, propagation="R", input_dtype="bf16" if dtype == torch.bfloat16 else "auto")
        t.w.copy_((torch.randn(F + 1, generator=torch.Generator().manual_seed(3)) * 0.02).to(dev))
        data = t.prepare(x, y) if hasattr(t, "prepare") else None
        # the row dtype is explicit: fp32 unless bf16 is asked for (or fp32 rows do not fit in HBM)
        want = "bf16" if (dev == "cuda" and dtype == torch.bfloat16) else "fp32"
        assert t.input_dtype == want and data[0].dtype == (torch.bfloat16 if want == "bf16" else torch.float32)
        errs[dev] = [t.step(data) for _ in range(3)]
        ws[dev] = t.w.cpu()
    for a, b in zip(errs["cpu"], errs["cuda"]):
        assert abs(a - b) / a < 1e-3, (errs)
    assert float((ws["cpu"] - ws["cuda"]).abs().max()) < 1e-3


def test_rowdot_coldot_kernels_match_torch():
    from shifu_amd.ops import stats_ops
    g = torch.Generator(device="cuda").manual_seed(1)
    for dt in (torch.float32, torch.bfloat16):
        x = torch.randn(3001, 700, device="cuda", generator=g).to(dt)
        w = torch.randn(700, device="cuda", generator=g)
        d = torch.randn(3001, device="cuda", generator=g)
        torch.testing.assert_close(stats_ops.rowdot(x, w), x.float() @ w, rtol=1e-4, atol=1e-3)
        torch.testing.assert_close(stats_ops.coldot(d, x), d @ x.float(), rtol=1e-4, atol=1e-3)
        r = stats_ops.rowdot(x, w, 0.5, 0)                       # + bias, sigmoid
        torch.testing.assert_close(r, torch.sigmoid(x.float() @ w + 0.5), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("act", ["tanh", "sigmoid", "relu"])
def test_sensitivity_kernel_matches_torch(act):
    from shifu_amd.algos import varsel as V
    from shifu_amd.formats.nn_format import NNNetwork
    rng = np.random.default_rng(0)
    F, H = 40, 24
    net = NNNetwork([F, H, 1], [act, "sigmoid"], [rng.normal(size=(H, F + 1)) * 0.3, rng.normal(size=(1, H + 1))])
    X = rng.normal(size=(3000, F)).astype(np.float32)
    m1, r1, _ = V.sensitivity(net, X, device=torch.device("cpu"))
    m2, r2, _ = V.sensitivity(net, X, device=torch.device("cuda"))
    np.testing.assert_allclose(m2, m1, rtol=2e-4, atol=1e-6)
    np.testing.assert_allclose(r2, r1, rtol=2e-4, atol=1e-6)


@pytest.mark.parametrize("acts", [("sigmoid", "tanh", "sigmoid"), ("relu", "sigmoid", "sigmoid"),
                                  ("tanh", "relu", "tanh", "sigmoid")])
def test_deep_sensitivity_mfma_tail_matches_torch(acts):
    """K14b (perturbed first layer as bf16 rows + MFMA GEMM tail) vs the fp32 torch oracle for 2-
    and 3-hidden-layer nets: per-input SE within bf16 accuracy, same top inputs."""
    from shifu_amd.algos import varsel as V
    from shifu_amd.formats.nn_format import NNNetwork
    rng = np.random.default_rng(1)
    F = 50
    sizes = [F] + [48, 24, 16][: len(acts) - 1] + [1]
    Ws = [rng.normal(size=(sizes[i + 1], sizes[i] + 1)) * (0.8 / np.sqrt(sizes[i])) for i in range(len(sizes) - 1)]
    Ws[0][:, :8] *= 4.0                                    # a few strongly used inputs
    net = NNNetwork(sizes, list(acts), Ws)
    X = rng.normal(size=(4000, F)).astype(np.float32)
    m1, r1, _ = V.sensitivity(net, X, device=torch.device("cpu"))
    m2, r2, _ = V.sensitivity(net, X, device=torch.device("cuda"), deep_rows=1024, feat_chunk=16)
    np.testing.assert_allclose(r2, r1, rtol=3e-2, atol=2e-3 * r1.max())
    np.testing.assert_allclose(m2, m1, rtol=3e-2, atol=1e-2 * m1.max())   # |d| keeps bf16 noise
    assert set(np.argsort(-r1)[:8]) == set(np.argsort(-r2)[:8])


def test_sensitivity_host_rows_stream_equals_resident():
    """SE over HostRows (pinned staging + H2D on a copy stream overlapping the kernels) equals SE
    over the same rows resident on the device (rows rounded to bf16, the staging precision)."""
    from shifu_amd.algos import varsel as V
    from shifu_amd.formats.nn_format import NNNetwork
    from shifu_amd.models.nn import HostRows
    rng = np.random.default_rng(2)
    F, H = 64, 32
    net = NNNetwork([F, H, 1], ["sigmoid", "sigmoid"], [rng.normal(size=(H, F + 1)) * 0.3,
                                                        rng.normal(size=(1, H + 1))])
    X = torch.from_numpy(rng.normal(size=(20000, F)).astype(np.float32)).to(torch.bfloat16).float().numpy()
    m1, r1, _ = V.sensitivity(net, torch.from_numpy(X).cuda(), device=torch.device("cuda"), row_chunk=256)
    m2, r2, _ = V.sensitivity(net, HostRows(X, F), device=torch.device("cuda"), row_chunk=256)
    np.testing.assert_allclose(r2, r1, rtol=1e-6)
    np.testing.assert_allclose(m2, m1, rtol=1e-6)


def test_sensitivity_stream_equals_resident_wide():
    """the streamed SE path at the bench's width class (F = 4096 inputs, H = 500)
    equals the resident one, and a sparse planted dependence is ranked on top by both."""
    from shifu_amd.algos import varsel as V
    from shifu_amd.formats.nn_format import NNNetwork
    from shifu_amd.models.nn import HostRows
    rng = np.random.default_rng(5)
    F, H, n = 4096, 500, 8192
    W1 = rng.normal(size=(H, F + 1)) * (0.5 / np.sqrt(F))
    strong = np.arange(0, F, F // 16)[:16]
    W1[:, strong] *= 40.0
    net = NNNetwork([F, H, 1], ["sigmoid", "sigmoid"], [W1, rng.normal(size=(1, H + 1)) * 0.3])
    X = torch.from_numpy(rng.normal(size=(n, F)).astype(np.float32)).to(torch.bfloat16).float().numpy()
    m1, r1, _ = V.sensitivity(net, torch.from_numpy(X).cuda(), device=torch.device("cuda"), row_chunk=1024)
    m2, r2, _ = V.sensitivity(net, HostRows(X, F), device=torch.device("cuda"), row_chunk=1024)
    np.testing.assert_allclose(r2, r1, rtol=1e-6)
    np.testing.assert_allclose(m2, m1, rtol=1e-6)
    assert set(np.argsort(-r1)[:16]) == set(strong.tolist())
    assert np.unique(r1).size > F // 2                  # not a degenerate (all-tied) result


@pytest.mark.gpu
def test_column_metrics_kernel_matches_host():
    """K3: KS / IV / WOE / per-bin WOE of many columns in one launch == the host
    ColumnStatsCalculator oracle (incl. > 64 bins: chunk carry of the cumulative sums, and
    columns with no positives)."""
    import numpy as np
    from shifu_amd.algos.stats import column_metrics
    from shifu_amd.ops.stats_ops import column_metrics_batch
    rng = np.random.default_rng(4)
    negs, poss = [], []
    for k, nb in enumerate([3, 11, 64, 65, 200, 1, 10]):
        cn, cp = rng.integers(0, 50, nb).astype(float), rng.integers(0, 50, nb).astype(float)
        if k == 5:
            cp[:] = 0
        negs.append((cn, cn * rng.random(nb)))
        poss.append((cp, cp * rng.random(nb)))
    got = column_metrics_batch(negs, poss, "cuda")
    for k in range(len(negs)):
        for v in range(2):
            ref = column_metrics(negs[k][v], poss[k][v])
            g = got[k][v]
            if ref is None:
                assert g is None
                continue
            np.testing.assert_allclose(g[:3], ref[:3], rtol=1e-12, atol=1e-12)
            np.testing.assert_allclose(g[3], ref[3], rtol=1e-12, atol=1e-12)


def test_se_first_layer_split_bf16_gemm_fp32_accurate():
    """The SE cached first layer S = X W1^T + b1 on the own MFMA GEMM (split-bf16 operands, EPI_F32
    tile) is fp32-accurate: within ~1e-5 of the fp64 product (a plain bf16 GEMM is ~1e-2 off)."""
    from shifu_amd.algos import varsel as V
    rng = np.random.default_rng(7)
    F, H = 333, 50
    W = rng.normal(size=(H, F + 1)) * 0.2
    X = rng.normal(size=(5000, F)).astype(np.float32)
    Wt = torch.tensor(W, dtype=torch.float32, device="cuda")
    S = V.first_layer_fp32(torch.from_numpy(X).cuda(), Wt[:, :F], Wt[:, F]).double().cpu().numpy()
    ref = X.astype(np.float64) @ W[:, :F].astype(np.float32).astype(np.float64).T + \
        W[:, F].astype(np.float32).astype(np.float64)
    err = np.abs(S - ref).max() / np.abs(ref).max()
    assert err < 2e-5, err
