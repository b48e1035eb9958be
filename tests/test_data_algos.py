"""Data reading / purifying / expressions and the stats, normalize, varsel algorithms
(parity model: DataPurifierTest, JexlTest, BinningTest, NormalizerTest, VariableSelectorTest)."""
import os

import numpy as np
import pytest

from shifu_amd.algos import binning as B
from shifu_amd.algos import normalize as N
from shifu_amd.algos import varsel as V
from shifu_amd.algos.stats import column_metrics, compute_column_stats, pearson_correlation
from shifu_amd.config.column_config import load_column_configs
from shifu_amd.config.model_config import ModelConfig
from shifu_amd.data import reader as R
from shifu_amd.data.expr import Evaluator
from shifu_amd.data.purifier import load_dataset

CJ = "example/cancer-judgement"


@pytest.fixture
def cancer(ref_resources):
    root = os.path.join(ref_resources, CJ)
    mc = ModelConfig.load(os.path.join(root, "ModelStore/ModelSet1/ModelConfig.json"))
    mc.dataSet["dataPath"] = os.path.join(root, "DataStore/DataSet1")
    mc.dataSet["headerPath"] = os.path.join(root, "DataStore/DataSet1/.pig_header")
    ccs = load_column_configs(os.path.join(root, "ModelStore/ModelSet1/ColumnConfig.json"))
    return mc, ccs


def test_native_and_python_parsers_agree(tmp_path):
    rows = ["a|1.5|x", "b||y", "a|?|", "c|3|x", "d|-2e3|z|extra"]
    (tmp_path / "part-0").write_text("\n".join(rows) + "\n")
    hdr = ["s", "n", "t"]
    t = R.read_table(str(tmp_path), hdr, "|", numeric=["n"], strings=["s", "t"])
    data = (tmp_path / "part-0").read_bytes()
    n, bad, py = R._parse_python(data, "|", [2, 1, 2], ["", "?"])
    assert t.n == n == 5
    np.testing.assert_array_equal(np.isnan(t["n"].values), np.isnan(py[1][1]))
    assert t["s"].strings().tolist() == ["a", "b", "a", "c", "d"]
    assert t["n"].values[0] == 1.5 and t["n"].values[4] == -2000.0
    assert t["t"].missing_mask().tolist() == [False, False, True, False, False]


def test_native_parser_numeric_missing_token(tmp_path):
    """A missing token that is itself a decimal ("-999", "0") must read as missing on the native
    parser's inline numeric fast path too (UpdateBinningInfoMapper checks missingOrInvalidValues
    before parsing); "-999.0" is a different token and stays a number."""
    rows = ["-999|1", "-999.0|0", "5|-999", "0|2.5", "-999|"]
    (tmp_path / "part-0").write_text("\n".join(rows) + "\n")
    miss = ["", "?", "-999", "0"]
    t = R.read_table(str(tmp_path), ["a", "b"], "|", numeric=["a", "b"], missing=miss)
    data = (tmp_path / "part-0").read_bytes()
    n, bad, py = R._parse_python(data, "|", [1, 1], miss)
    assert t.n == n == 5
    for ci, c in enumerate(["a", "b"]):
        np.testing.assert_array_equal(t[c].values, py[ci][1])
    assert np.isnan(t["a"].values[[0, 3, 4]]).all() and t["a"].values[1] == -999.0
    assert np.isnan(t["b"].values[[1, 2, 4]]).all() and t["b"].values[3] == 2.5


def test_native_parser_simd_fast_path_randomized():
    """The SSE field parser (<= 16-byte fields in one load + table shuffle + madd) and the scalar
    fallbacks give the python parser's values bit for bit: signs, leading zeros, "12." / "-.5",
    15- and 16-digit fields, exponents, Java "1.0d", padded fields, numeric missing tokens."""
    import random
    rng = random.Random(1)
    toks = ["", "?", "-999", "0", "1.5", "-0.000", "+12.25", "007.50", "12.", "-.5", ".", "-", "1e5", "1.0d",
            "123456789012345", "1234567890123456", "12345678901234567890", "0.1234567890123456789", "3.14159",
            " 4.5", "4.5 ", "99999999999999.9", "-0.00001", "1.", "00000000000000001", "-999999999999999."]
    rows = ["|".join(rng.choice(toks) if rng.random() < 0.7 else f"{rng.gauss(0, 100):.{rng.randint(0, 12)}f}"
                     for _ in range(23)) for _ in range(3000)]
    data = ("\n".join(rows) + "\n").encode()
    for miss in (["", "?"], ["", "?", "-999", "0"]):
        n, bad, py = R._parse_python(data, "|", [1] * 23, miss)
        nat = R._parse_native(bytearray(data), "|", [1] * 23, miss, 4)
        if nat is None:
            pytest.skip("native runtime not built")
        for c in range(23):
            np.testing.assert_array_equal(nat[2][c][1], py[c][1], err_msg=f"column {c} missing {miss}")


def test_native_parser_skipped_column_runs_randomized():
    """Runs of unparsed columns are jumped with the 16-byte delimiter count (nth_delim): random
    column subsets over ragged rows (short, long, blank, long fields > 16 bytes) give the same
    values, string codes and bad-row count as the python parser."""
    import random
    rng = random.Random(7)
    C = 41
    toks = ["", "1.5", "-2", "abc", "x" * 40, "3.25", "?", "1e3", " 7 "]
    rows = []
    for _ in range(2000):
        k = C + rng.choice([0, 0, 0, 0, -1, -7, 3, -C + 1])
        rows.append("|".join(rng.choice(toks) for _ in range(max(k, 1))))
        if rng.random() < 0.02:
            rows.append("  \t")
    data = ("\n".join(rows) + "\n").encode()
    for trial in range(12):
        kinds = [rng.choice([0, 0, 0, 1, 2]) for _ in range(C)]
        if trial == 0:
            kinds = [0] * C
            kinds[rng.randrange(C)] = 1
        n, bad, py = R._parse_python(data, "|", kinds, ["", "?"])
        nat = R._parse_native(bytearray(data), "|", kinds, ["", "?"], 3)
        if nat is None:
            pytest.skip("native runtime not built")
        assert nat[0] == n and nat[1] == bad, (trial, nat[:2], n, bad)
        for c, k in enumerate(kinds):
            if k == 1:
                np.testing.assert_array_equal(nat[2][c][1], py[c][1], err_msg=f"trial {trial} column {c}")
            elif k == 2:
                a = np.array(nat[2][c][2] + [None], dtype=object)[nat[2][c][1]]
                b = np.array(py[c][2] + [None], dtype=object)[py[c][1]]
                assert list(a) == list(b), (trial, c)


def test_expression_evaluator():
    from shifu_amd.data.reader import Column, RawTable
    cols = {"a": Column("a", "num", np.array([1.0, 2.0, np.nan, 4.0])),
            "s": Column("s", "str", np.array([0, 1, -1, 0], np.int32), ["x", "yy"])}
    t = RawTable(["a", "s"], cols, 4, 0)
    assert Evaluator("a > 1.5 && s == 'x'").mask(t).tolist() == [False, False, False, True]
    assert Evaluator("a * 2 + 1").values(t)[:2].tolist() == [3.0, 5.0]
    assert Evaluator("s != 'yy'").mask(t).tolist()[1] is False
    assert set(Evaluator("a > 1 || b < 2").columns()) == {"a", "b"}


def test_load_and_purify_cancer(cancer):
    mc, ccs = cancer
    nums = [c.name for c in ccs if not c.is_target() and not c.is_categorical()]
    md = load_dataset(mc, mc.dataSet, columns_num=nums)
    assert md.n == 429
    assert md.counters.pos + md.counters.neg == md.n
    assert set(np.unique(md.y)) <= {0.0, 1.0}


def test_equal_population_binning():
    rng = np.random.default_rng(0)
    v = rng.normal(size=10000)
    b = B.equal_population_boundaries(v, 10)
    assert b[0] == float("-inf") and len(b) == 10 and all(x < y for x, y in zip(b, b[1:]))
    idx = B.bin_index_numeric(v, b)
    counts = np.bincount(idx, minlength=10)
    assert counts.min() > 900 and counts.max() < 1100
    idx2 = B.bin_index_numeric(np.array([np.nan, -np.inf, np.inf]), b)
    assert idx2.tolist() == [10, 0, 9]


def test_column_metrics_ks_iv():
    neg, pos = np.array([40., 30., 20., 10.]), np.array([10., 20., 30., 40.])
    ks, iv, woe, bw = column_metrics(neg, pos)
    assert abs(ks - 40.0) < 1e-9
    p, n = pos / pos.sum(), neg / neg.sum()
    assert abs(iv - ((n - p) * np.log((n + 1e-10) / (p + 1e-10))).sum()) < 1e-12


def test_stats_and_normalize_cancer(cancer):
    mc, ccs = cancer
    nums = [c.name for c in ccs if not c.is_target() and not c.is_categorical()]
    md = load_dataset(mc, mc.dataSet, columns_num=nums)
    compute_column_stats(mc, ccs, md)
    c = next(c for c in ccs if c.name == "column_5")
    assert c.ks > 50 and c.iv > 5              # strongly predictive in this data set
    assert sum(c.bin_count_pos) == md.counters.pos or mc.binning_method != "EqualTotal"
    v = md.table["column_5"].numeric()
    assert abs(c.mean - np.nanmean(v)) < 1e-9 * abs(c.mean)
    for cc in ccs:
        if not cc.is_target():
            cc.final_select = True
    X, names, _ = N.normalize_table(mc, ccs, md.table, norm_type="ZSCALE")
    assert X.shape == (md.n, len(nums))
    j = names.index("column_5")
    cut = float(mc.normalize.get("stdDevCutOff", 6.0))
    ref = np.clip(v, c.mean - cut * c.std_dev, c.mean + cut * c.std_dev)
    np.testing.assert_allclose(X[:, j], (ref - c.mean) / c.std_dev, rtol=1e-5, atol=1e-6)
    Xw, _, _ = N.normalize_table(mc, ccs, md.table, norm_type="WOE")
    assert np.isin(np.round(Xw[:, j], 5), np.round(np.asarray(c.bin_count_woe, np.float32), 5)).all()
    C, nb, is_cat = N.tree_bin_codes(ccs, md.table, [cc for cc in ccs if not cc.is_target()])
    assert C.max() < nb.max() and (C >= 0).all()
    # WOE_ZSCALE_INDEX on a numeric column = z-scored WOE (Normalizer.fullNormalize :305-315)
    Xz, _, _ = N.normalize_table(mc, ccs, md.table, norm_type="WOE_ZSCALE_INDEX")
    Xwz, _, _ = N.normalize_table(mc, ccs, md.table, norm_type="WOE_ZSCALE")
    np.testing.assert_allclose(Xz[:, j], Xwz[:, j], rtol=1e-6)
    m, sd = N.woe_mean_std(c, False)
    np.testing.assert_allclose(Xz[:, j], N.zscore(Xw[:, j].astype(np.float64), m, sd, cut), rtol=1e-5, atol=1e-6)


def test_varsel_filter_ks_iv_mix(cancer):
    mc, ccs = cancer
    mc.varSelect["filterNum"] = 5
    for key in ("KS", "IV", "mix", "pareto"):
        mc.varSelect["filterBy"] = key
        V.select_by_filter(mc, ccs)
        sel = [c for c in ccs if c.final_select]
        assert len(sel) == 5, key
        if key == "KS":
            top = sorted([c for c in ccs if not c.is_target() and c.ks is not None], key=lambda c: -c.ks)[:5]
            assert {c.name for c in sel} == {c.name for c in top}


def test_pareto_epsilon_archive():
    """VariableSelector.Archives.sortInto semantics: epsilon boxes floor(ks/0.01), floor(iv/0.05);
    the smaller box dominates (the reference archive minimizes), mutually non-dominated boxes both
    stay, same box -> the tuple nearer the box corner stays."""
    pts = [(0, 1.0, 1.0), (1, 2.0, 0.5), (2, 0.5, 0.5), (3, 3.0, 3.0)]
    assert [p[0] for p in V.pareto_sort(pts)] == [2]
    assert [p[0] for p in V.pareto_sort([(0, 1.0, 1.0), (1, 2.0, 0.5)])] == [0, 1]
    # same box (eps 1.0): 0.1 is nearer the corner 0.0 than 0.9
    assert [p[0] for p in V.pareto_sort([(0, 0.9, 0.9), (1, 0.1, 0.1)], [1.0, 1.0])] == [1]


def test_pearson_pairwise_complete():
    rng = np.random.default_rng(0)
    X = rng.normal(size=(200, 3))
    X[:, 1] = X[:, 0] * 2 + rng.normal(size=200) * 0.1
    X[5, 0] = np.nan
    C = pearson_correlation(X)
    ok = np.isfinite(X[:, 0])
    ref = np.corrcoef(X[ok][:, 0], X[ok][:, 1])[0, 1]
    assert abs(C[0, 1] - ref) < 1e-9
    assert abs(C[2, 2] - 1.0) < 1e-9


def test_sensitivity_matches_bruteforce():
    from shifu_amd.formats.nn_format import NNNetwork
    rng = np.random.default_rng(0)
    net = NNNetwork([6, 5, 1], ["tanh", "sigmoid"], [rng.normal(size=(5, 7)), rng.normal(size=(1, 6))])
    X = rng.normal(size=(50, 6)).astype(np.float32)
    mean, rms, _ = V.sensitivity(net, X, feat_chunk=4, row_chunk=16)
    base = net.forward(X)[:, 0]
    for i in range(6):
        Z = X.astype(np.float64).copy()
        Z[:, i] = 0
        d = base - net.forward(Z)[:, 0]
        assert abs(np.abs(d).mean() - mean[i]) < 1e-5
        assert abs(np.sqrt((d * d).mean()) - rms[i]) < 1e-5


def test_parquet_input_matches_csv(tmp_path):
    import pyarrow as pa
    import pyarrow.parquet as pq
    rows = [("a", 1.5, "x"), ("b", None, "y"), ("a", 3.0, None), ("c", -2.0, "x")]
    (tmp_path / "csv").mkdir()
    (tmp_path / "csv" / "part-0").write_text("\n".join(f"{s}|{'' if n is None else n}|{'' if t is None else t}"
                                                       for s, n, t in rows) + "\n")
    (tmp_path / "pq").mkdir()
    pq.write_table(pa.table({"s": [r[0] for r in rows], "n": [r[1] for r in rows], "t": [r[2] for r in rows]}),
                   str(tmp_path / "pq" / "part-0.parquet"))
    hdr = R.read_header(None, "|", str(tmp_path / "pq"))
    assert hdr == ["s", "n", "t"]
    a = R.read_table(str(tmp_path / "csv"), hdr, "|", numeric=["n"], strings=["s", "t"])
    b = R.read_table(str(tmp_path / "pq"), hdr, "|", numeric=["n"], strings=["s", "t"])
    np.testing.assert_array_equal(a["n"].values, b["n"].values)
    assert a["s"].strings().tolist() == b["s"].strings().tolist()
    assert a["t"].missing_mask().tolist() == b["t"].missing_mask().tolist()


def test_pearson_chunked_equals_whole():
    rng = np.random.default_rng(3)
    X = rng.normal(size=(301, 5))
    X[:, 2] += X[:, 0]
    X[rng.random(X.shape) < 0.1] = np.nan
    np.testing.assert_allclose(pearson_correlation(X, chunk_rows=7), pearson_correlation(X), rtol=1e-12,
                               atol=1e-14)
    parts = [X[:100], X[100:250], X[250:]]
    np.testing.assert_allclose(pearson_correlation(iter(parts), chunk_rows=64), pearson_correlation(X),
                               rtol=1e-12, atol=1e-14)


def test_spdt_sketch_matches_reference_small_bin_rule():
    """EqualPopulationBinningTest.testExtraSmallBins: 60 outliers next to 2 x 100000 values are
    folded into a neighbour (< 0.3% of an average bin) -> 2 cut points; 61 -> 3."""
    from shifu_amd.algos import binning as B
    for n_out, want in ((60, 2), (61, 3)):
        v = np.concatenate([np.full(100000, 5.0), np.full(100000, 8.0), np.full(n_out, -10.0)])
        assert len(B.sketch_boundaries(v, 10, "SPDT")) == want


def test_sketch_cuts_track_exact_quantiles():
    from shifu_amd.algos import binning as B
    rng = np.random.default_rng(0)
    v = rng.normal(size=50000)
    exact = np.array(B.equal_population_boundaries(v, 10)[1:])
    spdt = np.array(B.sketch_boundaries(v, 10, "SPDTI")[1:])
    mp = B.sketch_boundaries(v, 10, "MunroPat")
    assert spdt.size == exact.size and np.abs(spdt - exact).max() < 0.02
    # MunroPat: min + 8 interior quantiles + max -> -inf + 8 cuts (MunroPatBinning.binMerge)
    assert mp[0] == -np.inf and len(mp) == 9
    # the alternate-element collapse (lower element of each pair) biases the estimate low by a
    # rank of ~1-3 %: compare ranks, not values
    ranks = np.searchsorted(np.sort(v), np.array(mp[1:])) / v.size
    assert np.abs(ranks - np.arange(1, 9) / 9).max() < 0.04
    with_nan = np.concatenate([v, [np.nan] * 100])
    assert B.sketch_boundaries(with_nan, 10, "SPDT") == B.sketch_boundaries(v, 10, "SPDT")


def test_stats_binning_parity_mode(tmp_path, monkeypatch):
    import json
    import os
    from shifu_amd.config import environment
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.steps.create import run_init
    from shifu_amd.steps.stats import run_stats
    from shifu_amd.utils.synthetic import make_model_set
    from shifu_amd.algos import binning as B
    from shifu_amd.data.purifier import load_dataset
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    root = make_model_set(str(tmp_path), "p", "NN", n_rows=3000, n_num=4, n_cat=1)
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    mc.stats["binningAlgorithm"] = "SPDTI"
    mc.save()
    run_init(root)
    monkeypatch.setitem(environment.props(), "shifu.stats.binning.parity", "true")
    run_stats(root)
    ccs = json.load(open(os.path.join(root, "ColumnConfig.json")))
    c = next(x for x in ccs if x["columnName"] == "num_0")
    md = load_dataset(ModelConfig.load(os.path.join(root, "ModelConfig.json")),
                      ModelConfig.load(os.path.join(root, "ModelConfig.json")).dataSet, ["num_0"], [])
    want = B.sketch_boundaries(md.table["num_0"].numeric(), 10, "SPDTI")
    assert c["columnBinning"]["binBoundary"][1:] == want[1:] and len(want) > 5
