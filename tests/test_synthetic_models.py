"""Pipelines over generated model sets on the CPU: WDL, multi-class (NATIVE / ONEVSALL),
auto-type init, stats -rebin, PSI."""
import json
import os

import numpy as np
import pytest


@pytest.fixture(autouse=True)
def _cpu(monkeypatch):
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")


def _run(root, steps):
    from shifu_amd.cli import main
    cwd = os.getcwd()
    os.chdir(root)
    try:
        for s in steps:
            assert main(s.split()) == 0, s
    finally:
        os.chdir(cwd)


def _mc(root):
    from shifu_amd.config.model_config import ModelConfig
    return ModelConfig.load(os.path.join(root, "ModelConfig.json"))


def test_wdl_pipeline(tmp_path):
    from shifu_amd.utils.synthetic import make_model_set
    root = make_model_set(str(tmp_path), "w", "WDL", n_rows=1500)
    mc = _mc(root)
    mc.train["numTrainEpochs"] = 60
    mc.train["baggingNum"] = 1
    mc.train["params"] = {"NumHiddenLayers": 1, "NumHiddenNodes": [16], "ActivationFunc": ["relu"],
                          "LearningRate": 0.01, "NumEmbedOuputs": 4, "WDLL2Reg": 0.0}
    mc.save()
    _run(root, ["init", "stats", "varsel", "norm", "train", "eval"])
    assert os.path.exists(os.path.join(root, "models/model0.wdl"))
    auc = json.load(open(os.path.join(root, "evals/Eval1/EvalPerformance.json")))["areaUnderRoc"]
    assert auc > 0.8
    # reference BinaryWDLSerializer layout: gzip, version 1, reserved fields, norm type, column stats
    import gzip
    import struct
    raw = gzip.open(os.path.join(root, "models/model0.wdl")).read()
    assert struct.unpack(">i", raw[:4])[0] == 1
    assert raw[4:20] == b"\0" * 16 and raw[20:22] == struct.pack(">h", 14) and raw[22:36] == b"Reserved field"
    # read back -> identical scores
    import torch
    from shifu_amd.formats.wdl_format import read_wdl_file
    from shifu_amd.models.wdl import read_wdl, write_wdl
    m = read_wdl(os.path.join(root, "models/model0.wdl"))
    _, norm, stats, spec = read_wdl_file(os.path.join(root, "models/model0.wdl"))
    assert spec.hidden == [16] and spec.acts == ["relu"] and spec.n_dense == len(spec.dense_ids)
    assert {cs.column_num for cs in stats} >= set(spec.dense_ids + spec.wide_ids)
    p2 = os.path.join(str(tmp_path), "again.wdl")
    write_wdl(p2, m)
    m2 = read_wdl(p2)
    for a, b in zip(m.net.parameters(), m2.net.parameters()):
        torch.testing.assert_close(a, b)
    assert m2.columns == m.columns


@pytest.mark.parametrize("method", ["NATIVE", "ONEVSALL"])
def test_multiclass_nn(tmp_path, method):
    from shifu_amd.utils.synthetic import make_model_set
    root = make_model_set(str(tmp_path), "mc", "NN", n_rows=1500, n_classes=3)
    mc = _mc(root)
    assert mc.is_multiclass()
    mc.train["numTrainEpochs"] = 40
    mc.train["multiClassifyMethod"] = method
    mc.save()
    _run(root, ["init", "stats", "varsel", "norm", "train", "eval"])
    perf = json.load(open(os.path.join(root, "evals/Eval1/EvalPerformance.json")))
    assert perf["accuracy"] > 0.55        # 3 balanced classes: chance = 0.33
    n_models = len(os.listdir(os.path.join(root, "models")))
    assert n_models == (3 if method == "ONEVSALL" else 1 * int(mc.train.get("baggingNum", 5)))


def test_autotype_rebin_psi(tmp_path, monkeypatch):
    """autoTypeThreshold with the documented ratio rule (the reference rule as written types a
    column categorical only when a sampled item is blank: tests/test_autotype_stream.py)."""
    from shifu_amd.config import environment
    from shifu_amd.utils.synthetic import make_model_set
    monkeypatch.setitem(environment.props(), "shifu.autoType.rule", "ratio")
    root = make_model_set(str(tmp_path), "a", "NN", n_rows=1200)
    mc = _mc(root)
    mc.dataSet["autoType"] = True
    mc.dataSet["autoTypeThreshold"] = 90
    mc.stats["psiColumnName"] = "cat_0"
    mc.stats["maxNumBin"] = 20
    mc.save()
    with open(os.path.join(root, "columns", "categorical.column.names"), "w") as f:
        f.write("")
    _run(root, ["init"])
    ccs = json.load(open(os.path.join(root, "ColumnConfig.json")))
    types = {c["columnName"]: c["columnType"] for c in ccs}
    assert types["cat_1"] == "C" and types["num_3"] == "N"
    _run(root, ["stats"])
    ccs = json.load(open(os.path.join(root, "ColumnConfig.json")))
    num3 = [c for c in ccs if c["columnName"] == "num_3"][0]
    assert num3["columnStats"]["psi"] is not None
    nb = len(num3["columnBinning"]["binBoundary"])
    _run(root, ["stats -rebin -n 5"])
    ccs = json.load(open(os.path.join(root, "ColumnConfig.json")))
    num3 = [c for c in ccs if c["columnName"] == "num_3"][0]
    assert nb > 5 and len(num3["columnBinning"]["binBoundary"]) == 5
    assert np.isclose(sum(num3["columnBinning"]["binCountPos"]) + sum(num3["columnBinning"]["binCountNeg"]),
                      1200 - 0, rtol=0.05)


@pytest.mark.parametrize("alg", ["NN", "GBT"])
def test_fault_injection_and_resume(tmp_path, alg):
    """SHIFU_FAULT_AT_ITER kills the trainer right after a checkpoint; re-running resumes and
    produces the same model as an uninterrupted run."""
    import subprocess
    import sys
    from shifu_amd.utils.synthetic import make_model_set
    roots = []
    for name in ("a", "b"):
        root = make_model_set(str(tmp_path), name, alg, n_rows=600)
        mc = _mc(root)
        mc.train["numTrainEpochs"] = 12
        mc.train["baggingNum"] = 1
        if alg == "GBT":
            mc.train["params"].update({"TreeNum": 12, "MaxDepth": 3, "CheckpointInterval": 4})
        else:
            mc.train["params"]["CheckpointInterval"] = 4
        mc.save()
        _run(root, ["init", "stats", "norm"])
        roots.append(root)
    env = dict(os.environ, SHIFU_FORCE_CPU="1", SHIFU_FAULT_AT_ITER="8", PYTHONPATH=os.getcwd())
    r = subprocess.run([sys.executable, "-m", "shifu_amd.cli", "train"], cwd=roots[0], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 17, r.stderr[-2000:]
    assert os.path.exists(os.path.join(roots[0], "tmp/checkpoints"))
    _run(roots[0], ["train"])                  # resumes from the iteration-8 checkpoint
    _run(roots[1], ["train"])                  # uninterrupted reference
    ext = "nn" if alg == "NN" else "gbt"
    if alg == "NN":
        from shifu_amd.formats.nn_format import read_encog
        wa = read_encog(os.path.join(roots[0], f"models/model0.{ext}")).weights
        wb = read_encog(os.path.join(roots[1], f"models/model0.{ext}")).weights
        for x, y in zip(wa, wb):
            np.testing.assert_allclose(x, y, rtol=1e-5, atol=1e-6)
    else:
        from shifu_amd.formats.tree_format import read_tree_model
        ta, tb = read_tree_model(os.path.join(roots[0], "models/model0.gbt")), \
            read_tree_model(os.path.join(roots[1], "models/model0.gbt"))
        assert len(ta.bags[0]) == len(tb.bags[0]) == 12
        x = {c: np.linspace(-3, 3, 50) for c in ta.names}
        np.testing.assert_allclose(ta.score(x, 50), tb.score(x, 50), rtol=1e-5)


def test_nn_dropout_minibatch_subset_fixedbias(tmp_path):
    from shifu_amd.utils.synthetic import make_model_set
    root = make_model_set(str(tmp_path), "d", "NN", n_rows=1500)
    mc = _mc(root)
    mc.train["numTrainEpochs"] = 40
    mc.train["baggingNum"] = 2
    mc.train["params"].update({"DropoutRate": 0.2, "MiniBatchs": 3, "FeatureSubsetStrategy": "HALF",
                               "FixedBias": True, "NumHiddenNodes": [20]})
    mc.save()
    _run(root, ["init", "stats", "norm", "train", "eval"])
    from shifu_amd.formats.nn_format import read_encog, read_binary_nn
    net = read_encog(os.path.join(root, "models/model0.nn"))
    sub = net.input_subset()
    assert sub is not None and len(sub) == net.n_in
    assert read_binary_nn(os.path.join(root, "bmodels/model0.nn"))["networks"][0].input_subset() == sub
    auc = json.load(open(os.path.join(root, "evals/Eval1/EvalPerformance.json")))["areaUnderRoc"]
    assert auc > 0.7


def test_dropout_gradient_matches_masked_network():
    """Dropout = zeroing dropped inputs/hidden outputs and scaling kept ones by 1/(1-rate)."""
    import torch
    from shifu_amd.models.nn import MLPSpec, MLPTrainer
    torch.manual_seed(0)
    spec = MLPSpec(6, [5], ["tanh"], 1, "sigmoid")
    tr = MLPTrainer(spec, "cpu", "R", 0.1, seed=1, dropout_rate=0.5)
    x, y = torch.randn(40, 6), (torch.rand(40, 1) > 0.5).float()
    d = tr.prepare(x, y)
    g = tr.compute_gradients(d)[: tr.params.numel].clone()
    scale = tr._scale
    # reference: autograd on explicitly scaled weights == masked activations
    W = [w.clone().requires_grad_(True) for w in tr.params.views()]
    sv = tr.params.views(scale)
    a = d.x.float()
    h = torch.tanh(a @ (W[0] * sv[0]).t())
    hp = torch.cat([h, torch.ones(40, 1), torch.zeros(40, spec.layer_kpad[1] - 6)], 1)
    p = torch.sigmoid(hp @ (W[1] * sv[1]).t())
    # ascent direction with Encog flat spots is checked in test_nn_cpu; here compare the sign pattern
    # and the zero pattern of the gradient (dropped connections get exactly zero)
    gv = tr.params.views(g)
    for l in range(2):
        zero_cols = (sv[l] == 0)
        assert torch.all(gv[l][zero_cols] == 0)


def test_segment_expansion_pipeline(tmp_path):
    from shifu_amd.utils.synthetic import make_model_set
    root = make_model_set(str(tmp_path), "s", "NN", n_rows=1500)
    with open(os.path.join(root, "columns", "segments.txt"), "w") as f:
        f.write("cat_0 == 'k1'\nnum_0 > 0\n")
    mc = _mc(root)
    mc.dataSet["segExpressionFile"] = "columns/segments.txt"
    mc.train["numTrainEpochs"] = 20
    mc.train["baggingNum"] = 1
    mc.varSelect["filterNum"] = 30
    mc.save()
    _run(root, ["init", "stats"])
    ccs = json.load(open(os.path.join(root, "ColumnConfig.json")))
    n = len(ccs) // 3
    assert len(ccs) == 3 * n
    byname = {c["columnName"]: c for c in ccs}
    assert byname["diagnosis_1"]["columnFlag"] == "ForceRemove" and byname["id_2"]["columnFlag"] == "Meta"
    assert byname["num_3_2"]["columnNum"] == 2 * n + byname["num_3"]["columnNum"]
    # segment 2 (num_0 > 0) keeps about half the rows; the rest are missing in the copy
    miss = byname["num_3_2"]["columnStats"]["missingCount"] - byname["num_3"]["columnStats"]["missingCount"]
    assert 0.35 * 1500 < miss < 0.65 * 1500
    assert byname["cat_0_1"]["columnBinning"]["binCategory"] == ["k1"]
    _run(root, ["varsel", "norm", "train", "eval"])
    auc = json.load(open(os.path.join(root, "evals/Eval1/EvalPerformance.json")))["areaUnderRoc"]
    assert auc > 0.7


def test_gbt_continuous_training(tmp_path):
    """isContinuous for GBT (TrainModelProcessor.checkContinuousTraining / DTMaster :1081-1104):
    3 trees, then TreeNum 6 continues from the stored model (existing trees kept, predictions
    replayed) and equals 6 trees trained straight; a changed loss restarts from scratch; an
    existing model with >= TreeNum trees leaves the trainer untouched."""
    from shifu_amd.formats.tree_format import read_tree_model
    from shifu_amd.utils.synthetic import make_model_set
    roots = []
    for name in ("a", "b"):
        root = make_model_set(str(tmp_path), name, "GBT", n_rows=800)
        mc = _mc(root)
        mc.train["baggingNum"] = 1
        mc.train["validSetRate"] = 0.0
        mc.train["params"].update({"TreeNum": 3 if name == "a" else 6, "MaxDepth": 3,
                                   "FeatureSubsetStrategy": "ALL", "LearningRate": 0.2})
        mc.save()
        _run(root, ["init", "stats", "norm", "train"])
        roots.append(root)
    a, b = roots
    mpath = os.path.join(a, "models/model0.gbt")
    first = read_tree_model(mpath)
    assert len(first.bags[0]) == 3
    mc = _mc(a)
    mc.train["isContinuous"] = True
    mc.train["params"]["TreeNum"] = 6
    mc.save()
    _run(a, ["train"])
    cont, straight = read_tree_model(mpath), read_tree_model(os.path.join(b, "models/model0.gbt"))
    assert len(cont.bags[0]) == 6
    x = {c: np.linspace(-3, 3, 64) for c in cont.names}
    np.testing.assert_allclose(cont.score(x, 64), straight.score(x, 64), rtol=1e-5, atol=1e-6)
    # >= TreeNum existing trees: skipped (model unchanged)
    mtime = os.path.getmtime(mpath)
    _run(a, ["train"])
    assert os.path.getmtime(mpath) == mtime
    # loss changed: from scratch (TreeNum trees, not appended)
    mc = _mc(a)
    mc.train["params"]["TreeNum"] = 8
    mc.train["params"]["Loss"] = "absolute"
    mc.save()
    _run(a, ["train"])
    assert len(read_tree_model(mpath).bags[0]) == 8
    assert read_tree_model(mpath).loss == "absolute"


def test_nn_continuous_structure_growth(tmp_path):
    """isContinuous with a larger network (NNMaster.fitExistingModelIn): the old 1-hidden-layer
    weights sit in the top-left blocks of the new [8, 6]-hidden network, the old bias columns in
    the new bias columns; FixedLayers [1] keeps the copied first-layer block (and its bias,
    FixedBias default true) frozen through training while the rest moves."""
    from shifu_amd.formats.nn_format import read_encog
    from shifu_amd.utils.synthetic import make_model_set
    root = make_model_set(str(tmp_path), "g", "NN", n_rows=900)
    mc = _mc(root)
    mc.train["numTrainEpochs"] = 5
    mc.train["baggingNum"] = 1
    mc.train["params"].update({"NumHiddenLayers": 1, "NumHiddenNodes": [4], "ActivationFunc": ["Sigmoid"]})
    mc.save()
    _run(root, ["init", "stats", "norm", "train"])
    old = read_encog(os.path.join(root, "models/model0.nn"))
    mc = _mc(root)
    mc.train["isContinuous"] = True
    mc.train["params"].update({"NumHiddenLayers": 2, "NumHiddenNodes": [8, 6], "ActivationFunc": ["Sigmoid", "Sigmoid"],
                               "FixedLayers": [1]})
    mc.save()
    _run(root, ["train"])
    new = read_encog(os.path.join(root, "models/model0.nn"))
    assert new.sizes == [old.sizes[0], 8, 6, 1]
    W0o, W0n = old.weights[0], new.weights[0]
    n_in = old.sizes[0]
    np.testing.assert_allclose(W0n[:4, :n_in], W0o[:, :n_in], rtol=1e-6, atol=1e-7)   # frozen block
    np.testing.assert_allclose(W0n[:4, n_in], W0o[:, n_in], rtol=1e-6, atol=1e-7)     # frozen bias
    assert not np.allclose(new.weights[1][:1, :4], old.weights[1][:, :4])            # layer 2 trains


def test_varsel_se_reuse_current_model(tmp_path, monkeypatch):
    """shifu.varsel.se.reuse=true: SE ranks the candidates with the existing models/model0.nn
    instead of training a sensitivity model (the trainer must not be called)."""
    from shifu_amd.config import environment
    from shifu_amd.steps import varsel as VS
    from shifu_amd.utils.synthetic import make_model_set
    root = make_model_set(str(tmp_path), "se", "NN", n_rows=800)
    mc = _mc(root)
    mc.train["numTrainEpochs"] = 5
    mc.train["baggingNum"] = 1
    mc.varSelect["filterBy"] = "SE"
    mc.varSelect["filterNum"] = 3
    mc.save()
    _run(root, ["init", "stats", "norm", "train"])

    def boom(*a, **k):
        raise AssertionError("sensitivity model retrained despite shifu.varsel.se.reuse")
    monkeypatch.setattr(VS, "_train_quick_nn", boom)
    environment.set_property("shifu.varsel.se.reuse", "true")
    try:
        _run(root, ["varsel"])
    finally:
        environment.set_property("shifu.varsel.se.reuse", "false")
    from shifu_amd.config.column_config import load_column_configs
    sel = [c for c in load_column_configs(os.path.join(root, "ColumnConfig.json")) if c.final_select]
    assert len(sel) >= 3


def test_multiclass_rf_native(tmp_path):
    """RF with Gini over 3 classes (no one-vs-all): native multi-class trees (class-value leaves,
    Impurity.java Gini), vote scoring in eval."""
    from shifu_amd.formats import tree_format
    from shifu_amd.utils.synthetic import make_model_set
    root = make_model_set(str(tmp_path), "mcrf", "RF", n_rows=2000, n_classes=3)
    mc = _mc(root)
    mc.train["multiClassifyMethod"] = "NATIVE"
    mc.train["baggingNum"] = 1
    mc.train["params"]["Impurity"] = "gini"
    mc.train["params"]["TreeNum"] = 8
    mc.train["params"]["MaxDepth"] = 6
    mc.save()
    _run(root, ["init", "stats", "norm", "train", "eval"])
    m = tree_format.read_tree_model(os.path.join(root, "models", "model0.rf"))
    assert m.is_classification and not m.is_one_vs_all
    leaves = [nd for t in m.bags[0] for nd in tree_format.iter_nodes(t.root) if nd.is_leaf()]
    assert {nd.class_value for nd in leaves} <= {0, 1, 2} and len({nd.class_value for nd in leaves}) > 1
    perf = json.load(open(os.path.join(root, "evals/Eval1/EvalPerformance.json")))
    assert perf["accuracy"] > 0.55
