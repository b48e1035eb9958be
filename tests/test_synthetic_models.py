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
                          "LearningRate": 0.05, "NumEmbedOuputs": 4, "WDLL2Reg": 0.0}
    mc.save()
    _run(root, ["init", "stats", "varsel", "norm", "train", "eval"])
    assert os.path.exists(os.path.join(root, "models/model0.wdl"))
    auc = json.load(open(os.path.join(root, "evals/Eval1/EvalPerformance.json")))["areaUnderRoc"]
    assert auc > 0.8


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


def test_autotype_rebin_psi(tmp_path):
    from shifu_amd.utils.synthetic import make_model_set
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
