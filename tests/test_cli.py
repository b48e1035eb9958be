"""CLI verbs end to end (parity model: ShifuCLITest + the bash driver scripts): every verb of
``shifu_amd.cli`` on the cancer-judgement data, in-process."""
import json
import os

import pytest

DS = "example/cancer-judgement/DataStore"


@pytest.fixture
def model_set(tmp_path, ref_resources, monkeypatch):
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    from shifu_amd.cli import main
    from shifu_amd.config.model_config import ModelConfig
    monkeypatch.chdir(tmp_path)
    assert main(["new", "cj", "-t", "NN"]) == 0
    monkeypatch.chdir(tmp_path / "cj")
    R = os.path.join(ref_resources, DS)
    mc = ModelConfig.load("ModelConfig.json")
    mc.dataSet["dataPath"] = R + "/DataSet1"
    mc.dataSet["headerPath"] = R + "/DataSet1/.pig_header"
    ev = mc.evals[0]
    ev.dataSet["dataPath"] = R + "/EvalSet1"
    ev.dataSet["headerPath"] = R + "/EvalSet1/.pig_header"
    mc.train["numTrainEpochs"] = 10
    mc.train["baggingNum"] = 1
    mc.varSelect["filterNum"] = 12
    mc.save()
    assert main(["init"]) == 0
    assert main(["stats"]) == 0
    return tmp_path / "cj"


def test_nn_verbs(model_set):
    from shifu_amd.cli import main
    assert main(["stats", "-c"]) == 0
    assert os.path.exists("correlation.csv")
    assert main(["varsel"]) == 0
    sel = [c for c in json.load(open("ColumnConfig.json")) if c["finalSelect"]]
    assert 0 < len(sel) <= 12
    assert main(["varsel", "-reset"]) == 0
    assert not any(c["finalSelect"] for c in json.load(open("ColumnConfig.json")))
    assert main(["varsel"]) == 0
    assert main(["norm", "-shuffle"]) == 0
    assert main(["train"]) == 0
    assert main(["posttrain"]) == 0
    assert any(c["columnBinning"].get("binAvgScore") for c in json.load(open("ColumnConfig.json")))
    assert main(["eval", "-new", "Eval2"]) == 0
    assert main(["eval", "-delete", "Eval2"]) == 0
    assert main(["eval"]) == 0
    perf = json.load(open("evals/Eval1/EvalPerformance.json"))
    assert perf["areaUnderRoc"] > 0.85
    for t in ("pmml", "columnstats", "woemapping", "bagging", "corr"):
        assert main(["export", "-t", t]) == 0, t
    assert os.path.exists("pmmls/cj0.pmml")
    assert main(["save", "v1"]) == 0 and main(["switch", "v1"]) == 0
    assert open(".HEAD").read().strip() == "v1"
    assert main(["test", "-filter"]) == 0
    assert main(["nosuchverb"]) == 1


def test_sensitivity_varsel(model_set):
    from shifu_amd.cli import main
    from shifu_amd.config.model_config import ModelConfig
    mc = ModelConfig.load("ModelConfig.json")
    mc.varSelect["filterBy"] = "SE"
    mc.varSelect["filterNum"] = 8
    mc.save()
    assert main(["varsel", "-r", "2"]) == 0
    assert os.path.exists("varsel/se.0") and os.path.exists("varsel/se.1")
    sel = [c for c in json.load(open("ColumnConfig.json")) if c["finalSelect"]]
    assert 0 < len(sel) <= 8


def test_tree_verbs(model_set, tmp_path):
    from shifu_amd.cli import main
    from shifu_amd.config.model_config import ModelConfig
    mc = ModelConfig.load("ModelConfig.json")
    mc.train["algorithm"] = "GBT"
    mc.train["params"] = {"TreeNum": 8, "MaxDepth": 4, "LearningRate": 0.1, "Loss": "squared",
                          "Impurity": "variance", "FeatureSubsetStrategy": "ALL", "MinInstancesPerNode": 5}
    mc.varSelect["filterBy"] = "FI"
    mc.save()
    assert main(["varsel"]) == 0
    assert main(["norm"]) == 0
    assert main(["train"]) == 0
    assert os.path.exists("models/model0.gbt")
    assert main(["eval"]) == 0
    assert main(["encode"]) == 0
    hdr = open("tmp/encodedTrainData/.pig_header").read().strip().split("|")
    assert hdr[-1] == "tree_vars_7"
    z = str(tmp_path / "m.zip")
    assert main(["convert", "-tozipb", "models/model0.gbt", z]) == 0
    assert main(["convert", "-totreeb", z, str(tmp_path / "back.gbt")]) == 0
    from shifu_amd.formats.tree_format import read_tree_model
    a, b = read_tree_model("models/model0.gbt"), read_tree_model(str(tmp_path / "back.gbt"))
    assert len(a.bags[0]) == len(b.bags[0]) == 8
    assert main(["analysis", "-fi", "models/model0.gbt"]) == 0
    assert main(["export", "-t", "pmml"]) == 0


def test_combo(model_set):
    from shifu_amd.cli import main
    assert main(["varsel"]) == 0
    assert main(["combo", "-new", "NN,LR,LR"]) == 0
    assert main(["combo", "-init"]) == 0
    assert main(["combo", "-run"]) == 0
    assert main(["combo", "-eval"]) == 0
    perf = json.load(open("cj_assemble/evals/Eval1/EvalPerformance.json"))
    assert perf["areaUnderRoc"] > 0.8
