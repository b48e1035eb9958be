"""End-to-end CLI-equivalent pipeline on the reference's cancer-judgement data set
(parity model: ``bin/shifutest`` / ``src/test/bash/driver_test.sh`` NN/LR/GBT smoke drivers):
new -> init -> stats -> norm -> varsel -> train -> posttrain -> eval -> export."""
import json
import os

import numpy as np
import pytest

DS = "example/cancer-judgement/DataStore"


def _make(tmp_path, ref_resources, alg="NN", epochs=30, bags=1, params=None):
    from shifu_amd.steps.base import ModelSet
    from shifu_amd.steps.create import run_init, run_new
    R = os.path.join(ref_resources, DS)
    run_new("cj", alg, parent=str(tmp_path))
    root = str(tmp_path / "cj")
    ms = ModelSet(root)
    mc = ms.mc
    mc.dataSet["dataPath"] = R + "/DataSet1"
    mc.dataSet["headerPath"] = R + "/DataSet1/.pig_header"
    mc.dataSet["weightColumnName"] = "column_3"
    ev = mc.evals[0]
    ev.dataSet["dataPath"] = R + "/EvalSet1"
    ev.dataSet["headerPath"] = R + "/EvalSet1/.pig_header"
    mc.train["numTrainEpochs"] = epochs
    mc.train["baggingNum"] = bags
    if params:
        mc.train["params"].update(params)
    mc.save()
    assert run_init(root) == 0
    return root


def _auc(root):
    return json.load(open(os.path.join(root, "evals/Eval1/EvalPerformance.json")))["areaUnderRoc"]


@pytest.fixture(autouse=True)
def _cpu(monkeypatch):
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")


def test_nn_pipeline(tmp_path, ref_resources):
    from shifu_amd.steps.evaluate import run_eval
    from shifu_amd.steps.norm import run_norm
    from shifu_amd.steps.stats import run_stats
    from shifu_amd.steps.train import run_train
    root = _make(tmp_path, ref_resources, "NN", epochs=40, bags=2)
    assert run_stats(root) == 0
    assert run_norm(root) == 0
    assert run_train(root) == 0
    assert sorted(os.listdir(os.path.join(root, "models"))) == ["model0.nn", "model1.nn"]
    assert os.path.exists(os.path.join(root, "bmodels/model0.nn"))
    log = open(os.path.join(root, "tmp/train.progress.log")).read()
    assert "Trainer 1 Epoch #40 Training Error:" in log
    assert run_eval(root) == 0
    assert _auc(root) > 0.9
    hdr = open(os.path.join(root, "evals/Eval1/EvalScore")).readline().strip().split("|")
    assert hdr[:8] == ["tag", "weight", "mean", "max", "min", "median", "model0", "model1"]


@pytest.mark.parametrize("alg,params,min_auc", [("LR", None, 0.9), ("GBT", {"TreeNum": 20}, 0.75),
                                                ("RF", {"TreeNum": 10}, 0.85)])
def test_other_algorithms(tmp_path, ref_resources, alg, params, min_auc):
    from shifu_amd.steps.evaluate import run_eval
    from shifu_amd.steps.norm import run_norm
    from shifu_amd.steps.stats import run_stats
    from shifu_amd.steps.train import run_train
    root = _make(tmp_path, ref_resources, alg, epochs=40, params=params)
    run_stats(root)
    run_norm(root)
    run_train(root)
    run_eval(root)
    assert _auc(root) > min_auc


def test_binary_nn_matches_text_model(tmp_path, ref_resources):
    from shifu_amd.data.purifier import load_dataset
    from shifu_amd.scoring.model_runner import IndependentNNModel, ModelRunner, load_model
    from shifu_amd.steps.base import ModelSet
    from shifu_amd.steps.norm import run_norm
    from shifu_amd.steps.stats import run_stats
    from shifu_amd.steps.train import run_train
    root = _make(tmp_path, ref_resources, "NN", epochs=5)
    run_stats(root)
    run_norm(root)
    run_train(root)
    ms = ModelSet(root)
    md = load_dataset(ms.mc, ms.mc.evals[0].dataSet, [c.name for c in ms.ccs if not c.is_target()], [],
                      require_target=False)
    a = IndependentNNModel(load_model(os.path.join(root, "bmodels/model0.nn")).obj).compute(md.table)[:, 0]
    b = ModelRunner(ms.mc, ms.ccs, model_paths=[os.path.join(root, "models/model0.nn")]).score_models(md.table)[0][:, 0]
    np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-7)


def test_grid_search_and_kfold(tmp_path, ref_resources):
    from shifu_amd.steps.norm import run_norm
    from shifu_amd.steps.stats import run_stats
    from shifu_amd.steps.train import flatten_grid, run_train
    assert len(flatten_grid({"LearningRate": [0.1, 0.2], "NumHiddenNodes": [[5], [10]], "Propagation": "R"})) == 4
    assert len(flatten_grid({"NumHiddenNodes": [5], "ActivationFunc": ["tanh"]})) == 1
    root = _make(tmp_path, ref_resources, "NN", epochs=5, params={"LearningRate": [0.1, 0.3]})
    run_stats(root)
    run_norm(root)
    run_train(root)
    best = json.load(open(os.path.join(root, "tmp/gridsearch.best.json")))
    assert best["index"] in (0, 1)
    from shifu_amd.steps.base import ModelSet
    ms = ModelSet(root)
    ms.mc.train["params"]["LearningRate"] = 0.1
    ms.mc.train["numKFold"] = 3
    ms.save_mc()
    run_train(root)
    assert len(os.listdir(os.path.join(root, "tmp/valerr"))) >= 3
