"""PMML score verification (PMMLVerifySuit.java:121-190): export a trained model set to PMML,
evaluate every record with an independent PMML evaluator (scoring/pmml_eval.py, written from the
PMML 4.2 semantics) and compare with the framework's own scores (ModelRunner, the `eval` path)."""
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


def _scores(root):
    from shifu_amd.scoring.model_runner import ModelRunner
    from shifu_amd.steps.base import ModelSet
    ms = ModelSet(root)
    mr = ModelRunner(ms.mc, ms.ccs, ms.pf.models_dir)
    table = ms.load_raw([c for c in ms.ccs if c.name in mr.raw_columns()]).table
    return mr, table, [o[:, 0] for o in mr.score_models(table)]


@pytest.mark.parametrize("alg,norm", [("NN", "ZSCALE"), ("NN", "WOE"), ("LR", "ZSCALE"), ("GBT", None),
                                      ("RF", None)])
def test_exported_pmml_reproduces_scores(tmp_path, alg, norm):
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.scoring.pmml_eval import PMMLModel, records_from_table
    from shifu_amd.utils.synthetic import make_model_set
    root = make_model_set(str(tmp_path), "p", alg, n_rows=600, n_num=5, n_cat=2)
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    mc.train["numTrainEpochs"] = 20
    mc.train["baggingNum"] = 2 if alg == "NN" else 1
    if norm:
        mc.normalize["normType"] = norm
    if alg in ("GBT", "RF"):
        mc.train["params"].update({"TreeNum": 5, "MaxDepth": 4})
    mc.save()
    _run(root, ["init", "stats", "norm", "train", "export -t pmml"])
    mr, table, own = _scores(root)
    names = sorted(mr.raw_columns())
    recs = records_from_table(table, names)[:200]
    for i, own_i in enumerate(own):
        pm = PMMLModel(os.path.join(root, "pmmls", f"{mc.name}{i}.pmml"))
        np.testing.assert_allclose(pm.evaluate(recs), own_i[:200], rtol=1e-5, atol=1e-6)
    if alg == "NN":
        _run(root, ["export -t baggingpmml"])
        pm = PMMLModel(os.path.join(root, "pmmls", f"{mc.name}.pmml"))
        np.testing.assert_allclose(pm.evaluate(recs), np.mean(np.stack(own, 1)[:200], 1), rtol=1e-5, atol=1e-6)
