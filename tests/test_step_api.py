"""Programmatic Step API (A5) chains the pipeline in-process."""
import json
import os


def test_step_api_pipeline(tmp_path, monkeypatch):
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.steps import api
    from shifu_amd.utils.synthetic import make_model_set
    root = make_model_set(str(tmp_path), "api", "LR", n_rows=1200)
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    mc.train["numTrainEpochs"] = 30
    mc.train["baggingNum"] = 1
    mc.save()
    ms = api.run_pipeline(root)
    assert any(c.final_select for c in ms.ccs)
    assert os.path.exists(os.path.join(root, "models", "model0.lr"))
    auc = json.load(open(os.path.join(root, "evals/Eval1/EvalPerformance.json")))["areaUnderRoc"]
    assert auc > 0.8
    ccs = api.ExportStep(ms, type="columnstats").process()
    assert ccs and os.path.exists(os.path.join(root, "ColumnStats.csv"))
