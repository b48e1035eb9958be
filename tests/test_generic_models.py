"""Generic models (I5): GenericModelConfig JSON under models/ scored by ModelRunner / eval
(python Computable and safetensors MLP implementations; tensorflow fails with a clear error)."""
import json
import os

import numpy as np
import pytest
import torch

PY_MODEL = '''
import numpy as np
class Mean:
    def init(self, config):
        self.scale = float(config["properties"].get("scale", 1.0))
    def compute(self, X):
        return 1.0 / (1.0 + np.exp(-self.scale * X.sum(1)))
    def release(self):
        pass
'''


def _model_set(tmp_path, monkeypatch):
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.steps import api
    from shifu_amd.utils.synthetic import make_model_set
    root = make_model_set(str(tmp_path), "gen", "LR", n_rows=1500)
    ms = api.run_pipeline(root, steps=(api.InitStep, api.StatsStep, api.VarSelStep, api.NormStep))
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    mc.train["algorithm"] = "GENERIC"
    mc.save()
    return root, ms


def test_python_and_safetensors_generic_models_score_in_eval(tmp_path, monkeypatch):
    from safetensors.torch import save_file
    from shifu_amd.steps import api
    from shifu_amd.scoring.model_runner import ModelRunner
    from shifu_amd.steps.base import ModelSet
    root, ms = _model_set(tmp_path, monkeypatch)
    models = os.path.join(root, "models")
    os.makedirs(models, exist_ok=True)
    sel = [c.name for c in ms.ccs if c.final_select]
    assert sel
    with open(os.path.join(models, "mymodel.py"), "w") as fh:
        fh.write(PY_MODEL)
    json.dump({"inputnames": sel, "properties": {"algorithm": "python", "class": "mymodel:Mean", "scale": 0.5}},
              open(os.path.join(models, "model0.json"), "w"))
    g = torch.Generator().manual_seed(0)
    save_file({"W0": torch.randn(8, len(sel), generator=g), "b0": torch.zeros(8),
               "W1": torch.randn(1, 8, generator=g), "b1": torch.zeros(1)}, os.path.join(models, "mlp.safetensors"))
    json.dump({"inputnames": sel, "properties": {"algorithm": "safetensors_mlp", "weights": "mlp.safetensors",
                                                 "activations": ["tanh", "sigmoid"]}},
              open(os.path.join(models, "model1.json"), "w"))
    ms2 = ModelSet(root)
    runner = ModelRunner(ms2.mc, ms2.ccs, models)
    assert [m.kind for m in runner.models] == ["generic", "generic"]
    by_name = {c.name: c for c in ms2.ccs}
    table = ms2.load_raw([by_name[n] for n in runner.raw_columns()]).table
    res = runner.score(table)
    assert res["model0"].shape == res["model1"].shape
    assert np.all((res["model0"] >= 0) & (res["model0"] <= 1000))
    api.EvalStep(ms2).process()
    perf = json.load(open(os.path.join(root, "evals/Eval1/EvalPerformance.json")))
    assert 0.0 <= perf["areaUnderRoc"] <= 1.0


def test_tensorflow_generic_model_reports_missing_runtime(tmp_path):
    from shifu_amd.scoring.generic import load_generic
    p = tmp_path / "model0.json"
    p.write_text(json.dumps({"inputnames": ["a"], "properties": {"algorithm": "tensorflow"}}))
    with pytest.raises(RuntimeError, match="TensorFlow runtime"):
        load_generic(str(p))


def test_generic_train_is_external(tmp_path, monkeypatch):
    from shifu_amd.steps import api
    root, ms = _model_set(tmp_path, monkeypatch)
    with pytest.raises(ValueError, match="trained outside"):
        api.TrainStep(root).process()
