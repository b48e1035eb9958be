"""The CLI pipeline on the MI355X: NN (HIP MFMA trainer), LR and GBT (HIP histogram trainer)
on the cancer-judgement data; scores must reach the same quality as the CPU path."""
import json
import os

import pytest

from test_pipeline_e2e import _auc, _make

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("alg,params,min_auc", [("NN", None, 0.9), ("LR", None, 0.9),
                                                ("GBT", {"TreeNum": 20}, 0.75), ("RF", {"TreeNum": 10}, 0.85)])
def test_pipeline_on_gpu(tmp_path, ref_resources, alg, params, min_auc):
    from shifu_amd.steps.evaluate import run_eval
    from shifu_amd.steps.norm import run_norm
    from shifu_amd.steps.stats import run_stats
    from shifu_amd.steps.train import run_train
    from shifu_amd.steps.varsel import run_varsel
    root = _make(tmp_path, ref_resources, alg, epochs=40, params=params)
    assert run_stats(root) == 0
    assert run_varsel(root) == 0
    assert run_norm(root) == 0
    assert run_train(root) == 0
    assert run_eval(root) == 0
    assert _auc(root) > min_auc


def test_sensitivity_varsel_gpu(tmp_path, ref_resources):
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.steps.stats import run_stats
    from shifu_amd.steps.varsel import run_varsel
    root = _make(tmp_path, ref_resources, "NN", epochs=20)
    run_stats(root)
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    mc.varSelect["filterBy"] = "SE"
    mc.varSelect["filterNum"] = 10
    mc.save()
    assert run_varsel(root) == 0
    sel = [c for c in json.load(open(os.path.join(root, "ColumnConfig.json"))) if c["finalSelect"]]
    assert 0 < len(sel) <= 10
