"""Local concurrency helpers (E6): retried tasks, thread-pool fan-out, CLI child processes, and
combo sub-models trained side by side as child processes."""
import json
import os

import pytest


def test_retry_then_success_and_order():
    from shifu_amd.runtime.executor import ExecutorManager
    calls = {"a": 0}

    def flaky():
        calls["a"] += 1
        if calls["a"] < 3:
            raise RuntimeError("transient")
        return "ok"
    assert ExecutorManager(2, retries=2).run([flaky, lambda: 7], ["flaky", "seven"]) == ["ok", 7]
    assert calls["a"] == 3


def test_retries_exhausted_raises():
    from shifu_amd.runtime.executor import ExecutorManager, TaskFailed

    def bad():
        raise ValueError("always")
    with pytest.raises(TaskFailed, match="after 2 attempts"):
        ExecutorManager(1, retries=1).run([bad], ["bad"])


def test_run_cli_child_process(tmp_path):
    from shifu_amd.runtime.executor import run_cli
    assert run_cli(["version"], str(tmp_path)) == 0
    assert run_cli(["init"], str(tmp_path)) != 0          # no model set here


def test_combo_parallel_sub_models(tmp_path, ref_resources, monkeypatch):
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    from shifu_amd.cli import main
    from shifu_amd.config.model_config import ModelConfig
    monkeypatch.chdir(tmp_path)
    assert main(["new", "cp", "-t", "LR"]) == 0
    monkeypatch.chdir(tmp_path / "cp")
    R = os.path.join(ref_resources, "example/cancer-judgement/DataStore")
    mc = ModelConfig.load("ModelConfig.json")
    mc.dataSet["dataPath"] = R + "/DataSet1"
    mc.dataSet["headerPath"] = R + "/DataSet1/.pig_header"
    mc.evals[0].dataSet["dataPath"] = R + "/EvalSet1"
    mc.evals[0].dataSet["headerPath"] = R + "/EvalSet1/.pig_header"
    mc.train["numTrainEpochs"] = 10
    mc.train["baggingNum"] = 1
    mc.save()
    assert main(["init"]) == 0 and main(["stats"]) == 0 and main(["varsel"]) == 0
    assert main(["combo", "-new", "LR,GBT,LR"]) == 0
    assert main(["combo", "-init"]) == 0
    assert main(["-Dshifu.combo.parallel=2", "combo", "-run"]) == 0
    subs = sorted(d for d in os.listdir(".") if d.startswith("cp_") and not d.endswith("assemble"))
    assert subs == ["cp_GBT_1", "cp_LR_0"]
    for d in subs:
        assert any(f.startswith("model0.") for f in os.listdir(os.path.join(d, "models")))
        assert os.path.exists(os.path.join(d, "combo_sub.log"))
    assert main(["combo", "-eval"]) == 0
    perf = json.load(open("cp_assemble/evals/Eval1/EvalPerformance.json"))
    assert perf["areaUnderRoc"] > 0.8
