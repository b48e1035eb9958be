"""Opt-in usage records (A3): off by default; when enabled the CLI appends one JSON line per
invocation to the model set's logs/usage.jsonl."""
import json
import os

import pytest


def test_usage_record_opt_in(tmp_path, monkeypatch):
    from shifu_amd.utils import telemetry
    ms = tmp_path / "ms"
    ms.mkdir()
    (ms / "ModelConfig.json").write_text("{}")
    monkeypatch.delenv("SHIFU_TELEMETRY", raising=False)
    monkeypatch.delenv("SHIFU_STATS_DIR", raising=False)
    assert telemetry.record_usage("stats", [], 0, 1.0, model_set_dir=str(ms)) is None
    assert not (ms / "logs").exists()
    monkeypatch.setenv("SHIFU_TELEMETRY", "1")
    p = telemetry.record_usage("stats", ["-c"], 0, 1.25, model_set_dir=str(ms))
    assert p == os.path.join(str(ms), "logs", "usage.jsonl")
    rec = json.loads(open(p).read().strip())
    assert rec["cmd"] == "stats" and rec["args"] == ["-c"] and rec["rc"] == 0 and rec["seconds"] == 1.25
    # outside a model set nothing is written
    assert telemetry.record_usage("new", [], 0, 0.1, model_set_dir=str(tmp_path)) is None


@pytest.mark.parametrize("alg", ["NN", "GBT"])
def test_metrics_stream_throughput_fields(tmp_path, monkeypatch, alg):
    """SURVEY §5.5 / VERDICT r3 #6: the training metrics stream carries throughput, all-reduce time
    and (trees) the per-level histogram table, next to the errors."""
    import json
    import os
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.steps.base import ModelSet
    from shifu_amd.steps.create import run_init
    from shifu_amd.steps.norm import run_norm
    from shifu_amd.steps.stats import run_stats
    from shifu_amd.steps.train import run_train
    from shifu_amd.utils.synthetic import make_model_set
    root = make_model_set(str(tmp_path), "m", alg, n_rows=800, n_num=5, n_cat=1)
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    mc.train["numTrainEpochs"] = 4
    mc.train["baggingNum"] = 1
    if alg == "GBT":
        mc.train["params"]["TreeNum"] = 3
        mc.train["params"]["MaxDepth"] = 4
    mc.save()
    run_init(root)
    run_stats(root)
    run_norm(root)
    run_train(root)
    path = ModelSet(root).pf.metrics_jsonl
    recs = [json.loads(l) for l in open(path) if l.strip()]
    recs = [r for r in recs if "train_error" in r]
    assert recs, path
    r = recs[-1]
    if alg == "NN":
        assert r["rows_per_s"] > 0 and r["epoch_ms"] > 0 and r["allreduce_ms"] >= 0
    else:
        assert r["tree_ms"] > 0 and r["hist_rows"] > 0 and r["allreduce_ms"] >= 0
        lv = r["levels"]
        assert lv and lv[0]["level"] == 1 and lv[0]["hist_rows"] > 0
        assert all("hist_split_ms" in e for e in lv)
