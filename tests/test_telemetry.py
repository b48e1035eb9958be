"""Opt-in usage records (A3): off by default; when enabled the CLI appends one JSON line per
invocation to the model set's logs/usage.jsonl."""
import json
import os


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
