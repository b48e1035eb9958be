"""Eval report files (algos/eval_reports.py) against the reference's layout: GainChart.generateCsv's
header and number formats (DecimalFormat("#.####"), Double.toString), the file names of
ConfusionMatrix.generateChartAndJsonPerfFiles (no champion column) and EvalModelProcessor.runDistEval
(champion columns + weights), on the reference's cancer-judgement data."""
import json
import os

import pytest

from shifu_amd.algos.eval_reports import CSV_HEADER, java_df, java_double

DS = "example/cancer-judgement/DataStore"


def test_java_number_formats():
    # DecimalFormat("#.####"): HALF_EVEN on the exact binary value, trailing zeros dropped
    assert [java_df(v) for v in (0.5, 1.0, 0.0, 0.12345, 0.00005, 0.000025, -0.00001, 12.34567, 100.0)] == \
        ["0.5", "1", "0", "0.1235", "0.0001", "0", "-0", "12.3457", "100"]
    assert java_df(float("nan")) == "NaN"
    # Double.toString: plain in [1e-3, 1e7), scientific outside
    assert [java_double(v) for v in (0.1, 1000.0, 1e7, 1.5e-4, 123456789.0, 0.0, -2.5, 0.001, 9999999.0)] == \
        ["0.1", "1000.0", "1.0E7", "1.5E-4", "1.23456789E8", "0.0", "-2.5", "0.001", "9999999.0"]


@pytest.fixture
def trained(tmp_path, ref_resources, monkeypatch):
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
    mc.train["numTrainEpochs"] = 5
    mc.train["baggingNum"] = 1
    mc.save()
    for verb in (["init"], ["stats"], ["norm"], ["train"]):
        assert main(verb) == 0, verb
    return tmp_path / "cj"


def _check_csv(path):
    lines = open(path).read().splitlines()
    assert lines[0] + "\n" == CSV_HEADER, path
    assert len(lines) > 2
    for ln in lines[1:]:
        assert len(ln.split(",")) == 9


def test_report_files_without_champion(trained):
    from shifu_amd.cli import main
    assert main(["eval"]) == 0
    d = "evals/Eval1"
    for f in ("Eval1_gainchart.html", "Eval1_prroc.html", "Eval1_unit_wise_gainchart.csv", "Eval1_unit_wise_pr.csv",
              "Eval1_unit_wise_roc.csv", "Eval1_modelscore_gainchart.csv", "EvalPerformance.json"):
        assert os.path.exists(os.path.join(d, f)), f
    assert not any("weighted" in f for f in os.listdir(d))        # no weight column: no weighted CSVs
    for f in os.listdir(d):
        if f.endswith(".csv"):
            _check_csv(os.path.join(d, f))
    perf = json.load(open(os.path.join(d, "EvalPerformance.json")))
    rows = open(os.path.join(d, "Eval1_unit_wise_roc.csv")).read().splitlines()[1:]
    assert len(rows) == len(perf["roc"])
    assert rows[-1].split(",")[2] == java_df(perf["roc"][-1]["recall"])
    page = open(os.path.join(d, "Eval1_gainchart.html")).read()
    assert page.count("<svg") == 7 and "var data_0" in page
    assert open(os.path.join(d, "Eval1_prroc.html")).read().count("<svg") == 8


def test_report_files_with_champions_and_weights(trained):
    from shifu_amd.cli import main
    from shifu_amd.config.model_config import ModelConfig
    mc = ModelConfig.load("ModelConfig.json")
    ev = mc.evals[0]
    ev.dataSet["weightColumnName"] = "column_5"
    meta = ev.get("scoreMetaColumnNameFile") or "columns/Eval1score.meta.column.names"
    ev["scoreMetaColumnNameFile"] = meta
    mc.save()
    os.makedirs(os.path.dirname(meta) or ".", exist_ok=True)
    with open(meta, "w") as f:
        f.write("column_3\ncolumn_9\n")
    assert main(["eval"]) == 0
    d = "evals/Eval1"
    names = ["cj-Eval1", "column_3", "column_9"]
    for f in ("Eval1_gainchart.html", "Eval1_prroc.html"):
        assert os.path.exists(os.path.join(d, f)), f
    for n in names:
        for suffix in ("unit_wise_gainchart", "unit_wise_pr", "unit_wise_roc", "weighted_gainchart", "weighted_pr",
                       "weighted_roc", "modelscore_gainchart"):
            p = os.path.join(d, f"{n}_{suffix}.csv")
            assert os.path.exists(p), p
            _check_csv(p)
    for m in ("column_3", "column_9"):
        assert os.path.exists(os.path.join(d, "EvalMetaScore", f"{m}EvalPerformance.json"))
    page = open(os.path.join(d, "Eval1_gainchart.html")).read()
    for j, n in enumerate(names):                   # every series overlaid on every chart
        assert f"var data_{j}" in page and n in page
