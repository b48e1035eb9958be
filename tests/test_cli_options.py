"""The secondary options of ShifuCLI (J/ShifuCLI.java:170-415, option table :702-813): cp,
init -model, varselect alias, stats -rebin -vars/-n/-ivr/-bic (ColumnConfigDynamicBinning
semantics), export woemapping/woe/corr file formats, eval -score sorted vs -nosort, eval -norm
-strict, on the cancer-judgement data."""
import json
import os

import numpy as np
import pytest

from tests.test_cli import model_set  # noqa: F401  (fixture)


def _ccs():
    return json.load(open("ColumnConfig.json"))


def test_cp_and_init_model(model_set, tmp_path):  # noqa: F811
    from shifu_amd.cli import main
    dst = str(tmp_path / "copied")
    assert main(["cp", ".", dst]) == 0
    mc = json.load(open(os.path.join(dst, "ModelConfig.json")))
    assert mc["basic"]["name"] == "copied"
    d = json.load(open("ModelConfig.json"))
    d["train"]["params"] = {}
    json.dump(d, open("ModelConfig.json", "w"))
    assert main(["init", "-model"]) == 0
    params = json.load(open("ModelConfig.json"))["train"]["params"]
    assert "LearningRate" in params and "NumHiddenLayers" in params


def test_rebin_vars_bic_and_backup(model_set):  # noqa: F811
    from shifu_amd.cli import main
    before = {c["columnName"]: c for c in _ccs()}
    num = [n for n, c in before.items() if c["columnType"] == "N" and c["columnFlag"] not in ("Target", "Meta")
           and len(c["columnBinning"].get("binBoundary") or []) > 6][:2]
    assert len(num) == 2
    assert main(["stats", "-rebin", "-vars", num[0], "-n", "4"]) == 0
    after = {c["columnName"]: c for c in _ccs()}
    assert len(after[num[0]]["columnBinning"]["binBoundary"]) == 4
    # untouched column keeps its bins
    assert after[num[1]]["columnBinning"]["binBoundary"] == before[num[1]]["columnBinning"]["binBoundary"]
    # counts are preserved by merging (missing bin carried over)
    cb0, cb1 = before[num[0]]["columnBinning"], after[num[0]]["columnBinning"]
    assert sum(cb1["binCountPos"]) == sum(cb0["binCountPos"]) and sum(cb1["binCountNeg"]) == sum(cb0["binCountNeg"])
    assert cb1["binCountPos"][-1] == cb0["binCountPos"][-1]
    # the second rebin starts from the backup (original) binning, not from the 4-bin result
    assert os.path.exists("tmp/ColumnConfig.json")
    assert main(["stats", "-rebin", "-vars", num[0], "-n", "6"]) == 0
    assert len({c["columnName"]: c for c in _ccs()}[num[0]]["columnBinning"]["binBoundary"]) == 6
    # -bic: every (non-missing) bin holds at least that many rows
    assert main(["stats", "-rebin", "-vars", num[1], "-bic", "60"]) == 0
    cb = {c["columnName"]: c for c in _ccs()}[num[1]]["columnBinning"]
    tot = np.array(cb["binCountPos"][:-1]) + np.array(cb["binCountNeg"][:-1])
    assert (tot >= 60).all() or len(tot) == 1


def test_dynamic_binning_entropy_merge():
    from shifu_amd.algos.dynamic_binning import dynamic_rebin
    # two pure groups: merging inside a group loses no entropy, across groups it does
    bounds = [-np.inf, 1, 2, 3]
    pos, neg = [10, 10, 0, 0, 0], [0, 0, 10, 10, 0]
    bins, miss = dynamic_rebin(False, bounds, pos, neg, pos, neg, expected_bins=2)
    assert [b.left for b in bins] == [-np.inf, 2]
    assert [b.pos for b in bins] == [20, 0] and [b.neg for b in bins] == [0, 20]
    # categorical: sorted by positive rate, merged groups joined with '@^'
    bins, _ = dynamic_rebin(True, ["a", "b", "c"], [9, 1, 8, 0], [1, 9, 2, 0], [9, 1, 8, 0], [1, 9, 2, 0],
                            expected_bins=2)
    assert sorted(len(b.values) for b in bins) == [1, 2]
    assert any(set(b.values) == {"a", "c"} for b in bins)


def test_export_woe_files(model_set):  # noqa: F811
    from shifu_amd.cli import main
    c = [c for c in _ccs() if c["columnType"] == "N" and c["columnFlag"] not in ("Target", "Meta")][0]
    assert main(["export", "-t", "woemapping", "-vars", c["columnName"], "-n", "3"]) == 0
    txt = open("woemapping.txt").read()
    assert txt.startswith("( case \n\twhen %s = . then " % c["columnName"])
    assert txt.rstrip().endswith("end ) as %s_3" % c["columnName"])
    assert txt.count("\twhen (") == 3
    assert main(["export", "-t", "woe"]) == 0
    lines = open("varwoe_info.txt", encoding="utf-8").read().split("\n")
    i = lines.index(c["columnName"])
    assert lines[i + 1].startswith("(-∞,")
    n = len(c["columnBinning"]["binBoundary"])
    assert lines[i + n].startswith("(") and "+∞]" in lines[i + n]
    assert lines[i + n + 1].startswith("MISSING\t")


def test_corr_csv_and_export(model_set):  # noqa: F811
    from shifu_amd.cli import main
    assert main(["stats", "-c"]) == 0
    lines = open("correlation.csv").read().strip().split("\n")
    ccs = _ccs()
    assert lines[0].startswith("ColumnIndex,,0,1")
    assert lines[1].split(",")[1] == "ColumnName" and lines[1].split(",")[2] == ccs[0]["columnName"]
    row = lines[2].split(",")
    assert len(row) == len(ccs) + 2
    k = int(row[0])
    assert abs(float(row[2 + k]) - 1.0) < 1e-6          # self correlation
    assert main(["export", "-t", "corr"]) == 0
    pairs = [l.split(",") for l in open("tmp/vars_corr.csv").read().strip().split("\n")]
    vals = [float(p[2]) for p in pairs]
    assert vals == sorted(vals, reverse=True)
    assert all(p[0] < p[1] for p in pairs)


def test_eval_score_sort_nosort_and_strict(model_set):  # noqa: F811
    from shifu_amd.cli import main
    assert main(["varselect"]) == 0
    assert main(["norm"]) == 0
    assert main(["train"]) == 0
    assert main(["eval", "-score", "Eval1"]) == 0
    path = "evals/Eval1/EvalScore"
    path = os.path.join(path, "part-00000") if os.path.isdir(path) else path

    def means():
        rows = [l.split("|") for l in open(path).read().strip().split("\n")]
        j = rows[0].index("mean")
        return [float(r[j]) for r in rows[1:]]
    s = means()
    assert s == sorted(s, reverse=True) and len(set(s)) > 5
    assert main(["eval", "-score", "Eval1", "-nosort"]) == 0
    s2 = means()
    assert sorted(s2, reverse=True) == s and s2 != s
    assert main(["eval", "-norm", "Eval1", "-strict"]) == 0
