"""Four gloo ranks against one process, verb by verb (the simulated-DP equivalence of the
reference's DTrainTest.java:96-180, at world 4): the data set is three part files of uneven size
plus one row so wide that a whole rank's byte range holds no line start, so one rank has no rows
at all and the others hold different row counts.  Covered: stats, stats -c, norm, varsel (SE),
train (NN), posttrain and eval with a champion score column; GBT training in its own model set
(trees bit-identical)."""
import json
import os
import shutil
import socket

import numpy as np
import torch.multiprocessing as mp

WORLD = 4


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_cli(rank, world, port, root, verb):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), SHIFU_FORCE_CPU="1")
    os.chdir(root)
    from shifu_amd.cli import main
    rc = main(verb.split())
    if rc != 0:
        raise SystemExit(rc)


def _uneven(root, rows_first=700):
    """Split DataSet1 into uneven parts and append one very wide row (its meta id field holds
    ~40 % of the data set's bytes): with 4 ranks one byte range starts no line."""
    from shifu_amd.config.model_config import ModelConfig
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    d = mc.resolve(mc.dataSet["dataPath"])
    src = os.path.join(d, "part-00000")
    lines = open(src).read().strip().split("\n")
    os.remove(src)
    with open(os.path.join(d, "part-00000"), "w") as f:
        f.write("\n".join(lines[:rows_first]) + "\n")
    with open(os.path.join(d, "part-00001"), "w") as f:
        f.write(lines[rows_first] + "\n")
    rest = lines[rows_first + 1:]
    total = sum(len(l) + 1 for l in lines)
    wide = rest[0].split("|")
    wide[0] = "w" * int(total * 0.7)                       # ~40 % of the final bytes
    with open(os.path.join(d, "part-00002"), "w") as f:
        f.write("\n".join(rest[1:]) + "\n" + "|".join(wide) + "\n")
    return d


def _run_one(root, verb):
    from shifu_amd.cli import main
    cwd = os.getcwd()
    os.chdir(root)
    try:
        assert main(verb.split()) == 0, verb
    finally:
        os.chdir(cwd)


def _run_world(root, verb):
    mp.start_processes(_rank_cli, args=(WORLD, _port(), root, verb), nprocs=WORLD, join=True, start_method="spawn")


def _byte_ranges_hold_a_rank_without_lines(d):
    from shifu_amd.data.reader import list_data_files
    from shifu_amd.data.stream import _lines_in_range, byte_ranges
    files = list_data_files(d)
    empty = 0
    for r in range(WORLD):
        n = 0
        for _, path, a, b in byte_ranges(files, r, WORLD):
            for _, blk in _lines_in_range(path, a, b, 1 << 20):
                n += bytes(blk).count(b"\n")
        empty += n == 0
    return empty


def test_nn_verbs_world4_match_single(tmp_path, monkeypatch):
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    from shifu_amd.config.column_config import load_column_configs
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.steps.base import load_dataset_cache
    from shifu_amd.steps.create import run_init
    from shifu_amd.steps.stats import read_correlation
    from shifu_amd.utils.synthetic import make_model_set
    a = make_model_set(str(tmp_path), "a", "NN", n_rows=1503, n_num=6, n_cat=2)
    mc = ModelConfig.load(os.path.join(a, "ModelConfig.json"))
    mc.varSelect["filterBy"] = "SE"
    mc.varSelect["filterNum"] = 5
    mc.varSelect["autoFilterEnable"] = False
    mc.train["numTrainEpochs"] = 10
    mc.train["baggingNum"] = 1
    mc.evals[0]["scoreMetaColumnNameFile"] = "columns/Eval1score.meta.column.names"
    mc.save()
    with open(os.path.join(a, "columns", "Eval1score.meta.column.names"), "w") as f:
        f.write("num_0\n")                                  # a champion score column
    d = _uneven(a)
    assert _byte_ranges_hold_a_rank_without_lines(d) >= 1
    run_init(a)
    b = str(tmp_path / "b")
    shutil.copytree(a, b)
    mcb = ModelConfig.load(os.path.join(b, "ModelConfig.json"))
    mcb.dataSet["dataPath"] = d.replace(a, b)
    mcb.save()

    # stats
    _run_one(a, "stats")
    _run_world(b, "stats")
    ca = json.load(open(os.path.join(a, "ColumnConfig.json")))
    cb = json.load(open(os.path.join(b, "ColumnConfig.json")))
    for x, y in zip(ca, cb):
        bx, by = x["columnBinning"], y["columnBinning"]
        assert bx.get("binBoundary") == by.get("binBoundary"), x["columnName"]
        assert bx.get("binCategory") == by.get("binCategory"), x["columnName"]
        assert bx.get("binCountPos") == by.get("binCountPos"), x["columnName"]
        for k in ("totalCount", "missingCount", "distinctCount", "max", "min"):
            assert x["columnStats"].get(k) == y["columnStats"].get(k), (x["columnName"], k)
        for k in ("mean", "stdDev", "ks", "iv"):
            if x["columnStats"].get(k) is not None:
                np.testing.assert_allclose(x["columnStats"][k], y["columnStats"][k], rtol=1e-9, atol=1e-9)

    # stats -c
    _run_one(a, "stats -c")
    _run_world(b, "stats -c")
    na, xa = read_correlation(os.path.join(a, "correlation.csv"))
    nb, xb = read_correlation(os.path.join(b, "correlation.csv"))
    assert na == nb
    np.testing.assert_allclose(xa, xb, atol=1e-10)

    # norm
    _run_one(a, "norm")
    _run_world(b, "norm")
    ma, da = load_dataset_cache(os.path.join(a, "tmp", "NormalizedData"), mmap=False)
    mb, db = load_dataset_cache(os.path.join(b, "tmp", "NormalizedData"), mmap=False)
    assert ma["n"] == mb["n"] and set(da) == set(db)
    for k in da:
        np.testing.assert_array_equal(da[k], db[k], err_msg=k)

    # varsel (SE): per-input sensitivities all-reduced over 4 ranks
    _run_one(a, "varsel")
    _run_world(b, "varsel")

    def se(root):
        rows = [l.split("\t") for l in open(os.path.join(root, "varsel", "se.0")).read().strip().split("\n")]
        return {r[1]: float(r[3]) for r in rows}
    sa, sb = se(a), se(b)
    assert sa.keys() == sb.keys()
    np.testing.assert_allclose([sa[k] for k in sa], [sb[k] for k in sa], rtol=2e-3, atol=1e-6)
    fa = sorted(c.name for c in load_column_configs(os.path.join(a, "ColumnConfig.json")) if c.final_select)
    fb = sorted(c.name for c in load_column_configs(os.path.join(b, "ColumnConfig.json")) if c.final_select)
    assert fa == fb and len(fa) == 5

    # train (NN): gradients all-reduced over 4 ranks
    _run_one(a, "train")
    _run_world(b, "train")
    from shifu_amd.formats.nn_format import is_binary_nn, read_binary_nn, read_encog

    def weights(root):
        p = os.path.join(root, "models", "model0.nn")
        net = read_binary_nn(p)["networks"][0] if is_binary_nn(p) else read_encog(p)
        return np.concatenate([np.ravel(np.asarray(x, dtype=np.float64)) for x in net.weights])
    wa, wb = weights(a), weights(b)
    np.testing.assert_allclose(wa, wb, rtol=1e-3, atol=1e-4)

    # posttrain and eval on the same model files
    shutil.rmtree(os.path.join(b, "models"))
    shutil.copytree(os.path.join(a, "models"), os.path.join(b, "models"))
    _run_one(a, "posttrain")
    _run_world(b, "posttrain")
    ba = {c.name: c.bin_avg_score for c in load_column_configs(os.path.join(a, "ColumnConfig.json")) if c.final_select}
    bb = {c.name: c.bin_avg_score for c in load_column_configs(os.path.join(b, "ColumnConfig.json")) if c.final_select}
    assert ba.keys() == bb.keys()
    for k in ba:
        assert np.max(np.abs(np.array(ba[k]) - np.array(bb[k]))) <= 1, k
    _run_one(a, "eval")
    _run_world(b, "eval")
    pa = json.load(open(os.path.join(a, "evals", "Eval1", "EvalPerformance.json")))
    pb = json.load(open(os.path.join(b, "evals", "Eval1", "EvalPerformance.json")))
    assert abs(pa["areaUnderRoc"] - pb["areaUnderRoc"]) < 1e-6
    meta = os.path.join("evals", "Eval1", "EvalMetaScore", "num_0EvalPerformance.json")
    qa, qb = json.load(open(os.path.join(a, meta))), json.load(open(os.path.join(b, meta)))
    assert abs(qa["areaUnderRoc"] - qb["areaUnderRoc"]) < 1e-9

    def score_rows(root):
        p = os.path.join(root, "evals", "Eval1", "EvalScore")
        p = os.path.join(p, "part-00000") if os.path.isdir(p) else p
        return open(p).read().strip().split("\n")
    ra, rb = score_rows(a), score_rows(b)
    assert ra[0] == rb[0] and len(ra) == len(rb)
    j = ra[0].split("|").index("mean")
    for x, y in zip(sorted(ra[1:], key=lambda r: r.split("|")[-1]), sorted(rb[1:], key=lambda r: r.split("|")[-1])):
        fx, fy = x.split("|"), y.split("|")
        assert fx[:2] == fy[:2] and fx[-1] == fy[-1]          # tag, weight, champion value
        assert abs(float(fx[j]) - float(fy[j])) < 1e-3        # fp32 GEMM blocking differs by batch shape
    assert "np.float64" not in "".join(ra)


def test_gbt_train_world4_bitwise(tmp_path, monkeypatch):
    """GBT over 4 ranks (one without rows): int64 fixed-point histograms all-reduced -> the same
    trees, byte for byte, as one process."""
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.steps.create import run_init
    from shifu_amd.utils.synthetic import make_model_set
    a = make_model_set(str(tmp_path), "a", "GBT", n_rows=1503, n_num=6, n_cat=2)
    mc = ModelConfig.load(os.path.join(a, "ModelConfig.json"))
    mc.train["baggingNum"] = 1
    mc.train["params"] = {"TreeNum": 4, "MaxDepth": 4, "LearningRate": 0.1, "Loss": "squared",
                          "Impurity": "variance", "FeatureSubsetStrategy": "ALL", "MinInstancesPerNode": 5}
    mc.save()
    d = _uneven(a)
    run_init(a)
    _run_one(a, "stats")
    _run_one(a, "norm")
    b = str(tmp_path / "b")
    shutil.copytree(a, b)
    mcb = ModelConfig.load(os.path.join(b, "ModelConfig.json"))
    mcb.dataSet["dataPath"] = d.replace(a, b)
    mcb.save()
    _run_one(a, "train")
    _run_world(b, "train")
    ga = open(os.path.join(a, "models", "model0.gbt"), "rb").read()
    gb = open(os.path.join(b, "models", "model0.gbt"), "rb").read()
    assert ga == gb
