"""Config JSON round trips and model file formats against the reference's own fixtures
(parity model: ModelConfigTest / ColumnConfig tests, IndependentNNModelTest, IndependentTreeModelTest)."""
import os

import numpy as np
import pytest

from conftest import REF_TR
from shifu_amd.config import jsonio
from shifu_amd.config.column_config import load_column_configs, save_column_configs
from shifu_amd.config.model_config import ModelConfig, create_init_model_config
from shifu_amd.formats import nn_format, tree_format

CJ = "example/cancer-judgement/ModelStore/ModelSet1"


def test_model_config_roundtrip_bytes(ref_resources, tmp_path):
    p = os.path.join(ref_resources, CJ, "ModelConfig.json")
    mc = ModelConfig.load(p)
    assert mc.is_binary() and not mc.is_multiclass()
    assert mc.algorithm == "NN"
    out = tmp_path / "mc.json"
    mc.save(str(out))
    assert jsonio.load(p) == jsonio.load(str(out))
    # a file we wrote ourselves round-trips byte for byte
    out2 = tmp_path / "mc2.json"
    ModelConfig.load(str(out)).save(str(out2))
    assert out.read_text() == out2.read_text()


def test_column_config_roundtrip_bytes(ref_resources, tmp_path):
    p = os.path.join(ref_resources, CJ, "ColumnConfig.json")
    ccs = load_column_configs(p)
    assert len(ccs) > 30
    assert sum(1 for c in ccs if c.is_target()) == 1
    out = tmp_path / "cc.json"
    save_column_configs(ccs, str(out))
    a, b = jsonio.load(p), jsonio.load(str(out))

    def subset(x, y):   # every field of the (older-version) fixture survives unchanged
        if isinstance(x, dict):
            return all(k in y and subset(v, y[k]) for k, v in x.items())
        if isinstance(x, list):
            return len(x) == len(y) and all(subset(u, v) for u, v in zip(x, y))
        return x == y
    assert subset(a, b)


def test_jsonio_special_values():
    d = {"a": float("nan"), "b": [1.0, 2.5], "c": [{"x": 1}], "d": None, "e": 1e-7}
    s = jsonio.dumps(d)
    back = jsonio.loads(s)
    assert back["b"] == [1.0, 2.5] and back["c"][0]["x"] == 1 and back["d"] is None


def test_init_model_config_defaults():
    mc = create_init_model_config("demo", "GBT")
    assert mc.algorithm == "GBT"
    assert mc.param("TreeNum") is not None


def test_encog_nn_fixture_and_roundtrip(ref_resources, tmp_path):
    net = nn_format.read_encog(os.path.join(ref_resources, CJ, "models/model0.nn"))
    assert net.sizes[0] == 30 and net.sizes[-1] == 1
    x = np.random.default_rng(0).normal(size=(7, net.n_in))
    y0 = net.forward(x)
    assert np.all((y0 > 0) & (y0 < 1))
    out = tmp_path / "m.nn"
    nn_format.write_encog(net, str(out))
    net2 = nn_format.read_encog(str(out))
    np.testing.assert_allclose(net2.forward(x), y0, rtol=1e-12)


def test_binary_nn_roundtrip(tmp_path):
    rng = np.random.default_rng(1)
    net = nn_format.NNNetwork([5, 4, 1], ["tanh", "sigmoid"],
                              [rng.normal(size=(4, 6)), rng.normal(size=(1, 5))], {"k": "v"}, [0, 1, 2, 3, 4])
    cs = [nn_format.NNColumnStats(i, f"c{i}", "N", 6.0, 0.1, 1.0, 0, 1, 0, 1, [float("-inf"), 0.0], [],
                                  [0.1, 0.2, 0.3], [0.0, 0.1, 0.2], [0.0, 0.1, 0.2]) for i in range(5)]
    p = tmp_path / "m.nn"
    nn_format.write_binary_nn(str(p), "ZSCALE", cs, {i: i for i in range(5)}, [net])
    assert nn_format.is_binary_nn(str(p))
    d = nn_format.read_binary_nn(str(p))
    assert d["norm_type"] == "ZSCALE" and len(d["column_stats"]) == 5
    x = rng.normal(size=(3, 5))
    np.testing.assert_allclose(d["networks"][0].forward(x), net.forward(x), rtol=1e-12)


def test_gbt_fixture_read_and_roundtrip(ref_resources, tmp_path):
    p = os.path.join(ref_resources, "example/readablespec/model0.gbt")
    m = tree_format.read_tree_model(p)
    assert m.algorithm.upper() == "GBT" and len(m.bags) == 1 and len(m.bags[0]) == 100
    out = tmp_path / "m.gbt"
    tree_format.write_tree_model(str(out), m)
    m2 = tree_format.read_tree_model(str(out))
    rng = np.random.default_rng(0)
    x = {c: rng.normal(size=5) * 10 for c in m.names}
    np.testing.assert_allclose(m.score(x, 5), m2.score(x, 5))
    fi = tree_format.feature_importance(m)
    assert abs(sum(fi.values()) - 1.0) < 1e-9


def test_readable_zip_spec_matches_reference_bytes(tmp_path, ref_resources):
    """convert -totreeb / -tozipb in the reference layout (IndependentTreeModelUtils): the
    reference's own conversion outputs are the oracle -- model0.zip -> .gbt reproduces
    model1.gbt's payload byte for byte, and model0.gbt -> zip reproduces model0.zip's ``trees``
    entry byte for byte and its ``model.ini`` JSON."""
    import gzip
    import json
    import zipfile
    from shifu_amd.steps.misc import gbt_to_zip, zip_to_gbt
    spec = os.path.join(REF_TR, "example", "readablespec")
    zip_to_gbt(os.path.join(spec, "model0.zip"), str(tmp_path / "m.gbt"))
    ours = gzip.decompress(open(tmp_path / "m.gbt", "rb").read())
    assert ours == gzip.decompress(open(os.path.join(spec, "model1.gbt"), "rb").read())
    gbt_to_zip(os.path.join(spec, "model0.gbt"), str(tmp_path / "m.zip"))
    z1, z2 = zipfile.ZipFile(tmp_path / "m.zip"), zipfile.ZipFile(os.path.join(spec, "model0.zip"))
    assert z1.read("trees") == z2.read("trees")
    assert json.loads(z1.read("model.ini")) == json.loads(z2.read("model.ini"))


def test_legacy_pre_versioned_gbt_fixture(ref_resources):
    """The wdbc model set's model0.gbt predates the version field (int-framed strings, impurity +
    leaf flag + weight ratio per node, column names in the splits).  Parsed completely (every byte
    consumed, 13 nodes) and scored through the same TreeModelFile path; the expected leaf values
    follow from the stored tree (root worst_concave_points < 0.14781, ...)."""
    import numpy as np
    from shifu_amd.formats.tree_format import read_tree_model, CONTINUOUS
    path = os.path.join(REF_TR, "example", "wdbc", "wdbcModelSetLocal", "models", "model0.gbt")
    m = read_tree_model(path)
    assert m.algorithm == "GBT" and m.loss == "squared" and m.version == 0
    t = m.bags[0][0]
    assert t.node_num == 13 and t.root_wgt_cnt == 290.0 and len(t.features) == 13
    assert t.root.split.column == 29 and t.root.split.ftype == CONTINUOUS
    assert abs(t.root.split.threshold - 0.14781) < 1e-12 and m.names[29] == "worst_concave_points"

    def count(nd):
        return 0 if nd is None else 1 + count(nd.left) + count(nd.right)
    assert count(t.root) == 13
    x = {c: np.array([0.1, 0.2, 0.2]) for c in m.names}
    x[15] = np.array([10.0, 10.0, 10.0])        # std_area
    x[22] = np.array([20.0, 20.0, 10.0])        # worst_radius
    # row 0: left, left (std_area < 31.68), left (worst_concavity < 0.378) -> leaf 8 (0.0)
    # row 1: right (0.2 >= 0.14781), right (worst_radius >= 16.095) -> leaf 7 (1.0)
    # row 2: right, left -> leaf 6 (0.714...)
    s = m.score(x, 3)
    np.testing.assert_allclose(s, [0.0, 0.1, 0.1 * 0.7142857142857143], rtol=1e-12)


def test_meta_validation_rules(ref_resources):
    """MetaFactory semantics: every reference fixture ModelConfig passes; typos in train.params,
    out-of-option values, non-boolean flags, non-integer counts fail with the reference's
    messages; a grid search exempts train#params#*; ModelInspector train ranges."""
    import glob
    import copy
    from shifu_amd.config.meta import validate_config
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.config.validator import ValidateResult, check_train
    files = glob.glob(os.path.join(ref_resources, "**", "ModelConfig.json"), recursive=True)
    assert len(files) >= 5
    for f in files:
        assert validate_config(ModelConfig.load(f)) == [], f
    mc = ModelConfig.load(os.path.join(ref_resources, "example/cancer-judgement/ModelStore/ModelSet1/ModelConfig.json"))
    bad = copy.deepcopy(mc)
    bad.train["params"]["Propagationn"] = "R"
    assert validate_config(bad) == ["train#params#Propagationn - not found meta info."]
    bad = copy.deepcopy(mc)
    bad.normalize["normType"] = "ZZSCALE"
    assert validate_config(bad)[0].startswith("normalize#normType - the value couldn't be found in the option")
    bad = copy.deepcopy(mc)
    bad.train["isContinuous"] = "yes"
    assert validate_config(bad) == ["train#isContinuous - the value is illegal.  Only true/false are perimited."]
    bad = copy.deepcopy(mc)
    bad.train["baggingNum"] = "two"
    assert validate_config(bad) == ["train#baggingNum - the value is not integer format."]
    grid = copy.deepcopy(mc)
    grid.train["params"]["LearningRate"] = [0.1, 0.2]
    grid.train["params"]["Whatever"] = 1
    assert validate_config(grid) == []
    r = ValidateResult()
    bad = copy.deepcopy(mc)
    bad.train["params"]["LearningRate"] = 0
    bad.train["params"]["DropoutRate"] = 1.0
    check_train(bad, r)
    assert not r and any("Learning rate" in c for c in r.causes) and any("Dropout" in c for c in r.causes)


def test_jsonio_dump_follows_symlink_and_umask(tmp_path):
    import os
    from shifu_amd.config import jsonio
    real = tmp_path / "real.json"
    jsonio.dump({"a": 1}, str(real))
    um = os.umask(0o027)
    try:
        jsonio.dump({"x": 2}, str(tmp_path / "new.json"))
    finally:
        os.umask(um)
    assert (os.stat(tmp_path / "new.json").st_mode & 0o777) == 0o640
    link = tmp_path / "link.json"
    os.symlink(real, link)
    jsonio.dump({"a": 3}, str(link))
    assert os.path.islink(link)
    assert jsonio.load(str(real))["a"] == 3
