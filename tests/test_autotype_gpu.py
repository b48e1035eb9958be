"""init -autotype on the device (ops/csrc/autotype_kernels.hip + algos/autotype._scan_gpu) against
the host scanner (runtime/csrc/autotype_scan.cpp) on the same files: identical counts / missing /
valid-number counts, distinct counts and exact flags, the same sketch above the exact cap, and the
same ColumnConfig types from `init`.  Items: the device keeps each column's first distinct values
in row order, the host scanner 21 per thread -- compared as sets where both hold every value."""
import json
import os
import random

import pytest

from shifu_amd.config.model_config import ModelConfig
from shifu_amd.utils.synthetic import make_model_set
from tests.test_autotype_stream import _setup

pytestmark = pytest.mark.gpu


def _scan(mc, hdr, mode, monkeypatch, **kw):
    from shifu_amd.algos import autotype
    from shifu_amd.config import environment
    monkeypatch.setitem(environment.props(), "shifu.autoType.gpu", mode)
    autotype.STATS.clear()
    st = autotype.scan(mc, hdr, list(range(1, len(hdr))), **kw)
    return st, bool(autotype.STATS.get("gpu"))


@pytest.mark.parametrize("block", [1 << 30, 64 << 10])
def test_gpu_scan_equals_host_scanner(tmp_path, monkeypatch, block):
    root, hdr = _setup(tmp_path, n=4000, seed=11)
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    host, g0 = _scan(mc, hdr, "false", monkeypatch, block_bytes=block)
    dev, g1 = _scan(mc, hdr, "true", monkeypatch, block_bytes=block)
    assert g1 and not g0
    for c in range(1, len(hdr)):
        h, d = host[c], dev[c]
        assert (d.count, d.invalid, d.validnum, d.distinct, d.exact) == \
               (h.count, h.invalid, h.validnum, h.distinct, h.exact), hdr[c]
        if h.distinct <= 21:                       # both hold every distinct value
            assert set(d.items) == set(h.items), hdr[c]
        else:
            assert len(d.items) == min(200, h.distinct), hdr[c]


def test_gpu_scan_hll_above_cap(tmp_path, monkeypatch):
    root = make_model_set(str(tmp_path), "h", "NN", n_rows=100)
    d = os.path.join(root, "big")
    os.makedirs(d)
    n = 60000
    with open(os.path.join(d, "p0"), "w") as f:
        f.write("tag|id|lo\n")
        for i in range(n):
            f.write(f"{i % 2}|id{i * 7919 % 1000003}|{i % 37}\n")
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    for k, v in dict(dataPath=d, headerPath=None, targetColumnName="tag", posTags=["1"], negTags=["0"]).items():
        mc.dataSet[k] = v
    host, _ = _scan(mc, ["tag", "id", "lo"], "false", monkeypatch, block_bytes=256 << 10)
    dev, g = _scan(mc, ["tag", "id", "lo"], "true", monkeypatch, block_bytes=256 << 10)
    assert g
    assert not dev[1].exact and dev[1].distinct == host[1].distinct      # same hashes -> same registers
    assert dev[2].exact and dev[2].distinct == 37 and set(dev[2].items) == {str(k) for k in range(37)}


@pytest.mark.parametrize("rule", ["reference", "ratio"])
def test_gpu_init_types_equal_host(tmp_path, monkeypatch, rule):
    from shifu_amd.config import environment
    from shifu_amd.steps.create import run_init
    monkeypatch.setitem(environment.props(), "shifu.autoType.rule", rule)
    out = {}
    for mode in ("false", "true"):
        root, hdr = _setup(tmp_path / mode, n=3000, seed=3)
        monkeypatch.setitem(environment.props(), "shifu.autoType.gpu", mode)
        run_init(root)
        out[mode] = {c["columnName"]: (c["columnType"], c["columnStats"]["distinctCount"])
                     for c in json.load(open(os.path.join(root, "ColumnConfig.json")))}
    assert out["true"] == out["false"]
