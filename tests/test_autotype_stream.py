"""Streamed, data-parallel auto-type (`init` with dataSet.autoType; algos/autotype.py +
runtime/csrc/autotype_scan.cpp) against a brute-force Python model of the reference mapper
(AutoTypeDistinctCountMapper.java:134-219: rows with an invalid trimmed tag skipped, the data set
filter applied, per column count / missing-or-invalid (lower-cased field in the missing list) /
Double.parseDouble-valid counts, distinct values, first-seen items), 2-rank gloo equality, the
HyperLogLog path above the exact cap, and bounded host memory on a large file."""
import json
import os
import random
import shutil
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from shifu_amd.config.model_config import ModelConfig
from shifu_amd.utils.synthetic import make_model_set


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _java_double(s: str) -> bool:
    t = s.strip()
    if not t:
        return False
    u = t.lstrip("+-")
    if u in ("NaN", "Infinity"):
        return True
    if t[-1] in "dDfF":
        t = t[:-1]
    try:
        float(t)
    except ValueError:
        return False
    return "x" not in t.lower() and "n" not in t.lower()       # no hex floats / nan / inf spellings


def _write_data(root, rng, n):
    """A header + n rows: numeric, string, 0/1, mixed, missing-token and short-row columns, some
    invalid tags, blank lines and CRLF endings."""
    hdr = ["tag", "num", "str", "bin", "mixed", "miss", "wide", "blank"]
    lines = ["|".join(hdr)]
    for i in range(n):
        tag = rng.choice(["1", "0", " 1 ", "0 ", "x"])
        row = [tag, f"{rng.gauss(0, 5):.3f}", rng.choice(["a", "b", "c", "dd", "e f"]), rng.choice(["0", "1"]),
               rng.choice(["1.5", "2e3", "abc", "1.0d", "-7", "NaN", " 4 "]),
               rng.choice(["NULL", "null", "?", "", "3", "Null"]), f"w{rng.randint(0, 50)}",
               rng.choice([" ", "x", "y", "1"])]
        if rng.random() < 0.02:
            row = row[:4]                                    # short row
        lines.append("|".join(row))
        if rng.random() < 0.01:
            lines.append("   ")
    eol = "\r\n" if rng.random() < 0.5 else "\n"
    d = os.path.join(root, "data")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "part-0"), "w", newline="") as f:
        f.write(eol.join(lines) + eol)
    return hdr


def _model(path, hdr, tags, missing, filt=None):
    stats = {h: dict(count=0, invalid=0, valid=0, vals=set()) for h in hdr}
    with open(path, newline="") as f:
        rows = f.read().replace("\r\n", "\n").split("\n")[1:]
    for ln in rows:
        if not ln.strip(" \t\r"):
            continue
        u = ln.split("|")
        if u[0].strip() not in tags:
            continue
        if filt is not None and not filt(u):
            continue
        for h, v in zip(hdr, u):
            st = stats[h]
            st["count"] += 1
            if v.lower() in missing:
                st["invalid"] += 1
                continue
            st["vals"].add(v)
            st["valid"] += _java_double(v)
    return stats


def _setup(tmp_path, n=3000, seed=3):
    rng = random.Random(seed)
    root = make_model_set(str(tmp_path), "m", "NN", n_rows=200)
    hdr = _write_data(root, rng, n)
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    mc.dataSet["dataPath"] = os.path.join(root, "data")
    mc.dataSet["headerPath"] = None
    mc.dataSet["targetColumnName"] = "tag"
    mc.dataSet["posTags"] = ["1"]
    mc.dataSet["negTags"] = ["0"]
    mc.dataSet["autoType"] = True
    mc.dataSet["autoTypeThreshold"] = 60
    mc.dataSet["weightColumnName"] = None
    mc.dataSet["missingOrInvalidValues"] = ["", "?", "null"]
    mc.save()
    for fn in ("meta.column.names", "categorical.column.names", "forceselect.column.names",
               "forceremove.column.names"):
        open(os.path.join(root, "columns", fn), "w").close()
    return root, hdr


def test_scan_matches_mapper_model(tmp_path, monkeypatch):
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    from shifu_amd.algos import autotype
    root, hdr = _setup(tmp_path)
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    ref = _model(os.path.join(root, "data", "part-0"), hdr, {"1", "0"}, {"", "?", "null"})
    for block in (1 << 30, 4096):                           # one block / many blocks and threads
        st = autotype.scan(mc, hdr, list(range(1, len(hdr))), block_bytes=block, nthreads=4)
        for c in range(1, len(hdr)):
            r, s = ref[hdr[c]], st[c]
            assert (s.count, s.invalid, s.validnum) == (r["count"], r["invalid"], r["valid"]), hdr[c]
            assert s.distinct == len(r["vals"]) and s.exact, hdr[c]
            # 21 first-seen values per scanner thread (the mapper's cap), at most 200 merged
            assert set(s.items) <= r["vals"] and min(len(r["vals"]), 21) <= len(s.items) <= 200, hdr[c]


def test_filter_expression_applies(tmp_path, monkeypatch):
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    from shifu_amd.algos import autotype
    root, hdr = _setup(tmp_path, n=1500, seed=5)
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    mc.dataSet["filterExpressions"] = "bin == 1"
    ref = _model(os.path.join(root, "data", "part-0"), hdr, {"1", "0"}, {"", "?", "null"},
                 filt=lambda u: len(u) > 3 and u[3].strip() == "1")
    st = autotype.scan(mc, hdr, list(range(1, len(hdr))))
    for c in range(1, len(hdr)):
        assert st[c].count == ref[hdr[c]]["count"], hdr[c]
        assert st[c].distinct == len(ref[hdr[c]]["vals"]), hdr[c]


@pytest.mark.parametrize("rule", ["reference", "ratio"])
def test_init_types(tmp_path, monkeypatch, rule):
    """reference rule (InitModelProcessor.setCategoricalColumnsAndDistinctAccount :181-219, with
    isDoubleFrequentVariable :243-254 as written): binary columns numeric, otherwise categorical
    exactly when a sampled item is whitespace-only; ratio rule: the documented valid-double ratio."""
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    from shifu_amd.config import environment
    from shifu_amd.steps.create import run_init
    monkeypatch.setitem(environment.props(), "shifu.autoType.rule", rule)
    root, hdr = _setup(tmp_path)
    run_init(root)
    cc = {c["columnName"]: c for c in json.load(open(os.path.join(root, "ColumnConfig.json")))}
    assert cc["num"]["columnType"] == "N" and cc["bin"]["columnType"] == "N"
    assert cc["miss"]["columnType"] == "N"        # the only non-missing value is "3"
    if rule == "ratio":
        assert cc["str"]["columnType"] == "C" and cc["wide"]["columnType"] == "C"
    else:
        assert cc["str"]["columnType"] == "N" and cc["wide"]["columnType"] == "N"
        assert cc["blank"]["columnType"] == "C"      # " " is a sampled item
    assert cc["str"]["columnStats"]["distinctCount"] == 5 and cc["bin"]["columnStats"]["distinctCount"] == 2


def test_hll_above_exact_cap(tmp_path, monkeypatch):
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    from shifu_amd.algos import autotype
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
    st = autotype.scan(mc, ["tag", "id", "lo"], [1, 2])
    assert not st[1].exact and abs(st[1].distinct - n) / n < 0.03
    assert st[2].exact and st[2].distinct == 37


def _rank_init(rank, world, port, root):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), SHIFU_FORCE_CPU="1")
    from shifu_amd.parallel import dist
    from shifu_amd.steps.create import run_init
    dist.init_from_env("gloo")
    run_init(root)
    dist.barrier()
    dist.shutdown()


@pytest.mark.parametrize("world", [2, 4])
def test_ranks_match_single_process(tmp_path, world, monkeypatch):
    """Per-rank byte ranges (a rank may hold no complete line at world 4 on a small file) merged
    over gloo: the same ColumnConfig as one process."""
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    from shifu_amd.steps.create import run_init
    a, _ = _setup(tmp_path, n=2501, seed=7)
    b = str(tmp_path / "b")
    shutil.copytree(a, b)
    mc = ModelConfig.load(os.path.join(b, "ModelConfig.json"))
    mc.dataSet["dataPath"] = os.path.join(b, "data")
    mc.save()
    run_init(a)
    mp.start_processes(_rank_init, args=(world, _port(), b), nprocs=world, join=True, start_method="spawn")
    ca = json.load(open(os.path.join(a, "ColumnConfig.json")))
    cb = json.load(open(os.path.join(b, "ColumnConfig.json")))
    for x, y in zip(ca, cb):
        assert x["columnType"] == y["columnType"], x["columnName"]
        assert x["columnStats"].get("distinctCount") == y["columnStats"].get("distinctCount"), x["columnName"]


def test_host_memory_bounded(tmp_path):
    """A ~260 MB text file: the scan's peak RSS stays far below the data size (blocks of 16 MB)."""
    root = make_model_set(str(tmp_path), "r", "NN", n_rows=100)
    d = os.path.join(root, "big")
    os.makedirs(d)
    rng = np.random.default_rng(0)
    cols = 40
    with open(os.path.join(d, "p0"), "w") as f:
        f.write("|".join(["tag"] + [f"c{j}" for j in range(cols)]) + "\n")
        blk = "\n".join("|".join([str(i % 2)] + [f"{v:.4f}" for v in rng.normal(size=cols)]) for i in range(20000))
        for _ in range(43):
            f.write(blk + "\n")
    size = os.path.getsize(os.path.join(d, "p0"))
    code = f"""
import resource, sys
sys.path.insert(0, {os.path.dirname(os.path.dirname(os.path.abspath(__file__)))!r})
from shifu_amd.config.model_config import ModelConfig
from shifu_amd.algos import autotype
mc = ModelConfig.load({os.path.join(root, "ModelConfig.json")!r})
for k, v in dict(dataPath={d!r}, headerPath=None, targetColumnName="tag", posTags=["1"], negTags=["0"]).items():
    mc.dataSet[k] = v
hdr = ["tag"] + ["c%d" % j for j in range({cols})]
before = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
st = autotype.scan(mc, hdr, list(range(1, len(hdr))), block_bytes=16 << 20)
assert st[1].count == 860000, st[1].count
print(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss - before)
"""
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600,
                         env=dict(os.environ, SHIFU_FORCE_CPU="1"))
    assert out.returncode == 0, out.stderr[-2000:]
    grew_kb = int(out.stdout.strip().splitlines()[-1])
    assert grew_kb * 1024 < size * 0.6, (grew_kb, size)
