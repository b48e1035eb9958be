"""Streamed per-rank row joins (data/join.py + runtime/csrc/eval_rows.cpp shifu_join_lines):
the native line join against a Python model (CRLF, blank, short and long rows, multi-byte
delimiters), ``stream_join`` over many blocks and 2 gloo ranks (parts in rank order == one
process), ``encode`` against the in-memory leaf-path encoder, the combo score join against a
direct ModelRunner score, and bounded host memory on a large file."""
import os
import random
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

DS = "example/cancer-judgement/DataStore"


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model_join(text: str, sep: str, nf: int, suffixes: list) -> str:
    out, i = [], 0
    for ln in text.split("\n"):
        if not ln.strip(" \t\r"):
            continue
        if ln.endswith("\r"):
            ln = ln[:-1]
        f = ln.split(sep)[:nf]
        f += [""] * (nf - len(f))
        out.append(sep.join(f) + sep + suffixes[i])
        i += 1
    assert i == len(suffixes)
    return "".join(x + "\n" for x in out)


@pytest.mark.parametrize("sep", ["|", ",", "::"])
def test_join_lines_matches_model(sep):
    from shifu_amd.data.join import DICT, FIXED6, format_fields, join_block
    rng = random.Random(1)
    lines = []
    for i in range(500):
        k = rng.choice([3, 5, 5, 5, 7])
        lines.append(sep.join(rng.choice(["a", "", " b ", "1.5", "x y"]) for _ in range(k)))
        if rng.random() < 0.05:
            lines.append(rng.choice(["", "  ", "\t", "\r"]))
    eol = "\r\n" if sep == "," else "\n"
    text = eol.join(lines) + eol
    n = sum(1 for ln in text.split("\n") if ln.strip(" \t\r"))
    v = np.random.default_rng(0).normal(size=n) * 1000
    codes = np.random.default_rng(1).integers(-1, 3, size=n).astype(np.int32)
    suffix, ends = format_fields([(FIXED6, v), (DICT, codes, ["LLR", "R", "LRRLLR"])], n, sep)
    got = bytes(join_block(text.encode(), sep, 5, suffix, ends, n, nthreads=1)).decode()
    assert bytes(join_block(text.encode() * 300, sep, 5, np.tile(np.asarray(suffix), 300),
                            np.concatenate([ends + k * ends[-1] for k in range(300)]), n * 300, nthreads=8)) \
        == got.encode() * 300
    sfx = [f"{x:.6f}{sep}{['LLR', 'R', 'LRRLLR'][c] if c >= 0 else ''}" for x, c in zip(v, codes)]
    assert got == _model_join(text, sep, 5, sfx)
    with pytest.raises(RuntimeError):
        join_block(text.encode(), sep, 5, suffix, ends, n - 1)


def _write_set(d, rng, nfiles=3, rows=700):
    os.makedirs(d, exist_ok=True)
    hdr = ["tag", "a", "b", "c"]
    with open(os.path.join(d, ".pig_header"), "w") as f:
        f.write("|".join(hdr) + "\n")
    for k in range(nfiles):
        with open(os.path.join(d, f"part-{k}"), "w") as f:
            for i in range(rows):
                r = [str(rng.randint(0, 1)), f"{rng.gauss(0, 3):.4f}", rng.choice(["u", "v", ""]), str(i)]
                if rng.random() < 0.03:
                    r = r[:2]
                f.write("|".join(r) + "\n")
                if rng.random() < 0.01:
                    f.write("\n")
    return hdr


def _plan(d):
    from shifu_amd.data.purifier import DatasetPlan
    from shifu_amd.data.reader import column_kinds
    hdr = open(os.path.join(d, ".pig_header")).read().strip().split("|")
    plan = DatasetPlan(data_path=d, delim="|", header=hdr, skip_header_line=False, target=None, weight=None,
                       filt=None, nums=["a"], strs=["b"], seg_names=[], seg_exprs=[], missing=["", "?"])
    return plan, column_kinds(hdr, ["a"], ["b"])


def _compute(table, n):
    from shifu_amd.data.join import DICT, FIXED6
    a = table["a"].numeric()
    b = table["b"]
    return [(FIXED6, np.where(np.isnan(a), -1.0, a * 2)), (DICT, b.values, b.dictionary)]


def _expected(d, hdr):
    out = []
    for k in range(3):
        for ln in open(os.path.join(d, f"part-{k}")).read().split("\n"):
            if not ln.strip():
                continue
            f = ln.split("|")
            f += [""] * (len(hdr) - len(f))
            a = float(f[1]) if f[1] else float("nan")
            out.append("|".join(f + [f"{(-1.0 if a != a else a * 2):.6f}", f[2]]))
    return out


def test_stream_join_blocks(tmp_path):
    from shifu_amd.data.join import stream_join
    d = str(tmp_path / "data")
    hdr = _write_set(d, random.Random(4))
    plan, kinds = _plan(d)
    for block in (1 << 30, 2048):
        out = str(tmp_path / f"out{block}")
        n = stream_join(plan, out, ["a2", "b2"], kinds, _compute, block_bytes=block)
        got = open(os.path.join(out, "part-00000")).read().splitlines()
        assert got == _expected(d, hdr) and n == len(got)
        assert open(os.path.join(out, ".pig_header")).read().strip() == "tag|a|b|c|a2|b2"


def _rank_join(rank, world, port, d, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), SHIFU_FORCE_CPU="1")
    from shifu_amd.data.join import stream_join
    from shifu_amd.parallel import dist
    dist.init_from_env("gloo")
    plan, kinds = _plan(d)
    stream_join(plan, out, ["a2", "b2"], kinds, _compute, rank, world, block_bytes=4096)
    dist.shutdown()


@pytest.mark.parametrize("world", [2, 4])
def test_stream_join_ranks(tmp_path, world):
    d = str(tmp_path / "data")
    hdr = _write_set(d, random.Random(9))
    out = str(tmp_path / "out")
    mp.start_processes(_rank_join, args=(world, _port(), d, out), nprocs=world, join=True, start_method="spawn")
    parts = sorted(f for f in os.listdir(out) if f.startswith("part-"))
    assert parts == [f"part-{r:05d}" for r in range(world)]
    got = []
    for p in parts:
        got += open(os.path.join(out, p)).read().splitlines()
    assert got == _expected(d, hdr)


@pytest.fixture
def cj(tmp_path, ref_resources, monkeypatch):
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    from shifu_amd.cli import main
    from shifu_amd.config.model_config import ModelConfig
    monkeypatch.chdir(tmp_path)
    assert main(["new", "cj", "-t", "GBT"]) == 0
    monkeypatch.chdir(tmp_path / "cj")
    R = os.path.join(ref_resources, DS)
    mc = ModelConfig.load("ModelConfig.json")
    mc.dataSet["dataPath"] = R + "/DataSet1"
    mc.dataSet["headerPath"] = R + "/DataSet1/.pig_header"
    mc.evals[0].dataSet["dataPath"] = R + "/EvalSet1"
    mc.evals[0].dataSet["headerPath"] = R + "/EvalSet1/.pig_header"
    mc.train["baggingNum"] = 1
    mc.train["params"] = {"TreeNum": 5, "MaxDepth": 3, "LearningRate": 0.1, "Loss": "squared",
                          "Impurity": "variance", "FeatureSubsetStrategy": "ALL", "MinInstancesPerNode": 5}
    mc.save()
    for v in ("init", "stats", "varsel", "norm", "train"):
        assert main([v]) == 0, v
    return tmp_path / "cj"


def _raw_lines(path_dir):
    from shifu_amd.data.reader import list_data_files
    out = []
    for f in list_data_files(path_dir):
        for ln in open(f).read().split("\n"):
            if ln.strip(" \t\r"):
                out.append(ln.rstrip("\r"))
    return out


def test_encode_matches_in_memory(cj):
    from shifu_amd.cli import main
    from shifu_amd.data.reader import read_header, read_table
    from shifu_amd.formats.tree_format import read_tree_model
    from shifu_amd.scoring.tree_ensemble import TreeScorer
    from shifu_amd.steps.base import ModelSet
    assert main(["encode"]) == 0
    ms = ModelSet(".")
    mc = ms.mc
    scorer = TreeScorer(read_tree_model("models/model0.gbt"), "cpu")
    m = scorer.model
    data = mc.resolve(mc.dataSet["dataPath"])
    header = read_header(mc.resolve(mc.dataSet["headerPath"]), "|", data, "|")
    num = {m.names[c] for c in m.names if c not in m.categories}
    tab = read_table(data, header, "|", numeric=[h for h in header if h in num],
                     strings=[h for h in header if h not in num], missing=mc.missing_values)
    codes = scorer.encode(tab, 3)
    raw = _raw_lines(data)
    want = ["|".join(raw[i].split("|")[:len(header)] + list(codes[i])) for i in range(len(raw))]
    out = ms.pf.encoded_train_data
    got = open(os.path.join(out, "part-00000")).read().splitlines()
    assert got == want
    hdr = open(os.path.join(out, ".pig_header")).read().strip().split("|")
    assert hdr == list(header) + [f"tree_vars_{i}" for i in range(5)]


def test_combo_join_scores(cj):
    from shifu_amd.data.reader import read_header, read_table
    from shifu_amd.scoring.model_runner import ModelRunner
    from shifu_amd.steps.base import ModelSet
    from shifu_amd.steps.combo import _join_scores
    ms = ModelSet(".")
    mc = ms.mc
    out = os.path.join(str(cj), "joined")
    delim = _join_scores([("sub0", ms), ("sub1", ms)], [mc.dataSet, mc.dataSet], out)
    assert delim == "|"
    data = mc.resolve(mc.dataSet["dataPath"])
    header = read_header(mc.resolve(mc.dataSet["headerPath"]), "|", data, "|")
    r = ModelRunner(mc, ms.ccs, ms.pf.models_dir)
    need = r.raw_columns()
    cats = {c.name for c in ms.ccs if c.is_categorical()}
    t = read_table(data, header, "|", numeric=[h for h in header if h in need and h not in cats],
                   strings=[h for h in header if h not in need or h in cats], missing=mc.missing_values)
    s = r.score(t, 1000.0)["mean"]
    raw = _raw_lines(data)
    want = ["|".join(raw[i].split("|")[:len(header)] + [f"{s[i]:.6f}", f"{s[i]:.6f}"]) for i in range(len(raw))]
    assert open(os.path.join(out, "part-00000")).read().splitlines() == want
    assert open(os.path.join(out, ".pig_header")).read().strip().split("|")[-2:] == ["sub0_score", "sub1_score"]


def test_join_host_memory_bounded(tmp_path):
    """~300 MB of text joined in 32 MB blocks: peak RSS growth far below the data size."""
    d = tmp_path / "big"
    d.mkdir()
    rng = np.random.default_rng(0)
    cols = 40
    with open(d / ".pig_header", "w") as f:
        f.write("|".join(["tag", "a", "b"] + [f"c{j}" for j in range(cols)]) + "\n")
    with open(d / "p0", "w") as f:
        blk = "\n".join("|".join([str(i % 2), f"{i * 0.5}", "s"] + [f"{v:.4f}" for v in rng.normal(size=cols)])
                        for i in range(20000))
        for _ in range(43):
            f.write(blk + "\n")
    size = os.path.getsize(d / "p0")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = f"""
import resource, sys
sys.path.insert(0, {repo!r})
sys.path.insert(0, {os.path.join(repo, 'tests')!r})
import numpy as np
from test_join_stream import _plan, _compute
from shifu_amd.data.join import stream_join
plan, kinds = _plan({str(d)!r})
before = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
n = stream_join(plan, {str(tmp_path / 'out')!r}, ["a2", "b2"], kinds, _compute, block_bytes=32 << 20)
assert n == 860000, n
print(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss - before)
"""
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600,
                         env=dict(os.environ, SHIFU_FORCE_CPU="1"))
    assert out.returncode == 0, out.stderr[-2000:]
    grew_kb = int(out.stdout.strip().splitlines()[-1])
    assert grew_kb * 1024 < size * 0.5, (grew_kb, size)
    assert os.path.getsize(tmp_path / "out" / "part-00000") > size


@pytest.fixture
def cj_gpu(tmp_path, monkeypatch):
    """A synthetic GBT model set trained on the GPU (the join's scorers then run there)."""
    from shifu_amd.cli import main
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.utils.synthetic import make_model_set
    root = make_model_set(str(tmp_path), "g", "GBT", n_rows=4000, n_num=8, n_cat=2)
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    mc.train["baggingNum"] = 1
    mc.train["params"] = {"TreeNum": 5, "MaxDepth": 3, "LearningRate": 0.1, "Loss": "squared",
                          "Impurity": "variance", "FeatureSubsetStrategy": "ALL", "MinInstancesPerNode": 5}
    mc.save()
    monkeypatch.chdir(root)
    for v in ("init", "stats", "norm", "train"):
        assert main([v]) == 0, v
    return root


@pytest.mark.gpu
def test_encode_and_combo_join_on_gpu(cj_gpu):
    """encode (HIP tree walk) and the combo score join (device scoring) on the GPU equal the CPU
    leaf paths exactly and the CPU scores within fp32 rounding."""
    from shifu_amd.cli import main
    from shifu_amd.data.reader import read_header, read_table
    from shifu_amd.formats.tree_format import read_tree_model
    from shifu_amd.scoring.model_runner import ModelRunner
    from shifu_amd.scoring.tree_ensemble import TreeScorer
    from shifu_amd.steps.base import ModelSet
    from shifu_amd.steps.combo import _join_scores
    assert main(["encode"]) == 0
    ms = ModelSet(".")
    mc = ms.mc
    data = mc.resolve(mc.dataSet["dataPath"])
    header = read_header(mc.resolve(mc.dataSet["headerPath"]), "|", data, "|")
    scorer = TreeScorer(read_tree_model("models/model0.gbt"), "cpu")
    m = scorer.model
    num = {m.names[c] for c in m.names if c not in m.categories}
    tab = read_table(data, header, "|", numeric=[h for h in header if h in num],
                     strings=[h for h in header if h not in num], missing=mc.missing_values)
    codes = scorer.encode(tab, 3)
    raw = _raw_lines(data)
    want = ["|".join(raw[i].split("|")[:len(header)] + list(codes[i])) for i in range(len(raw))]
    assert open(os.path.join(ms.pf.encoded_train_data, "part-00000")).read().splitlines() == want
    out = os.path.join(str(cj_gpu), "joined")
    _join_scores([("sub0", ms)], [mc.dataSet], out)
    r = ModelRunner(mc, ms.ccs, ms.pf.models_dir, device="cpu")
    need = r.raw_columns()
    cats = {c.name for c in ms.ccs if c.is_categorical()}
    t = read_table(data, header, "|", numeric=[h for h in header if h in need and h not in cats],
                   strings=[h for h in header if h not in need or h in cats], missing=mc.missing_values)
    s = r.score(t, 1000.0)["mean"]
    got = open(os.path.join(out, "part-00000")).read().splitlines()
    assert len(got) == len(raw)
    for i, line in enumerate(got):
        f = line.split("|")
        assert f[:-1] == raw[i].split("|")[:len(header)]
        assert abs(float(f[-1]) - s[i]) < 2e-3
