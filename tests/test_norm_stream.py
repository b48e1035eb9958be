"""Streamed (out-of-core) `norm` (steps/norm.py _norm_one_streamed + the fused K5 NormPlan pass):
the per-rank part caches equal the in-memory NormalizedData / CleanedData -- single process and
2 gloo ranks, with and without -shuffle; bf16 GEMM-ready rows are the fp32 rows rounded to bf16
with the bias column; host memory stays bounded by the chunk size."""
import json
import os
import shutil
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _set(mode, chunk_kb=None, dtype=None):
    from shifu_amd.config import environment
    environment.props()["shifu.norm.streaming"] = mode
    if chunk_kb is not None:
        environment.props()["shifu.norm.chunkMB"] = str(chunk_kb / 1024)
    if dtype is not None:
        environment.props()["shifu.norm.dtype"] = dtype


def _model_set(tmp_path, alg, n_rows=1503):
    from shifu_amd.steps.create import run_init
    from shifu_amd.steps.stats import run_stats
    from shifu_amd.utils.synthetic import make_model_set
    a = make_model_set(str(tmp_path), "a", alg, n_rows=n_rows, n_num=6, n_cat=2)
    run_init(a)
    run_stats(a)
    return a


def _rank_norm(rank, world, port, root, shuffle):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), SHIFU_FORCE_CPU="1")
    from shifu_amd.parallel import dist
    from shifu_amd.steps.norm import run_norm
    _set("true", chunk_kb=16)
    dist.init_from_env("gloo")
    run_norm(root, shuffle=shuffle)
    dist.barrier()
    dist.shutdown()


@pytest.mark.parametrize("alg,shuffle", [("NN", False), ("NN", True), ("GBT", False), ("GBT", True)])
def test_streamed_norm_equals_in_memory(tmp_path, monkeypatch, alg, shuffle):
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    from shifu_amd.steps.base import load_dataset_cache
    from shifu_amd.steps.norm import run_norm
    a = _model_set(tmp_path, alg)
    b, c = str(tmp_path / "b"), str(tmp_path / "c")
    shutil.copytree(a, b)
    shutil.copytree(a, c)
    _set("false")
    run_norm(a, shuffle=shuffle)
    _set("true", chunk_kb=8)                    # many chunks
    run_norm(b, shuffle=shuffle)
    mp.start_processes(_rank_norm, args=(2, _port(), c, shuffle), nprocs=2, join=True, start_method="spawn")
    _set("auto")
    for sub in (["CleanedData", "NormalizedData"] if alg == "GBT" else ["NormalizedData"]):
        ma, xa = load_dataset_cache(os.path.join(a, "tmp", sub), mmap=False)
        for other in (b, c):
            mb, xb = load_dataset_cache(os.path.join(other, "tmp", sub))
            assert mb["n"] == ma["n"] and mb.get("streamed")
            assert set(xa) <= set(xb), (set(xa), set(xb))
            for k in xa:
                np.testing.assert_array_equal(np.asarray(xb[k]), xa[k], err_msg=f"{sub} {k}")
            for k in ("input_names", "input_nums", "nbins", "is_cat", "column_nums"):
                if k in ma:
                    assert mb[k] == ma[k], k


def test_streamed_norm_bf16_rows(tmp_path, monkeypatch):
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    import torch
    from shifu_amd.steps.base import load_dataset_cache
    from shifu_amd.steps.norm import run_norm
    a = _model_set(tmp_path, "NN")
    b = str(tmp_path / "b")
    shutil.copytree(a, b)
    _set("false")
    run_norm(a)
    _set("true", chunk_kb=8, dtype="bf16")
    try:
        run_norm(b)
    finally:
        _set("auto", dtype="float32")
    ma, xa = load_dataset_cache(os.path.join(a, "tmp", "NormalizedData"), mmap=False)
    mb, xb = load_dataset_cache(os.path.join(b, "tmp", "NormalizedData"))
    X = xa["X"]
    want = torch.from_numpy(X).to(torch.bfloat16).float().numpy()
    np.testing.assert_array_equal(np.asarray(xb["X"]), want)
    raw = xb["X"].raw
    assert raw.shape == (len(X), mb["x_kpad"]) and mb["x_kpad"] % 128 == 0
    assert np.all(raw[:, mb["x_width"]] == 0x3F80) and not raw[:, mb["x_width"] + 1:].any()


_RSS = r"""
import os, sys, json
sys.path.insert(0, {root!r})
os.environ["SHIFU_FORCE_CPU"] = "1"
from shifu_amd.config import environment
from shifu_amd.steps.norm import run_norm
environment.props()["shifu.norm.streaming"] = {mode!r}
environment.props()["shifu.norm.chunkMB"] = "2"
def status(key):
    for line in open("/proc/self/status"):
        if line.startswith(key):
            return int(line.split()[1])
open("/proc/self/clear_refs", "w").write("5")
base = status("VmRSS:")
run_norm({root2!r})
print(json.dumps({{"base_kb": base, "peak_kb": status("VmHWM:")}}))
"""


def _rss_growth(root, mode):
    r = subprocess.run([sys.executable, "-c", _RSS.format(root=ROOT, mode=mode, root2=root)], capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    return (res["peak_kb"] - res["base_kb"]) * 1024


def test_streamed_norm_host_memory_bounded_by_chunk(tmp_path):
    """peak RSS growth of streamed norm is flat in the data size (2 MB chunks)."""
    from shifu_amd.steps.create import run_init
    from shifu_amd.steps.stats import run_stats
    from shifu_amd.utils.synthetic import make_model_set
    roots = {}
    for n in (40_000, 120_000):
        roots[n] = make_model_set(str(tmp_path / str(n)), "m", "NN", n_rows=n, n_num=40, n_cat=2)
        run_init(roots[n])
        os.environ["SHIFU_FORCE_CPU"] = "1"
        run_stats(roots[n])
    s_small, s_big = _rss_growth(roots[40_000], "true"), _rss_growth(roots[120_000], "true")
    m_big = _rss_growth(roots[120_000], "false")
    print("norm rss growth MB: streamed 40K %.1f, streamed 120K %.1f, in-memory 120K %.1f"
          % (s_small / 1e6, s_big / 1e6, m_big / 1e6))
    assert s_big - s_small < 24e6, (s_small, s_big)
    assert s_big < 0.6 * m_big, (s_big, m_big)


def test_block_matrix_rows_upload_in_place():
    """The parser's numeric columns are rows of one block matrix; the normalize upload uses them
    in place (contiguous run, permuted gather, sliced/filtered fallback) and equals the gather."""
    import numpy as np
    import torch
    from shifu_amd.algos.normalize import _raw_matrix, _raw_matrix_dev
    from shifu_amd.data.reader import numeric_rows, parse_block, table_from_parts

    rng = np.random.default_rng(3)
    header = [f"c{i}" for i in range(6)]
    vals = rng.normal(size=(50, 6)).round(3)
    text = "\n".join("|".join("" if (r * 7 + c) % 11 == 0 else ("ab"[r % 2] if c == 2 else repr(vals[r, c]))
                              for c in range(6))
                     for r in range(50)).encode() + b"\n"
    kinds = [1, 1, 2, 1, 1, 1]
    part = parse_block(bytearray(text), "|", kinds, ["", "?"], 2)
    t = table_from_parts(header, kinds, [part])

    class CC:
        def __init__(self, name, cat=False):
            self.name, self.cat = name, cat
            self.bin_category = ["a", "b"]

        def is_categorical(self):
            return self.cat

    native = numeric_rows([t["c0"].values, t["c1"].values]) is not None
    for names in (["c3", "c4", "c5"], ["c5", "c0", "c4"], ["c1"], ["c5", "c0"]):
        cols = [CC(n) for n in names]
        if len(cols) > 1:
            cols.insert(1, CC("c2", cat=True))          # a host-side categorical row among them
        want = _raw_matrix(cols, t)
        got = _raw_matrix_dev(cols, t, torch.device("cpu")).numpy()
        np.testing.assert_array_equal(np.isnan(got), np.isnan(want))
        np.testing.assert_array_equal(np.nan_to_num(got), np.nan_to_num(want))
    if native:
        base, idx = numeric_rows([t[n].values for n in ("c4", "c0")])
        assert base.shape == (5, 50) and list(idx) == [3, 0]
    sub = t.take(np.arange(10))
    assert numeric_rows([sub["c0"].values]) is None            # filtered rows: generic path
    assert numeric_rows([t["c0"].values[:10]]) is None          # row slices are not full rows


def test_bf16rows_subset_and_device_rows():
    """Column subsets of the bf16 NormalizedData view and the bf16-bits upload (rows gathered,
    columns picked on the device) equal the host fp32 expansion."""
    import numpy as np
    import torch
    from shifu_amd.data.rowstore import Bf16Rows

    rng = np.random.default_rng(5)
    n, width, kpad = 1000, 37, 128
    x = torch.from_numpy(rng.normal(size=(n, width)).astype(np.float32)).to(torch.bfloat16)
    raw = np.zeros((n, kpad), np.uint16)
    raw[:, :width] = x.view(torch.int16).numpy().view(np.uint16)
    raw[:, width] = 0x3F80
    v = Bf16Rows(raw, width)
    full = np.asarray(v)
    np.testing.assert_array_equal(full, x.float().numpy())
    idx = [3, 0, 36, 10]
    sub = v.subset(idx)
    assert sub.shape == (n, 4)
    np.testing.assert_array_equal(np.asarray(sub), full[:, idx])
    np.testing.assert_array_equal(sub[5:9], full[5:9][:, idx])
    rows = np.sort(rng.choice(n, 300, replace=False))
    for view, want in ((v, full), (sub, full[:, idx])):
        d = view.device_rows(torch.device("cpu"), block=128)
        assert d.dtype == torch.bfloat16
        np.testing.assert_array_equal(d.float().numpy(), want)
        d = view.device_rows(torch.device("cpu"), rows=rows, block=128)
        np.testing.assert_array_equal(d.float().numpy(), want[rows])
        # several row sets from one pass (train / validation split), an empty set included
        rest = np.setdiff1d(np.arange(n), rows)
        da, db, de, dn = view.device_rows_multi(torch.device("cpu"), [rows, rest, rows[:0], None], block=128)
        np.testing.assert_array_equal(da.float().numpy(), want[rows])
        np.testing.assert_array_equal(db.float().numpy(), want[rest])
        assert de.shape == (0, want.shape[1])
        np.testing.assert_array_equal(dn.float().numpy(), want)
    np.testing.assert_array_equal(np.asarray(sub.subset([1, 2])), full[:, [0, 36]])


@pytest.mark.gpu
def test_bf16_cache_varsel_train_gpu_match_host_expansion(tmp_path, monkeypatch):
    """varsel (SE) and NN train read the bf16 NormalizedData as bf16 bits uploaded to HBM
    (Bf16Rows.device_rows); the result equals the host fp32 expansion route."""
    import torch
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.data import rowstore
    from shifu_amd.steps.norm import run_norm
    from shifu_amd.steps.train import run_train
    from shifu_amd.steps.varsel import run_varsel
    a = _model_set(tmp_path, "NN", n_rows=6000)
    mc = ModelConfig.load(os.path.join(a, "ModelConfig.json"))
    mc.varSelect["filterBy"], mc.varSelect["filterNum"] = "SE", 5
    mc.varSelect["autoFilterEnable"] = False
    mc.train["numTrainEpochs"], mc.train["baggingNum"] = 6, 1
    mc.save()
    _set("true", chunk_kb=64, dtype="bf16")
    try:
        run_norm(a)
    finally:
        _set("auto", dtype="float32")
    b = str(tmp_path / "b")
    shutil.copytree(a, b)
    calls = []
    orig = rowstore.Bf16Rows.device_rows

    orig_m = rowstore.Bf16Rows.device_rows_multi

    def spy(self, device, rows=None, block=1 << 18):
        calls.append(len(self) if rows is None else len(rows))
        return orig(self, device, rows, block)

    def spy_m(self, device, row_sets, block=1 << 18):
        calls.extend(len(self) if r is None else len(r) for r in row_sets)
        return orig_m(self, device, row_sets, block)
    monkeypatch.setattr(rowstore.Bf16Rows, "device_rows", spy)
    monkeypatch.setattr(rowstore.Bf16Rows, "device_rows_multi", spy_m)
    run_varsel(a)
    run_train(a)
    assert len(calls) >= 2, calls                       # varsel rows + train rows went as bf16

    def host(self, device, rows=None, block=1 << 18):   # the previous route: fp32 on the host
        x = np.asarray(self) if rows is None else self[rows]
        return torch.from_numpy(np.ascontiguousarray(x)).to(device, torch.bfloat16)
    monkeypatch.setattr(rowstore.Bf16Rows, "device_rows", host)
    monkeypatch.setattr(rowstore.Bf16Rows, "device_rows_multi",
                        lambda self, device, row_sets, block=1 << 18: [host(self, device, r) for r in row_sets])
    run_varsel(b)
    run_train(b)
    sa = open(os.path.join(a, "varsel", "se.0")).read().split("\n")
    sb = open(os.path.join(b, "varsel", "se.0")).read().split("\n")
    assert [l.split("\t")[:2] for l in sa] == [l.split("\t")[:2] for l in sb]
    from shifu_amd.formats.nn_format import read_encog
    na, nb = read_encog(os.path.join(a, "models", "model0.nn")), read_encog(os.path.join(b, "models", "model0.nn"))
    for wa, wb in zip(na.weights, nb.weights):
        np.testing.assert_allclose(wa, wb, rtol=0, atol=1e-6)


def _set_norm_type(root, norm_type):
    from shifu_amd.config.model_config import ModelConfig
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    mc.normalize["normType"] = norm_type
    mc.save()


@pytest.mark.parametrize("norm_type", ["ONEHOT", "ZSCALE_ONEHOT"])
def test_streamed_gbt_onehot_norm_equals_in_memory(tmp_path, monkeypatch, norm_type):
    """Tree model + one-hot norm types (host one-hot columns beside a codes-only K5 launch)."""
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    _check_gbt_onehot(tmp_path, norm_type)


@pytest.mark.gpu
@pytest.mark.parametrize("norm_type,alg", [("ONEHOT", "GBT"), ("ZSCALE_ONEHOT", "GBT"), ("ONEHOT", "NN"),
                                           ("ZSCALE_ONEHOT", "NN")])
def test_streamed_gbt_onehot_norm_gpu_equals_in_memory(tmp_path, norm_type, alg):
    """the codes-only norm_codes_kernel launch (ip == nullptr) of a streamed GBT norm
    runs on the GPU and equals the in-memory CleanedData; the one-hot columns come from the K5
    one-hot kernel (shifu_onehot) and equal the host expansion."""
    import torch
    assert torch.cuda.is_available()
    _check_gbt_onehot(tmp_path, norm_type, alg)


def _check_gbt_onehot(tmp_path, norm_type, alg="GBT"):
    from shifu_amd.steps.base import load_dataset_cache
    from shifu_amd.steps.norm import run_norm
    a = _model_set(tmp_path, alg)
    _set_norm_type(a, norm_type)
    b = str(tmp_path / "b")
    shutil.copytree(a, b)
    _set("false")
    run_norm(a)
    _set("true", chunk_kb=8)
    try:
        run_norm(b)
    finally:
        _set("auto")
    for sub in (("CleanedData", "NormalizedData") if alg == "GBT" else ("NormalizedData",)):
        ma, xa = load_dataset_cache(os.path.join(a, "tmp", sub), mmap=False)
        mb, xb = load_dataset_cache(os.path.join(b, "tmp", sub))
        assert mb["n"] == ma["n"] and mb.get("streamed")
        for k in xa:
            np.testing.assert_array_equal(np.asarray(xb[k]), xa[k], err_msg=f"{norm_type} {sub} {k}")


@pytest.mark.gpu
def test_bf16rows_device_rows_staged_equals_pageable(monkeypatch):
    """Bf16Rows.device_rows: the page-locked multi-thread staging (COPY_THREADS > 0) uploads the
    same rows / columns as the default pageable path (row gathers and column subsets included)."""
    import numpy as np
    import torch
    from shifu_amd.data.rowstore import Bf16Rows
    rng = np.random.default_rng(9)
    n, width, kpad = 5000, 37, 128
    raw = rng.integers(0, 1 << 15, size=(n, kpad)).astype(np.uint16)
    rows = np.sort(rng.choice(n, 1700, replace=False))
    dev = torch.device("cuda", 0)
    for view in (Bf16Rows(raw, width), Bf16Rows(raw, width).subset([3, 0, 36, 10])):
        monkeypatch.setattr(Bf16Rows, "COPY_THREADS", 0)
        a = view.device_rows(dev, block=1024)
        b = view.device_rows(dev, rows=rows, block=1024)
        monkeypatch.setattr(Bf16Rows, "COPY_THREADS", 4)
        assert torch.equal(view.device_rows(dev, block=1024).view(torch.int16), a.view(torch.int16))
        assert torch.equal(view.device_rows(dev, rows=rows, block=1024).view(torch.int16), b.view(torch.int16))
