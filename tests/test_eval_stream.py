"""Streamed (out-of-core) `eval` (steps/evaluate.py _score_eval_streamed + runtime/csrc/eval_rows.cpp):
EvalScore equals the in-memory writer's (same header / layout / row set, scores equal up to the
fp32 GEMM blocking of a different batch shape, the same descending order) and the performance
numbers agree -- single process and 2 gloo ranks (rank-local ORDER BY + native k-way merge);
host memory bounded."""
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


def _trained(tmp_path, n_rows=1500, alg="NN"):
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.steps import api
    from shifu_amd.utils.synthetic import make_model_set
    root = make_model_set(str(tmp_path), "e", alg, n_rows=n_rows, n_num=6, n_cat=2)
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    mc.train["numTrainEpochs"] = 8
    mc.train["baggingNum"] = 2
    mc.save()
    for cls in (api.InitStep, api.StatsStep, api.NormStep, api.TrainStep):
        cls(root).process()
    return root


def _mode(m, chunk_kb=None):
    from shifu_amd.config import environment
    environment.props()["shifu.eval.streaming"] = m
    if chunk_kb is not None:
        environment.props()["shifu.eval.chunkMB"] = str(chunk_kb / 1024)


def _outputs(root):
    d = os.path.join(root, "evals", "Eval1")
    p = os.path.join(d, "EvalScore")
    p = os.path.join(p, "part-00000") if os.path.isdir(p) else p
    return open(p).read(), json.load(open(os.path.join(d, "EvalPerformance.json")))


def _rank_eval(rank, world, port, root):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), SHIFU_FORCE_CPU="1")
    from shifu_amd.parallel import dist
    from shifu_amd.steps.evaluate import run_eval
    _mode("true", chunk_kb=12)
    dist.init_from_env("gloo")
    run_eval(root)
    dist.barrier()
    dist.shutdown()


@pytest.mark.parametrize("alg", ["NN", "GBT"])
def test_streamed_eval_equals_in_memory(tmp_path, monkeypatch, alg):
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    from shifu_amd.steps.evaluate import run_eval
    root = _trained(tmp_path, alg=alg)
    _mode("false")
    run_eval(root)
    text0, perf0 = _outputs(root)
    _mode("true", chunk_kb=8)
    try:
        run_eval(root)
    finally:
        _mode("auto")
    text1, perf1 = _outputs(root)
    _same(text0, text1, perf0, perf1)
    assert not os.path.exists(os.path.join(root, "evals", "Eval1", ".parts"))
    mp.start_processes(_rank_eval, args=(2, _port(), root), nprocs=2, join=True, start_method="spawn")
    text2, perf2 = _outputs(root)
    _same(text0, text2, perf0, perf2)


def _same(t0, t1, p0, p1):
    r0 = [l.split("|") for l in t0.strip().split("\n")]
    r1 = [l.split("|") for l in t1.strip().split("\n")]
    assert r0[0] == r1[0] and len(r0) == len(r1)
    j = r0[0].index("mean")
    m0 = np.array([float(r[j]) for r in r0[1:]])
    m1 = np.array([float(r[j]) for r in r1[1:]])
    np.testing.assert_allclose(m1, m0, atol=1e-3)
    assert np.all(np.diff(m1) <= 0)                       # ORDER BY score DESC
    assert sorted((r[0], r[1]) for r in r0[1:]) == sorted((r[0], r[1]) for r in r1[1:])
    for line in t1.strip().split("\n")[1:]:               # every numeric field in the writer's formats
        f = line.split("|")
        assert float(f[1]) == float(f[1]) and all(len(x.split(".")[1]) == 6 for x in f[2:j + 4])
    for k in ("areaUnderRoc", "weightedAreaUnderRoc", "areaUnderPr"):
        assert abs(p0[k] - p1[k]) < 1e-4, k


_RSS = r"""
import os, sys, json
sys.path.insert(0, {root!r})
os.environ["SHIFU_FORCE_CPU"] = "1"
from shifu_amd.config import environment
from shifu_amd.steps.evaluate import run_eval
environment.props()["shifu.eval.streaming"] = {mode!r}
environment.props()["shifu.eval.chunkMB"] = "2"
def status(key):
    for line in open("/proc/self/status"):
        if line.startswith(key):
            return int(line.split()[1])
open("/proc/self/clear_refs", "w").write("5")
base = status("VmRSS:")
run_eval({root2!r})
print(json.dumps({{"base_kb": base, "peak_kb": status("VmHWM:")}}))
"""


def _rss_growth(root, mode):
    r = subprocess.run([sys.executable, "-c", _RSS.format(root=ROOT, mode=mode, root2=root)], capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    return (res["peak_kb"] - res["base_kb"]) * 1024


def test_streamed_eval_host_memory_bounded_by_chunk(tmp_path, monkeypatch):
    """peak RSS growth of streamed eval is (nearly) flat in the data size; only the
    17 B/row numeric metric columns grow on rank 0."""
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    from shifu_amd.config.model_config import ModelConfig
    small = _trained(tmp_path / "s", n_rows=2000)
    big = str(tmp_path / "b")
    shutil.copytree(small, big)
    # same models, 3 eval sets' worth of rows: append the data file to itself
    mc = ModelConfig.load(os.path.join(big, "ModelConfig.json"))
    dp = mc.resolve(mc.evals[0].dataSet.get("dataPath"))
    files = [os.path.join(dp, f) for f in sorted(os.listdir(dp))] if os.path.isdir(dp) else [dp]
    for f in files:
        body = open(f).read()
        lines = body.splitlines(True)
        hdr = lines[0] if lines and not lines[0][:1].isdigit() and "|" in lines[0] and lines[0].split("|")[0].isalpha() else ""
        rows = "".join(lines[1:] if hdr else lines)
        with open(f, "w") as o:
            o.write(hdr + rows * 300)
    s_small, s_big = _rss_growth(small, "true"), _rss_growth(big, "true")
    m_big = _rss_growth(big, "false")
    print("eval rss growth MB: streamed small %.1f, streamed 300x %.1f, in-memory 300x %.1f"
          % (s_small / 1e6, s_big / 1e6, m_big / 1e6))
    assert s_big - s_small < 30e6, (s_small, s_big, m_big)   # 600K more rows: +17 B/row metric columns
    assert m_big - s_big > 20e6, (s_small, s_big, m_big)     # the in-memory eval grows with the data


def test_gather_and_merge_with_small_flush_buffer(tmp_path):
    """shifu_gather_lines / shifu_merge_runs stage their output in a fixed-size buffer flushed when
    full (bounded memory on the merging rank): with a 100-byte buffer the files equal the ones
    written with the default 256-MB buffer."""
    import ctypes
    from shifu_amd.ops import _native
    lib = _native.rt()
    g = np.random.default_rng(0)
    runs = []
    for r in range(3):
        n = 400 + 50 * r
        key = np.round(g.random(n), 4)
        lines = [("%d|%s|%.4f\n" % (r, "y" * int(g.integers(0, 300)), v)).encode() for v in key]
        blob = np.frombuffer(b"".join(lines), dtype=np.uint8).copy()
        ends = np.cumsum([len(l) for l in lines]).astype(np.int64)
        runs.append((blob, ends, key))

    def write(flush, tag):
        lib.shifu_eval_set_flush_bytes(flush)
        sorted_runs = []
        for i, (blob, ends, key) in enumerate(runs):
            order = np.argsort(-key, kind="stable").astype(np.int64)
            new_end = np.zeros(len(key), np.int64)
            out = str(tmp_path / f"{tag}_s{i}.bin")
            assert lib.shifu_gather_lines(blob.ctypes.data, ends.ctypes.data, order.ctypes.data, len(key),
                                          out.encode(), new_end.ctypes.data) == ends[-1]
            sorted_runs.append((np.fromfile(out, dtype=np.uint8), new_end, np.ascontiguousarray(key[order])))
        path = str(tmp_path / f"{tag}_merged")
        open(path, "w").close()
        R = len(sorted_runs)
        assert lib.shifu_merge_runs(R, (ctypes.c_void_p * R)(*[b.ctypes.data for b, _, _ in sorted_runs]),
                                    (ctypes.c_void_p * R)(*[e.ctypes.data for _, e, _ in sorted_runs]),
                                    (ctypes.c_void_p * R)(*[k.ctypes.data for _, _, k in sorted_runs]),
                                    (ctypes.c_long * R)(*[len(k) for _, _, k in sorted_runs]),
                                    path.encode()) == sum(len(k) for _, _, k in sorted_runs)
        return [open(str(tmp_path / f"{tag}_s{i}.bin"), "rb").read() for i in range(R)], open(path, "rb").read()
    try:
        big = write(256 << 20, "big")
        small = write(100, "small")
    finally:
        lib.shifu_eval_set_flush_bytes(256 << 20)
    assert small == big
    merged = big[1].decode().strip().split("\n")
    keys = [float(l.rsplit("|", 1)[1]) for l in merged]
    assert len(merged) == 1350 and keys == sorted(keys, reverse=True)
