"""Streamed stats (algos/stats_stream.py + data/stream.py): per-rank byte ranges partition the rows
exactly; stats over tiny row chunks (many passes, no device cache) write the same ColumnConfig as
the in-memory pass; host memory stays bounded by the chunk size."""
import gzip
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write(path, lines, trailing_nl=True):
    with open(path, "w") as f:
        f.write("\n".join(lines) + ("\n" if trailing_nl else ""))


@pytest.mark.parametrize("world", [1, 2, 3, 7])
@pytest.mark.parametrize("chunk", [7, 64, 1 << 20])
def test_byte_ranges_partition_rows(tmp_path, world, chunk):
    from shifu_amd.data import stream as DS
    rng = np.random.default_rng(world * 100 + chunk)
    d = tmp_path / "data"
    d.mkdir()
    rows = []
    for k in range(3):
        lines = [f"{k}-{i}|" + "x" * int(rng.integers(0, 30)) for i in range(int(rng.integers(1, 40)))]
        rows += lines
        _write(str(d / f"part-{k}"), lines, trailing_nl=(k != 1))
    gz = [f"g-{i}|z" for i in range(5)]
    with gzip.open(str(d / "part-9.gz"), "wt") as f:
        f.write("\n".join(gz) + "\n")
    files = DS.list_data_files(str(d))
    got = []
    for r in range(world):
        for fi, path, a, b in DS.byte_ranges(files, r, world):
            if a is None:
                got += [(fi, 0, l) for l in gzip.open(path, "rt").read().splitlines()]
                continue
            for off, blk in DS._lines_in_range(path, a, b, chunk):
                got += [(fi, off, l) for l in bytes(blk).decode().splitlines()]
    got.sort(key=lambda t: (t[0], t[1]))
    assert [g[2] for g in got] == rows + gz


def _model_set(tmp_path, method):
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.steps.create import run_init
    from shifu_amd.utils.synthetic import make_model_set
    a = make_model_set(str(tmp_path), "a", "NN", n_rows=2503, n_num=7, n_cat=3)
    mc = ModelConfig.load(os.path.join(a, "ModelConfig.json"))
    mc.stats["binningMethod"] = method
    mc.stats["maxNumBin"] = 9
    mc.save()
    run_init(a)
    return a


@pytest.mark.parametrize("method,cache_gb", [("EqualPositive", None), ("EqualTotal", None),
                                             ("WeightEqualPositive", None), ("EqualInterval", None),
                                             ("EqualPositive", "0.00004"), ("EqualTotal", "0.00004")])
def test_streamed_stats_equal_in_memory(tmp_path, monkeypatch, method, cache_gb):
    """cache_gb: an HBM-cache budget that holds only the first chunks -- later passes take the
    cached prefix and re-parse from the first uncached block (data/stream.py resume)."""
    import shutil
    from shifu_amd.config import environment
    from shifu_amd.steps.stats import run_stats
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    a = _model_set(tmp_path, method)
    b = str(tmp_path / "b")
    shutil.copytree(a, b)
    monkeypatch.setitem(environment.props(), "shifu.stats.streaming", "false")
    run_stats(a)
    monkeypatch.setitem(environment.props(), "shifu.stats.streaming", "true")
    monkeypatch.setitem(environment.props(), "shifu.stats.chunkMB", str(8 / 1024))      # 8 KB chunks
    if cache_gb is not None:
        monkeypatch.setenv("SHIFU_STATS_CACHE_GB", cache_gb)
        from shifu_amd.data import stream as DS
        resumed = []
        orig = DS.iter_model_data

        def spy(*a, **k):
            if k.get("resume") is not None:
                resumed.append(k["resume"])
            return orig(*a, **k)
        monkeypatch.setattr(DS, "iter_model_data", spy)
    run_stats(b)
    if cache_gb is not None:
        assert resumed and all(r[1] > 0 or r[0] > 0 for r in resumed), resumed   # a partial prefix was cached
    ca = json.load(open(os.path.join(a, "ColumnConfig.json")))
    cb = json.load(open(os.path.join(b, "ColumnConfig.json")))
    for x, y in zip(ca, cb):
        bx, by = x["columnBinning"], y["columnBinning"]
        for k in ("binBoundary", "binCategory", "binCountPos", "binCountNeg"):
            assert bx.get(k) == by.get(k), (x["columnName"], k)
        for k in ("binWeightedPos", "binWeightedNeg", "binCountWoe"):
            if bx.get(k) is not None:
                np.testing.assert_allclose(bx[k], by[k], rtol=1e-9, atol=1e-9)
        sx, sy = x["columnStats"], y["columnStats"]
        for k in ("totalCount", "missingCount", "distinctCount", "max", "min"):
            assert sx.get(k) == sy.get(k), (x["columnName"], k)
        for k in ("mean", "stdDev", "ks", "iv", "median", "skewness", "kurtosis"):
            if sx.get(k) is not None:
                np.testing.assert_allclose(sx[k], sy[k], rtol=1e-9, atol=1e-9, err_msg=f"{x['columnName']} {k}")


_RSS = r"""
import os, resource, sys, json
sys.path.insert(0, {root!r})
os.environ["SHIFU_FORCE_CPU"] = "1"
from shifu_amd.config import environment
from shifu_amd.steps.stats import run_stats
environment.props()["shifu.stats.streaming"] = {mode!r}
environment.props()["shifu.stats.chunkMB"] = "2"
def status(key):
    for line in open("/proc/self/status"):
        if line.startswith(key):
            return int(line.split()[1])
open("/proc/self/clear_refs", "w").write("5")      # reset the peak (VmHWM) to the current RSS
base = status("VmRSS:")
run_stats({root2!r})
print(json.dumps({{"base_kb": base, "peak_kb": status("VmHWM:")}}))
"""


def _rss_growth(root, mode):
    code = _RSS.format(root=ROOT, mode=mode, root2=root)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    return (res["peak_kb"] - res["base_kb"]) * 1024


def test_streamed_host_memory_bounded_by_chunk(tmp_path):
    """Peak RSS growth of the streamed pass (2 MB blocks) is flat in the data size: tripling the
    rows adds almost nothing, while the in-memory pass grows with the table."""
    from shifu_amd.steps.create import run_init
    from shifu_amd.utils.synthetic import make_model_set
    roots = {}
    for n in (50_000, 150_000):
        roots[n] = make_model_set(str(tmp_path / str(n)), "m", "NN", n_rows=n, n_num=30, n_cat=2)
        run_init(roots[n])
    s_small, s_big = _rss_growth(roots[50_000], "true"), _rss_growth(roots[150_000], "true")
    m_big = _rss_growth(roots[150_000], "false")
    print("rss growth MB: streamed 50K %.1f, streamed 150K %.1f, in-memory 150K %.1f"
          % (s_small / 1e6, s_big / 1e6, m_big / 1e6))
    assert s_big - s_small < 24e6, (s_small, s_big)
    # (the in-memory parse writes straight into its table -- one copy of the data -- so at this
    # small size the margin is the table minus the streamed pass's fixed buffers)
    assert s_big < 0.9 * m_big, (s_big, m_big)


@pytest.mark.gpu
@pytest.mark.parametrize("method", ["EqualPositive", "WeightEqualTotal"])
def test_streamed_stats_gpu_equal_cpu_in_memory(tmp_path, monkeypatch, method):
    """The streamed pass on the HIP kernels (qprep/qhist/qgather + column_stats) over 16 KB chunks
    writes the ColumnConfig of the CPU in-memory oracle."""
    import shutil
    from shifu_amd.config import environment
    from shifu_amd.steps.stats import run_stats
    a = _model_set(tmp_path, method)
    b = str(tmp_path / "b")
    shutil.copytree(a, b)
    monkeypatch.setitem(environment.props(), "shifu.stats.streaming", "false")
    run_stats(a, device="cpu")
    monkeypatch.setitem(environment.props(), "shifu.stats.streaming", "true")
    monkeypatch.setitem(environment.props(), "shifu.stats.chunkMB", str(16 / 1024))
    monkeypatch.setenv("SHIFU_STATS_CACHE_GB", "0")          # re-parse every pass
    run_stats(b, device="cuda")
    ca = json.load(open(os.path.join(a, "ColumnConfig.json")))
    cb = json.load(open(os.path.join(b, "ColumnConfig.json")))
    for x, y in zip(ca, cb):
        bx, by = x["columnBinning"], y["columnBinning"]
        for k in ("binBoundary", "binCategory", "binCountPos", "binCountNeg"):
            assert bx.get(k) == by.get(k), (x["columnName"], k)
        for k in ("binWeightedPos", "binWeightedNeg"):
            if bx.get(k) is not None:
                np.testing.assert_allclose(bx[k], by[k], rtol=1e-9, atol=1e-9)
        sx, sy = x["columnStats"], y["columnStats"]
        for k in ("totalCount", "missingCount", "distinctCount", "max", "min"):
            assert sx.get(k) == sy.get(k), (x["columnName"], k)
        for k in ("mean", "stdDev", "ks", "iv"):
            if sx.get(k) is not None:
                np.testing.assert_allclose(sx[k], sy[k], rtol=1e-7, atol=1e-9, err_msg=f"{x['columnName']} {k}")


def test_block_reader_helpers(tmp_path, monkeypatch):
    """data/stream.py: the newline search over uint8 ndarrays (page-locked blocks) equals the
    bytearray search, and the threaded pread fills a block exactly (short reads at end of file)."""
    from shifu_amd.data import stream as DS
    rng = np.random.default_rng(0)
    raw = bytearray(rng.choice(list(b"abc|\n"), size=300_000).astype(np.uint8).tobytes())
    arr = np.frombuffer(bytes(raw), np.uint8).copy()
    for lo, hi in ((0, len(raw)), (1000, 250_000), (5, 6), (299_990, 300_000)):
        for last in (True, False):
            assert DS._find_nl(arr, lo, hi, last) == DS._find_nl(raw, lo, hi, last), (lo, hi, last)
    assert DS._find_nl(np.zeros(10, np.uint8), 0, 10, True) == -1
    p = tmp_path / "blob"
    data = rng.integers(0, 256, size=(40 << 20) + 12345, dtype=np.uint8).tobytes()
    p.write_bytes(data)
    import os
    fd = os.open(str(p), os.O_RDONLY)
    try:
        monkeypatch.setattr(DS, "READ_THREADS", 5)
        buf = bytearray(len(data) + 100)
        got = DS._pread_into(fd, memoryview(buf), 7, len(data))          # runs past EOF by 7 bytes
        assert got == len(data) - 7 and bytes(buf[:got]) == data[7:]
    finally:
        os.close(fd)


def _corr_pair(tmp_path, monkeypatch, device):
    import shutil
    from shifu_amd.config import environment
    from shifu_amd.steps.create import run_init
    from shifu_amd.steps.stats import read_correlation, run_stats
    from shifu_amd.utils.synthetic import make_model_set
    a = make_model_set(str(tmp_path), "a", "NN", n_rows=4001, n_num=9, n_cat=2)
    run_init(a)
    run_stats(a, device=device)
    b = str(tmp_path / "b")
    shutil.copytree(a, b)
    monkeypatch.setitem(environment.props(), "shifu.stats.streaming", "false")
    run_stats(a, correlation=True, device=device)
    monkeypatch.setitem(environment.props(), "shifu.stats.streaming", "true")
    monkeypatch.setitem(environment.props(), "shifu.stats.chunkMB", str(16 / 1024))   # many blocks
    run_stats(b, correlation=True, device=device)
    na, ca = read_correlation(os.path.join(a, "correlation.csv"))
    nb, cb = read_correlation(os.path.join(b, "correlation.csv"))
    assert na == nb and len(na) >= 9
    return np.asarray(ca), np.asarray(cb)


def test_correlation_streamed_equals_in_memory(tmp_path, monkeypatch):
    """`stats -c` streamed chunk by chunk (no whole-table load) == the in-memory pass."""
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    ca, cb = _corr_pair(tmp_path, monkeypatch, "cpu")
    np.testing.assert_allclose(ca, cb, atol=1e-10)


@pytest.mark.gpu
def test_correlation_streamed_gpu_parse_exact(tmp_path, monkeypatch):
    """On the GPU: streamed `stats -c` with GPU-parsed blocks fed as device views == the in-memory
    pass (int8-digit MFMA sums; only the per-chunk digit scales and their fp64 flush order differ)."""
    ca, cb = _corr_pair(tmp_path, monkeypatch, "cuda")
    np.testing.assert_allclose(ca, cb, atol=1e-12)


def _posttrain_pair(tmp_path, monkeypatch, device):
    import json
    import shutil
    from shifu_amd.config import environment
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.steps.create import run_init
    from shifu_amd.steps.norm import run_norm
    from shifu_amd.steps.posttrain import run_posttrain
    from shifu_amd.steps.stats import run_stats
    from shifu_amd.steps.train import run_train
    from shifu_amd.utils.synthetic import make_model_set
    a = make_model_set(str(tmp_path), "a", "NN", n_rows=3001, n_num=7, n_cat=2)
    mc = ModelConfig.load(os.path.join(a, "ModelConfig.json"))
    mc.train["numTrainEpochs"], mc.train["baggingNum"] = 5, 1
    mc.save()
    run_init(a)
    run_stats(a, device=device)
    run_norm(a)
    run_train(a)
    b = str(tmp_path / "b")
    shutil.copytree(a, b)
    monkeypatch.setitem(environment.props(), "shifu.stats.streaming", "false")
    run_posttrain(a, device=device)
    monkeypatch.setitem(environment.props(), "shifu.stats.streaming", "true")
    monkeypatch.setitem(environment.props(), "shifu.stats.chunkMB", str(16 / 1024))
    run_posttrain(b, device=device)
    ca = {c["columnName"]: c["columnBinning"].get("binAvgScore") for c in json.load(open(os.path.join(a, "ColumnConfig.json")))}
    cb = {c["columnName"]: c["columnBinning"].get("binAvgScore") for c in json.load(open(os.path.join(b, "ColumnConfig.json")))}
    assert any(v for v in ca.values())
    return ca, cb


def test_posttrain_streamed_equals_in_memory(tmp_path, monkeypatch):
    """posttrain streamed chunk by chunk == the in-memory pass (binAvgScore of every column)."""
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    ca, cb = _posttrain_pair(tmp_path, monkeypatch, "cpu")
    assert ca == cb


@pytest.mark.gpu
def test_posttrain_streamed_gpu_equals_in_memory(tmp_path, monkeypatch):
    """On the GPU (GPU-parsed inputs binned in HBM): streamed posttrain == the in-memory pass."""
    ca, cb = _posttrain_pair(tmp_path, monkeypatch, "cuda")
    assert ca == cb


def test_pinned_blocks_stay_below_the_device_parse_limit(tmp_path, monkeypatch):
    """Blocks read for the GPU parse (pinned) are carry + read bytes: the read is capped so every
    block stays below the parser's int32 limit (a block at or above it would fall back to a host
    parse).  The limit is scaled down here; chunk_bytes equals it, as with 2-GB chunks."""
    from shifu_amd.data import gpu_parse, stream
    monkeypatch.setattr(gpu_parse, "BLOCK_LIMIT", 5000)
    monkeypatch.setattr(stream, "_new_buf", lambda n, pinned: bytearray(n))
    lines = [("%d|%s|%.3f\n" % (i, "x" * (i % 23), i * 0.37)).encode() for i in range(6000)]
    path = tmp_path / "t.csv"
    path.write_bytes(b"".join(lines))
    got = []
    for off, blk in stream._lines_in_range(str(path), 0, path.stat().st_size, 5000, nbuf=2, pinned=True):
        assert len(blk) < 5000
        got.append(bytes(blk))
    assert b"".join(got) == path.read_bytes()
    assert len(got) > 20
