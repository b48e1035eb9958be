"""GPU text parsing (K0: ops/csrc/csv_kernels.hip + data/gpu_parse.py).

CPU: device-resident columns (DeviceBlock / DevRef on a CPU tensor) behave like host columns
(lazy ``values``, ``take`` gathers each block once, ``device_rows`` views / gathers).  GPU: the
kernel + host framing give the host parser's values bit for bit on adversarial text (signs,
leading zeros, exponents, Java "1.0d", padded fields, numeric missing tokens, CRLF, blank lines,
short / long rows, 20+ digit fields), and a streamed stats + norm run with GPU parsing on equals
the run with it off.
"""
import os
import random

import numpy as np
import pytest
import torch

from shifu_amd.data import reader as R
from shifu_amd.data.gpu_parse import DeviceBlock, DevRef, device_rows


def test_device_columns_cpu_semantics():
    D = torch.arange(12, dtype=torch.float64).view(3, 4)
    blk = DeviceBlock(D)
    cols = {f"c{j}": R.Column(f"c{j}", "num", dev=DevRef(blk, j)) for j in range(3)}
    t = R.RawTable(["c0", "c1", "c2"], cols, 4)
    assert len(t["c1"]) == 4 and t["c1"]._values is None
    v = device_rows([t["c0"], t["c1"]], "cpu")
    assert torch.equal(v, D[0:2]) and v.data_ptr() == D.data_ptr()          # a view, no copy
    assert torch.equal(device_rows([t["c2"], t["c0"]], "cpu"), D[[2, 0]])
    sub = t.take(np.array([3, 1]))
    assert sub["c0"].dev.block is sub["c2"].dev.block                         # one gather per block
    np.testing.assert_array_equal(sub["c1"].values, [7.0, 5.0])
    np.testing.assert_array_equal(t["c2"].values, [8.0, 9.0, 10.0, 11.0])   # lazy host copy
    assert R.numeric_rows([t["c0"].values, t["c1"].values]) is not None      # rows of one host block
    assert device_rows([t["c0"], None], "cpu") is None


def _adversarial_text(rng, ncols, nrows, crlf=False, ragged=True):
    toks = ["", "?", "-999", "0", "1.5", "-0.000", "+12.25", "007.50", "12.", "-.5", ".", "-", "1e5", "1.0d",
            "123456789012345", "1234567890123456", "12345678901234567890", "0.1234567890123456789", "3.14159",
            " 4.5", "4.5 ", "\t-2.25", "99999999999999.9", "-0.00001", "1.", "00000000000000001", "NaN", "abc",
            "9007199254740993", "1.7976931348623157e308", "1" * 30, "0." + "0" * 25 + "1"]
    lines = []
    for _ in range(nrows):
        k = ncols + (rng.choice([0] * 12 + [-1, -5, 2]) if ragged else 0)
        f = [rng.choice(toks) if rng.random() < 0.4 else f"{rng.gauss(0, 1000):.{rng.randint(0, 9)}f}"
             for _ in range(max(1, k))]
        lines.append("|".join(f))
        if rng.random() < 0.01:
            lines.append(rng.choice(["", "   ", "\t \r"]))
    eol = "\r\n" if crlf else "\n"
    return (eol.join(lines) + eol).encode()


@pytest.mark.gpu
@pytest.mark.parametrize("crlf,miss", [(False, ["", "?"]), (True, ["", "?", "-999", "0", "NA"])])
def test_gpu_parse_bit_identical(crlf, miss):
    from shifu_amd.data.gpu_parse import GpuBlockParser
    rng = random.Random(11 + crlf)
    C = 37
    data = _adversarial_text(rng, C, 6000, crlf)
    kinds = [rng.choice([1, 1, 1, 0, 2]) for _ in range(C)]
    gcols = [c for c in range(C) if kinds[c] == 1 and rng.random() < 0.8]
    pinned = torch.empty(len(data), dtype=torch.uint8, pin_memory=True).numpy()
    pinned[:] = np.frombuffer(data, np.uint8)
    gp = GpuBlockParser(kinds, gcols, "|", miss, torch.device("cuda", 0))
    assert gp.usable
    n, bad, out = gp.parse(memoryview(pinned), 4)
    n2, bad2, ref = R._parse_native(bytearray(data), "|", kinds, miss, 4)
    assert (n, bad) == (n2, bad2) and n > 5000
    assert gp.stats["fallback_fields"] > 0
    for c in range(C):
        if kinds[c] == 1:
            got = out[c][1].host() if c in gcols else out[c][1]
            assert got.tobytes() == ref[c][1].tobytes(), f"column {c}"
        elif kinds[c] == 2:
            assert list(out[c][1]) == list(ref[c][1]) and out[c][2] == ref[c][2]


@pytest.mark.gpu
@pytest.mark.parametrize("crlf", [False, True])
def test_gpu_parse_host_columns_from_field_bounds(crlf):
    """No ragged rows: the host columns (strings with empty / missing / padded values, a numeric
    one) are parsed from the field bounds the kernel returns (shifu_gather_fields), blank lines
    dropped -- same values, codes, dictionaries and row count as the full host parse."""
    from shifu_amd.data.gpu_parse import GpuBlockParser
    rng = random.Random(5 + crlf)
    C = 29
    data = _adversarial_text(rng, C, 5000, crlf, ragged=False)
    kinds = [1] * C
    for c in (0, 7, C - 1):
        kinds[c] = 2
    gcols = [c for c in range(C) if kinds[c] == 1 and c != 3]        # column 3: numeric on the host
    pinned = torch.empty(len(data), dtype=torch.uint8, pin_memory=True).numpy()
    pinned[:] = np.frombuffer(data, np.uint8)
    miss = ["", "?", "NA"]
    gp = GpuBlockParser(kinds, gcols, "|", miss, torch.device("cuda", 0))
    n, bad, out = gp.parse(memoryview(pinned), 4)
    n2, bad2, ref = R._parse_native(bytearray(data), "|", kinds, miss, 4)
    assert (n, bad) == (n2, bad2) == (n, 0) and n == 5000
    assert gp.stats.get("gathered_blocks") == 1
    for c in range(C):
        if kinds[c] == 1:
            got = out[c][1].host() if c in gcols else out[c][1]
            assert got.tobytes() == ref[c][1].tobytes(), f"column {c}"
        else:
            assert list(out[c][1]) == list(ref[c][1]) and out[c][2] == ref[c][2], f"column {c}"


@pytest.mark.gpu
def test_gpu_parse_blank_lines_after_poisoned_allocator():
    """Blank lines leave the host-column bounds of those lines unwritten by the kernel: the gather
    buffer must be sized without them.  Fill and free a large block with huge int32 values first,
    so the caching allocator hands that memory back to the parser's bounds tensor."""
    from shifu_amd.data.gpu_parse import GpuBlockParser
    rng = random.Random(9)
    C = 11
    lines = []
    for i in range(20000):
        lines.append("|".join(f"{rng.gauss(0, 10):.3f}" if c != 4 else f"s{i % 13}" for c in range(C)))
        if i % 7 == 0:
            lines.append("")
    data = ("\n".join(lines) + "\n").encode()
    poison = torch.full((64 << 20,), 0x7ffffff0, dtype=torch.int32, device="cuda")
    del poison                                              # back to the caching allocator, not zeroed
    kinds = [1] * C
    kinds[4] = 2
    pinned = torch.empty(len(data), dtype=torch.uint8, pin_memory=True).numpy()
    pinned[:] = np.frombuffer(data, np.uint8)
    gp = GpuBlockParser(kinds, [c for c in range(C) if c not in (4, 8)], "|", [""], torch.device("cuda", 0))
    n, bad, out = gp.parse(memoryview(pinned), 4)
    n2, bad2, ref = R._parse_native(bytearray(data), "|", kinds, [""], 4)
    assert (n, bad) == (n2, bad2) == (20000, 0)
    assert list(out[4][1]) == list(ref[4][1]) and out[8][1].tobytes() == ref[8][1].tobytes()


@pytest.mark.gpu
def test_gpu_parse_no_trailing_newline_and_wide_rows():
    from shifu_amd.data.gpu_parse import GpuBlockParser
    rng = np.random.default_rng(3)
    C = 1500
    rows = ["|".join(f"{v:.6f}" for v in rng.normal(size=C)) for _ in range(300)]
    data = "\n".join(rows).encode()                        # last line without '\n'
    pinned = torch.empty(len(data), dtype=torch.uint8, pin_memory=True).numpy()
    pinned[:] = np.frombuffer(data, np.uint8)
    kinds = [1] * C
    gp = GpuBlockParser(kinds, list(range(1, C)), "|", [""], torch.device("cuda", 0))
    n, bad, out = gp.parse(memoryview(pinned), 4)
    _, _, ref = R._parse_native(bytearray(data), "|", kinds, [""], 4)
    assert n == 300 and bad == 0
    for c in (1, 2, 700, C - 1):
        assert out[c][1].host().tobytes() == ref[c][1].tobytes()
    assert gp.stats["fallback_fields"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("alg", ["NN", "GBT"])
def test_streamed_stats_and_norm_same_with_gpu_parse(tmp_path, alg):
    """CLI stats + streamed norm on a generated model set (many small blocks): GPU parsing on ==
    off -- ColumnConfig stats and the NormalizedData / CleanedData caches byte for byte."""
    import json
    import shutil
    from shifu_amd.config import environment
    from shifu_amd.steps.base import load_dataset_cache
    from shifu_amd.steps.create import run_init
    from shifu_amd.steps.norm import run_norm
    from shifu_amd.steps.stats import run_stats
    from shifu_amd.utils.synthetic import make_model_set
    a = make_model_set(str(tmp_path), "a", alg, n_rows=20000, n_num=30, n_cat=2)
    run_init(a)
    b = str(tmp_path / "b")
    shutil.copytree(a, b)
    P = environment.props()
    old = {k: P.get(k) for k in ("shifu.data.gpuParse", "shifu.stats.streaming", "shifu.norm.streaming",
                                 "shifu.stats.chunkMB", "shifu.norm.chunkMB")}
    try:
        P.update({"shifu.stats.streaming": "true", "shifu.norm.streaming": "true", "shifu.stats.chunkMB": "0.5",
                  "shifu.norm.chunkMB": "0.5"})
        for root, mode in ((a, "false"), (b, "true")):
            P["shifu.data.gpuParse"] = mode
            run_stats(root)
            run_norm(root)
    finally:
        for k, v in old.items():
            if v is None:
                P.pop(k, None)
            else:
                P[k] = v
    ca = json.load(open(os.path.join(a, "ColumnConfig.json")))
    cb = json.load(open(os.path.join(b, "ColumnConfig.json")))
    assert ca == cb
    for sub in (["CleanedData", "NormalizedData"] if alg == "GBT" else ["NormalizedData"]):
        ma, xa = load_dataset_cache(os.path.join(a, "tmp", sub), mmap=False)
        mb, xb = load_dataset_cache(os.path.join(b, "tmp", sub), mmap=False)
        assert ma["n"] == mb["n"] > 0
        for k in xa:
            assert np.asarray(xa[k]).tobytes() == np.asarray(xb[k]).tobytes(), (sub, k)


def test_gather_fields_cpu():
    """shifu_gather_fields (the host half of the GPU parse: the host columns rebuilt from field
    bounds) on bounds computed here: blank lines skipped, empty / padded fields kept, every line
    ends with the unparsed "x" field so a line of empty fields never reads as blank."""
    from shifu_amd.ops import _native as nat
    lib = nat.rt()
    if lib is None:
        pytest.skip("native runtime not built")
    lines = ["a|1.5|x1", "|2|", "   ", " b |  |q", "c|-3|z"]
    text = ("\n".join(lines) + "\n").encode()
    buf = np.frombuffer(bytearray(text), np.uint8)
    want_cols = [0, 2]                       # host columns
    offs = np.zeros((len(want_cols), len(lines), 2), np.int32)
    flags = np.zeros(len(lines), np.int32)
    pos = 0
    for li, ln in enumerate(lines):
        if not ln.strip():
            flags[li] = 1
        starts, p = [], pos
        for f in ln.split("|"):
            starts.append((p, p + len(f)))
            p += len(f) + 1
        for j, c in enumerate(want_cols):
            offs[j, li] = starts[c] if c < len(starts) else (pos, pos)
        pos += len(ln) + 1
    cap = 256
    out = np.zeros(cap, np.uint8)
    nb = lib.shifu_gather_fields(buf.ctypes.data, offs.ctypes.data, len(lines), len(want_cols), flags.ctypes.data,
                                 b"|", out.ctypes.data, cap)
    got = bytes(out[:nb]).decode()
    assert got == "a|x1|x\n||x\n b |q|x\nc|z|x\n"
    assert lib.shifu_gather_fields(buf.ctypes.data, offs.ctypes.data, len(lines), len(want_cols), flags.ctypes.data,
                                   b"|", out.ctypes.data, 8) == -1        # cap too small


@pytest.mark.gpu
def test_streamed_tables_gpu_parse_equal_host_multi_file(tmp_path):
    """data/stream.iter_tables over several part files (a header line in the first, a gzip part
    parsed on the host, small blocks with carried lines, CRLF rows, a weight column kept on the
    host): GPU-parsed tables equal host-parsed ones column for column, bit for bit."""
    import gzip
    from shifu_amd.data import stream as DS
    from shifu_amd.data.purifier import DatasetPlan
    rng = random.Random(3)
    C = 12
    header = ["tag", "w"] + [f"x{j}" for j in range(C)] + ["cat"]
    def line():
        vals = [rng.choice(["M", "B"]), f"{rng.random():.3f}"]
        vals += [rng.choice(["", "?", "1e3", " 2.5 "]) if rng.random() < 0.1 else f"{rng.gauss(0, 10):.{rng.randint(0, 7)}f}"
                 for _ in range(C)]
        vals.append(rng.choice(["a", "b", "", "c c"]))
        return "|".join(vals) + rng.choice(["\n", "\n", "\r\n"])
    d = tmp_path / "data"
    d.mkdir()
    (d / "part-00000").write_text("|".join(header) + "\n" + "".join(line() for _ in range(3000)))
    (d / "part-00001").write_text("".join(line() for _ in range(2500)))
    with gzip.open(d / "part-00002.gz", "wt") as f:
        f.write("".join(line() for _ in range(700)))
    nums = ["w"] + [f"x{j}" for j in range(C)]
    plan = DatasetPlan(str(d), "|", header, True, "tag", "w", None, nums, ["tag", "cat"], [], [], ["", "?"])
    gp = DS.gpu_parser(plan, [f"x{j}" for j in range(C)] + ["w"], torch.device("cuda", 0))
    assert gp is not None and "w" not in [header[c] for c in gp.gpu_cols]
    host = list(DS.iter_tables(plan, 64 << 10))
    dev = list(DS.iter_tables(plan, 64 << 10, gpu=gp))
    assert len(host) == len(dev) >= 8
    for (ka, ta), (kb, tb) in zip(host, dev):
        assert ka == kb and ta.n == tb.n and ta.bad_rows == tb.bad_rows
        for name in header:
            a, b = ta[name], tb[name]
            assert np.asarray(a.values).tobytes() == np.asarray(b.values).tobytes(), (ka, name)
            assert a.dictionary == b.dictionary, (ka, name)
    assert sum(t.n for _, t in dev) == 6200


@pytest.mark.gpu
def test_newline_index_kernel_matches_nonzero():
    """The own newline index (csv_kernels.hip: segment counts, scan, ordered writes) equals
    torch.nonzero over blocks with short / long lines, CR bytes and a tail without a newline."""
    import torch
    from shifu_amd.data.gpu_parse import GpuBlockParser
    rng = np.random.default_rng(3)
    p = GpuBlockParser([1, 1], [0, 1], "|", [""], "cuda")
    for L in (1, 300, 65536, 65536 * 3 + 17, 5_000_001):
        b = rng.integers(32, 127, size=L).astype(np.uint8)
        nl = rng.random(L) < rng.choice([0.0005, 0.02, 0.3])
        b[nl] = 10
        d = torch.zeros(L + 64, dtype=torch.uint8, device="cuda")
        d[:L] = torch.as_tensor(b, device="cuda")
        got = p._newlines(d, L)
        want = torch.nonzero(d[:L] == 10).flatten()
        assert torch.equal(got, want), L
