"""Segmented part files (data/rowstore.SegmentAppender): blocks split into several files written
at once read back, through load_parts / RowParts, as the rows appended, in order; a rewrite
replaces old segments; an empty array still has a segment; the streamed norm writes them."""
import json
import os

import numpy as np

from shifu_amd.data import rowstore as R


def test_segments_roundtrip_in_order(tmp_path, monkeypatch):
    monkeypatch.setattr(R.SegmentAppender, "MIN_SPLIT_BYTES", 0)
    monkeypatch.setattr(R.SegmentAppender, "SPLIT", 3)
    d = tmp_path / "part-00000"
    d.mkdir()
    rng = np.random.default_rng(0)
    blocks = [rng.integers(0, 60000, size=(n, 7)).astype(np.uint16) for n in (10, 1, 0, 25, 2)]
    ap = R.SegmentAppender(str(d), "Xb", np.uint16, (7,))
    yap = R.SegmentAppender(str(d), "y", np.float32)
    for b in blocks:
        ap.append(b)
        yap.append(b[:, 0].astype(np.float32))
    assert ap.close() == 38 and yap.close() == 38
    ref = np.concatenate(blocks)
    assert R.part_names(str(d)) == ["Xb", "y"]
    segs = R.part_arrays(str(d), "Xb")
    assert len(segs) == 3 + 1 + 3 + 2                      # 10 -> 3, 1 -> 1, 25 -> 3, 2 -> 2 files
    meta = {"parts": [{"dir": "part-00000", "n": 38}]}
    arrs = R.load_parts(str(tmp_path), meta)
    x = arrs["Xb"]
    assert isinstance(x, R.RowParts) and x.shape == (38, 7)
    np.testing.assert_array_equal(np.asarray(x), ref)
    np.testing.assert_array_equal(x[5:30], ref[5:30])
    np.testing.assert_array_equal(x[[0, 12, 37, 11]], ref[[0, 12, 37, 11]])
    assert sum(len(v) for v in x.blocks(9, 13)) == 4
    np.testing.assert_array_equal(np.asarray(arrs["y"]), ref[:, 0].astype(np.float32))
    # a rewrite replaces every old segment
    ap2 = R.SegmentAppender(str(d), "Xb", np.uint16, (7,))
    ap2.append(ref[:4])
    ap2.close()
    np.testing.assert_array_equal(np.concatenate(R.part_arrays(str(d), "Xb")), ref[:4])
    # an empty array keeps one (empty) segment so readers see the name
    e = R.SegmentAppender(str(d), "w", np.float32)
    assert e.close() == 0
    assert [len(a) for a in R.part_arrays(str(d), "w")] == [0]


def test_streamed_norm_writes_segments_equal_to_in_memory(tmp_path, monkeypatch):
    """The streamed norm with several chunks and split segments gives the in-memory norm's rows."""
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    monkeypatch.setattr(R.SegmentAppender, "MIN_SPLIT_BYTES", 0)
    monkeypatch.setattr(R.SegmentAppender, "SPLIT", 4)
    from shifu_amd.cli import main
    from shifu_amd.steps.base import load_dataset_cache
    from shifu_amd.utils.synthetic import make_model_set
    roots = []
    for name, stream in (("a", "true"), ("b", "false")):
        r = make_model_set(str(tmp_path), name, "NN", n_rows=1200, n_num=5, n_cat=2)
        cwd = os.getcwd()
        os.chdir(r)
        try:
            assert main(["init"]) == 0 and main(["stats"]) == 0
            assert main(["norm", f"-Dshifu.norm.streaming={stream}", "-Dshifu.norm.chunkMB=0.05"]) == 0
        finally:
            os.chdir(cwd)
        roots.append(r)
    (ma, da), (mb, db) = (load_dataset_cache(os.path.join(r, "tmp", "NormalizedData"), mmap=False) for r in roots)
    pa = os.path.join(roots[0], "tmp", "NormalizedData", "part-00000")
    assert any("@" in fn for fn in os.listdir(pa))
    assert ma["n"] == mb["n"]
    for k in ("y", "w"):
        np.testing.assert_array_equal(np.asarray(da[k]).reshape(-1), np.asarray(db[k]).reshape(-1))
    np.testing.assert_allclose(np.asarray(da["X"]), np.asarray(db["X"]), rtol=0, atol=0)
