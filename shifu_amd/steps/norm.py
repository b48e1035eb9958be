"""``norm`` / ``normalize`` / ``transform`` step (B5) with ``-shuffle`` (D6).

``NormalizeModelProcessor.run`` (J/core/processor/NormalizeModelProcessor.java:67-110): purify the
training data with ``normalize.sampleRate``/``sampleNegOnly``, normalize the selected (or, before
varsel, every good candidate) column with ``normalize.normType`` -> NormalizedData; tree
algorithms get CleanedData (bin codes) instead (``runDataClean``
J/core/processor/BasicModelProcessor.java:584-634).  A validation data path produces the matching
Normalized/CleanedValidationData.  ``-shuffle`` permutes rows (``MapReduceShuffle``
J/core/shuffle/MapReduceShuffle.java:59-186) — here a single in-memory permutation.

Output: columnar ``.npy`` caches (see :mod:`.base`).  Targets: binary 0/1, multi-class index,
regression value; weights from the weight column/expression.
"""
from __future__ import annotations

import numpy as np

from ..algos import normalize as N
from ..utils.device import is_gpu_available
from ..utils.log import get_logger
from .base import ModelSet, save_dataset

_log = get_logger("steps.norm")

TREE_ALGS = ("GBT", "RF", "DT")


def _write_shared(path: str, arrays: dict, meta: dict, lo: int, hi: int, n: int, positions=None):
    """Data-parallel cache write: rank 0 creates the full-size .npy files, every rank writes its
    rows in place (np.lib.format memmaps) -- at [lo, hi), or at ``positions`` (shuffled output),
    rank 0 writes meta.json last."""
    import json
    import os
    import shutil
    from ..parallel import dist
    if dist.info().rank == 0:
        if os.path.isdir(path):
            shutil.rmtree(path)
        os.makedirs(path, exist_ok=True)
        for k, v in arrays.items():
            np.lib.format.open_memmap(os.path.join(path, f"{k}.npy"), mode="w+", dtype=v.dtype,
                                      shape=(n,) + tuple(v.shape[1:])).flush()
    dist.barrier()
    for k, v in arrays.items():
        mm = np.load(os.path.join(path, f"{k}.npy"), mmap_mode="r+")
        if positions is None:
            mm[lo:hi] = v
        else:
            mm[positions] = v
        mm.flush()
        del mm
    dist.barrier()
    if dist.info().rank == 0:
        with open(os.path.join(path, "meta.json"), "w") as f:
            json.dump(meta, f, indent=1)
    dist.barrier()


def _norm_one(ms: ModelSet, cols, data_conf, out_x, out_tree, sample_rate, neg_only, shuffle, seed, is_tree):
    """Normalize one data set into the NormalizedData / CleanedData caches.  Under more than one
    rank every rank normalizes the output row range [n*r/R, n*(r+1)/R) (rows of the global
    shuffle permutation when shuffling) and writes it in place: the caches are identical to the
    single-process ones."""
    from ..parallel import dist
    mc = ms.mc
    info = dist.info()
    positions = None
    if info.world_size > 1:
        # this rank's byte range only (data/stream.py); its rows are the contiguous global row
        # range [lo, hi) of the single-process table (same per-row sampling draws)
        from ..data.stream import load_rank_dataset
        md = load_rank_dataset(mc, data_conf, [c.name for c in cols if not c.is_categorical()],
                               [c.name for c in cols if c.is_categorical()], sample_rate, neg_only, seed,
                               rank=info.rank, world=info.world_size)
        counts = dist.all_gather_objects(int(md.n))
        n = int(sum(counts))
        lo = int(sum(counts[: info.rank]))
        hi = lo + int(md.n)
        if shuffle:                  # row g lands at inv[g] (output[i] = row perm[i])
            perm = np.random.default_rng(seed).permutation(n)
            inv = np.empty(n, np.int64)
            inv[perm] = np.arange(n)
            positions = inv[lo:hi]
    else:
        md = ms.load_raw(cols, data_conf, sample_rate, neg_only, seed)
        n = int(md.n)
        lo, hi = 0, n
        if shuffle:
            idx = np.random.default_rng(seed).permutation(n)
            from dataclasses import replace
            md = replace(md, table=md.table.take(idx), y=md.y[idx], w=md.w[idx], tag_index=md.tag_index[idx])
    y, w = md.y.astype(np.float32), md.w.astype(np.float32)
    meta = {"n": n, "columns": [c.name for c in cols], "column_nums": [c.num for c in cols],
            "counters": md.counters.as_dict(), "is_binary": mc.is_binary(), "tags": mc.flatten_tags(),
            "shuffled": bool(shuffle)}
    gpu = is_gpu_available()
    save = (lambda p_, a_, m_: _write_shared(p_, a_, m_, lo, hi, n, positions)) if info.world_size > 1 \
        else save_dataset
    if is_tree:
        r = N.tree_bin_codes_gpu(ms.ccs, md.table, cols) if gpu else None
        C, nb, is_cat = r if r is not None else N.tree_bin_codes(ms.ccs, md.table, cols)
        dt = np.uint8 if (nb.max(initial=1) <= 256) else np.int16
        C = C.astype(dt)
        meta.update(nbins=nb.tolist(), is_cat=is_cat.tolist())
        save(out_tree, {"codes": C, "y": y, "w": w}, meta)
        _log.info("CleanedData: %s rows x %s cols -> %s", n, C.shape[1], out_tree)
    X, names, nums = (N.normalize_table_gpu if gpu else N.normalize_table)(mc, ms.ccs, md.table, columns=cols)
    meta.update(norm_type=mc.norm_type, input_names=names, input_nums=nums)
    save(out_x, {"X": X, "y": y, "w": w}, meta)
    _log.info("NormalizedData: %s rows x %s inputs (%s) -> %s", n, X.shape[1], mc.norm_type, out_x)
    return n


def run_norm(root: str = ".", shuffle: bool = False, seed: int = 0) -> int:
    ms = ModelSet(root).setup("NORMALIZE")
    mc = ms.mc
    cols = ms.norm_columns()
    if not cols:
        raise ValueError("no candidate/selected columns to normalize; run stats (and varsel) first")
    is_tree = mc.algorithm in TREE_ALGS
    sr = float(mc.normalize.get("sampleRate", 1.0))
    neg = bool(mc.normalize.get("sampleNegOnly", False))
    _norm_one(ms, cols, mc.dataSet, ms.pf.normalized_data, ms.pf.cleaned_data, sr, neg, shuffle, seed, is_tree)
    vpath = mc.dataSet.get("validationDataPath")
    if vpath:
        vconf = mc.dataSet.copy_with(dataPath=vpath,
                                     filterExpressions=mc.dataSet.get("validationFilterExpressions") or
                                     mc.dataSet.get("filterExpressions"))
        _norm_one(ms, cols, vconf, ms.pf.normalized_validation_data, ms.pf.cleaned_validation_data, 1.0, False,
                  False, seed, is_tree)
    return 0
