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

import time

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


def _streaming(ms) -> bool:
    """``shifu.norm.streaming``: ``true`` / ``false`` / ``auto`` (default: stream when this rank's
    share of the data exceeds ``shifu.norm.inMemoryMB``, 1024)."""
    from ..config import environment
    from ..data.purifier import plan_dataset
    from ..data.stream import data_bytes
    from ..parallel import dist
    mode = str(environment.get("shifu.norm.streaming", "auto")).lower()
    if mode in ("true", "1", "on"):
        return True
    if mode in ("false", "0", "off"):
        return False
    try:
        nbytes = data_bytes(plan_dataset(ms.mc, ms.mc.dataSet))
    except (OSError, ValueError):
        return False
    return nbytes / max(1, dist.info().world_size) > float(environment.get("shifu.norm.inMemoryMB", 1024)) * (1 << 20)


def _norm_one_streamed(ms: ModelSet, cols, data_conf, out_x, out_tree, sample_rate, neg_only, shuffle, seed,
                       is_tree):
    """Out-of-core norm (the reference streams rows through ``P/Normalize.pig:35-46`` ->
    ``NormalizeUDF.exec``): this rank's byte range is parsed chunk by chunk; each chunk goes through
    ONE fused K5 launch (``NormPlan``: raw values read once -> fp32 or bf16 GEMM-ready rows + uint8
    tree codes) and is appended to this rank's ``part-RRRRR`` of the caches (``data/rowstore.py``).
    Host memory holds one chunk.  ``-shuffle`` then permutes the written parts out of core with the
    single-process permutation (``_shuffle_parts``), so every output equals the in-memory norm."""
    import os
    import shutil
    from ..config import environment
    from ..data import stream as DS
    from ..data.purifier import plan_dataset
    from ..data.rowstore import SegmentAppender, write_parts_meta
    from ..parallel import dist
    mc = ms.mc
    info = dist.info()
    plan = plan_dataset(mc, data_conf, [c.name for c in cols if not c.is_categorical()],
                        [c.name for c in cols if c.is_categorical()])
    x_dtype = str(environment.get("shifu.norm.dtype", "float32")).lower()
    x_dtype = "bf16" if x_dtype in ("bf16", "bfloat16") else "float32"
    row0 = DS.rank_row_offset(plan, info.rank, info.world_size) if sample_rate < 1.0 else 0
    dev = None
    if is_gpu_available():
        import torch
        dev = torch.device("cuda", torch.cuda.current_device())
        # blocks a previous step of this process left cached (the stats pass's device cache of
        # parsed chunks: ~200 GB at 20M x 1600) go back to the driver now, so it has cleared them
        # by the time a later step makes its big allocation (released at the end of this pass
        # instead, the varsel 64-GB cache allocation took 0.6-4.4 s)
        t_e = time.perf_counter()
        torch.cuda.empty_cache()
        _log.info("norm: cached HBM of earlier steps released in %.2fs", time.perf_counter() - t_e)
    # two rotating pinned output buffers: chunk i is written while chunk i + 1 is normalized
    nplan = N.NormPlan(mc, ms.ccs, cols, want_x=True, want_codes=is_tree, x_dtype=x_dtype, device=dev,
                       pinned_out=2 if dev is not None else 0)
    nplan.async_out = dev is not None        # the writer waits for the chunk's D2H, not the consumer
    # 2-GB text chunks on the GPU-parse path: 20M x 1600 norm pass 9.3 -> 8.3 s (profiles/r5/pipeline)
    chunk = int(float(environment.get("shifu.norm.chunkMB", 2048 if dev is not None else 256)) * (1 << 20))
    outs = [out_x] + ([out_tree] if is_tree else [])
    if info.rank == 0:
        for o in outs:
            if os.path.isdir(o):
                shutil.rmtree(o)
            os.makedirs(o, exist_ok=True)
    dist.barrier()
    pdir = f"part-{info.rank:05d}"
    for o in outs:
        os.makedirs(os.path.join(o, pdir), exist_ok=True)
    xname = "Xb" if x_dtype == "bf16" else "X"
    # segmented part files: a chunk's rows go out as several files written at once (one tmpfs
    # inode takes one writer at a time; data/rowstore.SegmentAppender)
    xd, td = os.path.join(out_x, pdir), os.path.join(out_tree, pdir)
    apx = {xname: SegmentAppender(xd, xname, np.uint16 if x_dtype == "bf16" else np.float32,
                                  (nplan.kpad if x_dtype == "bf16" else nplan.width,)),
           "y": SegmentAppender(xd, "y", np.float32),
           "w": SegmentAppender(xd, "w", np.float32)}
    apt = {}
    if is_tree:
        apt = {"codes": SegmentAppender(td, "codes", nplan.code_dtype, (len(cols),)),
               "y": SegmentAppender(td, "y", np.float32),
               "w": SegmentAppender(td, "w", np.float32)}
    counters = {}
    n_local = 0

    def write(res, y, w, ev):
        if ev is not None:
            ev.synchronize()                  # this chunk's D2H into the pinned buffers landed
        apx[xname].append(res[xname])
        apx["y"].append(y)
        apx["w"].append(w)
        if is_tree:
            apt["codes"].append(res["codes"])
            apt["y"].append(y)
            apt["w"].append(w)

    # the cache writes of chunk i (file writes release the GIL) run on a writer thread while
    # chunk i+1 is normalized; one write in flight keeps the part files in row order
    from concurrent.futures import ThreadPoolExecutor
    pending = None
    t_pass = time.perf_counter()
    try:
        with ThreadPoolExecutor(1, thread_name_prefix="shifu-norm-write") as ex:
            gpu_cols = [c.name for c in cols if not c.is_categorical()] if dev is not None else None
            for md in DS.iter_model_data(mc, plan, chunk, info.rank, info.world_size, sample_rate, neg_only, seed,
                                         row0=row0, gpu_cols=gpu_cols, dev=dev):
                with DS._span("consume"):
                    res = nplan.run(md.table)
                    y, w = md.y.astype(np.float32), md.w.astype(np.float32)
                with DS._span("write_wait"):
                    if pending is not None:
                        pending.result()
                pending = ex.submit(write, res, y, w, nplan.last_event)
                n_local += md.n
                for k, v in md.counters.as_dict().items():
                    counters[k] = counters.get(k, 0) + v
            if pending is not None:
                pending.result()
    finally:
        for a in list(apx.values()) + list(apt.values()):
            a.close()
    t_rel = time.perf_counter()
    mem = ""
    if dev is not None:
        import torch
        mem = " (HBM reserved %.1f GB, peak allocated %.1f GB)" % (torch.cuda.memory_reserved(dev) / 1e9,
                                                                  torch.cuda.max_memory_allocated(dev) / 1e9)
        getattr(nplan, "_bufs", {}).clear()
        getattr(nplan, "_pins", {}).clear()
    if dev is not None:
        import torch
        mem += " -> %.1f GB allocated after" % (torch.cuda.memory_allocated(dev) / 1e9)
    _log.info("norm pass %.2fs (writes closed)%s", t_rel - t_pass, mem)
    got = dist.all_gather_objects((n_local, counters))
    rows = [g[0] for g in got]
    tot_counters = {}
    for _, c in got:
        for k, v in c.items():
            tot_counters[k] = tot_counters.get(k, 0) + v
    meta = {"columns": [c.name for c in cols], "column_nums": [c.num for c in cols], "counters": tot_counters,
            "is_binary": mc.is_binary(), "tags": mc.flatten_tags(), "shuffled": bool(shuffle), "streamed": True}
    metas = {out_x: dict(meta, norm_type=nplan.nt, input_names=nplan.names, input_nums=nplan.nums,
                         x_dtype=x_dtype, **({"x_kpad": nplan.kpad, "x_width": nplan.width} if x_dtype == "bf16"
                                             else {}))}
    if is_tree:
        tm = {"nbins": nplan.nbins.tolist(), "is_cat": nplan.is_cat.tolist()}
        metas[out_tree] = dict(meta, **tm)
        metas[out_x].update(tm)
    dist.barrier()
    for o in outs:
        if shuffle:
            _shuffle_parts(o, rows, seed)
        if info.rank == 0:
            write_parts_meta(o, metas[o], rows)
    dist.barrier()
    n = int(sum(rows))
    _log.info("NormalizedData (streamed%s, %s, rank %d/%d): %d rows (%d here) x %d inputs (%s) -> %s",
              ", shuffled" if shuffle else "", x_dtype, info.rank, info.world_size, n, n_local, nplan.width,
              nplan.nt, out_x)
    return n


def _shuffle_parts(path: str, rows: list, seed: int) -> None:
    """Out-of-core ``-shuffle`` of a partitioned cache: output row i = input row perm[i] with the
    single-process permutation (``default_rng(seed).permutation(n)``); rank r writes output rows
    [n r / R, n (r + 1) / R) as its new part, reading its rows by (sorted) memmap gathers in
    blocks, then the new parts replace the old ones."""
    import os
    import shutil
    from ..data.rowstore import NpyAppender, RowParts, part_arrays, part_names
    from ..parallel import dist
    info = dist.info()
    n = int(sum(rows))
    perm = np.random.default_rng(seed).permutation(n)
    parts = [f"part-{r:05d}" for r in range(len(rows))]
    names = part_names(os.path.join(path, parts[info.rank]))
    lo, hi = n * info.rank // info.world_size, n * (info.rank + 1) // info.world_size
    mine = perm[lo:hi]
    newdir = os.path.join(path, f"shuf-{info.rank:05d}")
    os.makedirs(newdir, exist_ok=True)
    block = 1 << 20
    for name in names:
        arrs = [x for p in parts for x in part_arrays(os.path.join(path, p), name)]
        src = RowParts(arrs)
        ap = NpyAppender(os.path.join(newdir, f"{name}.npy"), src.dtype, src.shape[1:])
        try:
            for b0 in range(0, len(mine), block):
                idx = mine[b0: b0 + block]
                order = np.argsort(idx, kind="stable")          # sequential-ish reads
                got = src[idx[order]]
                out = np.empty_like(got)
                out[order] = got
                ap.append(out)
        finally:
            ap.close()
        del arrs, src
    dist.barrier()
    shutil.rmtree(os.path.join(path, parts[info.rank]))
    os.replace(newdir, os.path.join(path, parts[info.rank]))
    # the new part r holds output rows [lo, hi): rewrite the row counts the caller will publish
    rows[:] = [n * (r + 1) // info.world_size - n * r // info.world_size for r in range(info.world_size)]
    dist.barrier()


def run_norm(root: str = ".", shuffle: bool = False, seed: int = 0) -> int:
    ms = ModelSet(root).setup("NORMALIZE")
    mc = ms.mc
    cols = ms.norm_columns()
    if not cols:
        raise ValueError("no candidate/selected columns to normalize; run stats (and varsel) first")
    is_tree = mc.algorithm in TREE_ALGS
    sr = float(mc.normalize.get("sampleRate", 1.0))
    neg = bool(mc.normalize.get("sampleNegOnly", False))
    one = _norm_one_streamed if _streaming(ms) else _norm_one
    one(ms, cols, mc.dataSet, ms.pf.normalized_data, ms.pf.cleaned_data, sr, neg, shuffle, seed, is_tree)
    vpath = mc.dataSet.get("validationDataPath")
    if vpath:
        vconf = mc.dataSet.copy_with(dataPath=vpath,
                                     filterExpressions=mc.dataSet.get("validationFilterExpressions") or
                                     mc.dataSet.get("filterExpressions"))
        one(ms, cols, vconf, ms.pf.normalized_validation_data, ms.pf.cleaned_validation_data, 1.0, False,
            False, seed, is_tree)
    return 0
