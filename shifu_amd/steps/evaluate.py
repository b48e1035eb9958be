"""``eval`` step (B9): ``-new/-list/-delete/-run/-score/-norm/-confmat/-perf``.

``EvalModelProcessor.run`` (J/core/processor/EvalModelProcessor.java:138): score every eval set
with all models (``runDistScore`` :399 -> Pig ``Eval.pig`` + ``EvalScoreUDF``), sort by score,
sweep the confusion matrix into performance buckets and AUC (``runDistEval`` :901-1005,
``ConfusionMatrix`` / ``PerformanceEvaluator``), write ``EvalPerformance.json`` and gain charts;
``scoreMetaColumnNameFile`` columns (champion scores) are evaluated the same way.

EvalScore layout (``|``-delimited with a header line): tag | weight | mean | max | min | median |
model0..N | meta columns.  Scores are scaled by ``scoreScale`` (default 1000).
"""
from __future__ import annotations

import math
import os
from collections import OrderedDict

import numpy as np

from ..algos import evaluation as E
from ..algos.normalize import normalize_table
from ..config.model_config import EvalConf
from ..scoring.model_runner import ModelRunner
from ..utils.log import get_logger
from .base import ModelSet, save_dataset

_log = get_logger("steps.eval")


def _eval_confs(ms, name=None):
    evs = ms.mc.evals
    if name:
        evs = [e for e in evs if e.get("name") == name]
        if not evs:
            raise ValueError(f"eval set {name} not found")
    return evs


def new_eval(ms: ModelSet, name: str):
    if any(e.get("name") == name for e in ms.mc.evals):
        raise ValueError(f"eval set {name} already exists")
    ds = ms.mc.dataSet.to_dict()
    for k in ("validationDataPath", "validationFilterExpressions", "categoricalColumnNameFile", "autoType",
              "autoTypeThreshold"):
        ds.pop(k, None)
    ds["metaColumnNameFile"] = f"columns/{name}.meta.column.names"
    ev = EvalConf(OrderedDict(name=name, dataSet=ds, performanceBucketNum=10, performanceScoreSelector="mean",
                              scoreMetaColumnNameFile=f"columns/{name}score.meta.column.names",
                              customPaths=OrderedDict()))
    ms.mc.evals.append(ev)
    for fn in (f"{name}.meta.column.names", f"{name}score.meta.column.names"):
        p = os.path.join(ms.root, "columns", fn)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        if not os.path.exists(p):
            open(p, "w").close()
    ms.save_mc()


def delete_eval(ms: ModelSet, name: str):
    ms.mc.evals = [e for e in ms.mc.evals if e.get("name") != name]
    ms.save_mc()


def _meta_names(ms, section, key):
    p = section.get(key) if section is not None else None
    if not p:
        return []
    try:
        return ms.mc._read_names(p)
    except FileNotFoundError:
        return []


def _load_eval_data(ms, ev, runner_cols, extra_cols=()):
    from ..data.purifier import load_dataset
    ccs = {c.name: c for c in ms.ccs}
    nums, strs = [], []
    for n in set(runner_cols) | set(extra_cols):
        c = ccs.get(n)
        if c is not None and c.is_categorical():
            strs.append(n)
        elif c is not None:
            nums.append(n)
        else:
            strs.append(n)
    ds = ev.dataSet
    from ..parallel import dist
    info = dist.info()
    if info.world_size > 1:          # this rank's byte range only (no parse-all-then-slice)
        from ..data.stream import load_rank_dataset
        return load_rank_dataset(ms.mc, ds, nums, strs, require_target=False, rank=info.rank,
                                 world=info.world_size)
    return load_dataset(ms.mc, ds, nums, strs, require_target=False)


# ---- streamed eval -------------------------------------------------------------------
FIXED6, REPR, DICT, REPR_OR_EMPTY = 0, 1, 2, 3


def format_rows(fields, n: int):
    """EvalScore lines of ``n`` rows in one native pass (runtime/csrc/eval_rows.cpp).  ``fields``:
    (kind, values[, dictionary]) per column -> (bytes, int64 line ends)."""
    import ctypes
    from ..ops import _native
    lib = _native.rt()
    ncols = len(fields)
    keep, cols, blobs, offs, dn = [], [], [], [], []
    kinds = []
    for f in fields:
        kind, v = f[0], f[1]
        if kind == DICT:
            v = np.ascontiguousarray(v, dtype=np.int32)
            enc = [str(x).encode("utf-8") for x in f[2]]
            blob = np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8)
            off = np.zeros(len(enc) + 1, np.int64)
            off[1:] = np.cumsum([len(e) for e in enc]) if enc else []
            keep += [v, blob, off]
            blobs.append(blob.ctypes.data)
            offs.append(off.ctypes.data)
            dn.append(len(enc))
        else:
            v = np.ascontiguousarray(v, dtype=np.float64)
            keep.append(v)
            blobs.append(None)
            offs.append(None)
            dn.append(0)
        cols.append(v.ctypes.data)
        kinds.append(kind)
    ka = (ctypes.c_int * ncols)(*kinds)
    ca = (ctypes.c_void_p * ncols)(*cols)
    ba = (ctypes.c_void_p * ncols)(*blobs)
    oa = (ctypes.c_void_p * ncols)(*offs)
    na = (ctypes.c_long * ncols)(*dn)
    ends = np.zeros(n, np.int64)
    cap = max(1024, n * (ncols * 26 + 16))
    while True:
        buf = ctypes.create_string_buffer(cap)
        got = lib.shifu_format_rows(n, ncols, ka, ca, ba, oa, na, buf, cap, ends.ctypes.data)
        if got >= 0:
            return buf.raw[:got], ends
        cap *= 2


def _text_field(table, name, n):
    """A tag / meta column as a formatter field ('' where missing / absent)."""
    if name not in table:
        return (DICT, np.full(n, -1, np.int32), [])
    col = table[name]
    if col.kind == "str":
        return (DICT, col.values, col.dictionary)
    return (REPR_OR_EMPTY, col.values)


def _eval_streaming(ms, ev) -> bool:
    """``shifu.eval.streaming``: true / false / auto (default: stream when this rank's share of the
    eval data exceeds ``shifu.eval.inMemoryMB``, 1024)."""
    from ..config import environment
    from ..data.purifier import plan_dataset
    from ..data.stream import data_bytes
    from ..parallel import dist
    mode = str(environment.get("shifu.eval.streaming", "auto")).lower()
    if mode in ("true", "1", "on"):
        return True
    if mode in ("false", "0", "off") or ms.mc.is_multiclass():
        return False
    try:
        nbytes = data_bytes(plan_dataset(ms.mc, ev.dataSet))
    except (OSError, ValueError):
        return False
    return nbytes / max(1, dist.info().world_size) > float(environment.get("shifu.eval.inMemoryMB", 1024)) * (1 << 20)


class _StreamedEval:
    """Rank 0's view of every rank's streamed numeric eval parts (memory-mapped; ``perf_eval`` input)."""

    def __init__(self, n, w, cols):
        self.n, self.w, self.table = n, w, _GTable(cols)


def _score_eval_streamed(ms, ev, runner, meta_cols, score_meta, scale, write, nosort, local_metrics=False):
    """Out-of-core eval (the reference streams Eval.pig: EvalScoreUDF per row, then ORDER BY): this
    rank's byte range is scored chunk by chunk; each chunk's EvalScore lines are formatted natively
    and appended to the rank's run with the numeric (score, label, weight, score-meta) columns;
    each rank then orders its run by score (stable) and rank 0 k-way merges the runs into
    EvalScore (byte-identical to the in-memory writer) and reads the numeric parts memory-mapped
    for the confusion sweep.  Host memory: one chunk (+ rank 0's numeric columns for metrics)."""
    import shutil
    from ..config import environment
    from ..data import stream as DS
    from ..data.purifier import plan_dataset
    from ..data.rowstore import NpyAppender, RowParts
    from ..ops import _native
    from ..parallel import dist
    mc = ms.mc
    info = dist.info()
    ccs = {c.name: c for c in ms.ccs}
    names = set(runner.raw_columns()) | set(meta_cols) | set(score_meta)
    nums = [n for n in names if n in ccs and not ccs[n].is_categorical()]
    strs = [n for n in names if n not in nums]
    target = ev.dataSet.get("targetColumnName") or mc.dataSet.get("targetColumnName")
    if target and target not in strs and target not in nums:
        strs.append(target)
    plan = plan_dataset(mc, ev.dataSet, nums, strs)
    gpu_run = getattr(runner, "dev", None) is not None and runner.dev.type == "cuda"
    chunk = int(float(environment.get("shifu.eval.chunkMB", 2048 if gpu_run else 256)) * (1 << 20))   # 8.1 -> 7.1 s at 20M
    sel = ev.get("performanceScoreSelector", "mean") or "mean"
    pos = set(str(t) for t in (ev.dataSet.get("posTags") or mc.pos_tags))
    neg = set(str(t) for t in (ev.dataSet.get("negTags") or mc.neg_tags))
    d = ms.pf.eval_dir(ev.get("name"))
    os.makedirs(d, exist_ok=True)
    path = ms.pf.eval_score(ev)
    if os.path.isdir(path):
        path = os.path.join(path, "part-00000")
    tmp = os.path.join(d, ".parts")
    if info.rank == 0 and os.path.isdir(tmp):
        shutil.rmtree(tmp)
    dist.barrier()
    pdir = os.path.join(tmp, f"part-{info.rank:05d}")
    os.makedirs(pdir, exist_ok=True)
    aps = {k: NpyAppender(os.path.join(pdir, f"{k}.npy"), dt) for k, dt in
           (("key", np.float64), ("lab", np.int8), ("w", np.float64), ("ends", np.int64))}
    for m in score_meta:
        aps["meta:" + m] = NpyAppender(os.path.join(pdir, f"meta_{len(aps)}.npy"), np.float64)
    meta_file = {m: os.path.basename(aps["meta:" + m].path)[:-4] for m in score_meta}
    lines = open(os.path.join(pdir, "lines.bin"), "wb")
    off, n_local, cols = 0, 0, None
    try:
        # the models' numeric inputs are parsed on the GPU (K0) and normalized where they land
        gpu_cols = None
        if getattr(runner, "dev", None) is not None and runner.dev.type == "cuda":
            host_side = set(meta_cols) | set(score_meta) | {target}
            gpu_cols = [n for n in runner.raw_columns() if n in nums and n not in host_side]
        for md in DS.iter_model_data(mc, plan, chunk, info.rank, info.world_size, require_target=False,
                                     gpu_cols=gpu_cols, dev=_cuda_index(runner.dev) if gpu_cols else None):
            res = runner.score(md.table, scale)
            if cols is None:
                cols = [k for k in res if k not in ("class_scores", "pred_class")]
            n = md.n
            if write:
                fields = [_text_field(md.table, target, n), (REPR, md.w)] + [(FIXED6, res[k]) for k in cols] + \
                         [_text_field(md.table, m, n) for m in list(meta_cols) + list(score_meta)]
                blob, ends = format_rows(fields, n)
                lines.write(blob)
                aps["ends"].append(ends + off)
                off += len(blob)
            key = np.asarray(res.get(sel, res["mean"]), dtype=np.float64)
            aps["key"].append(key)
            tcol = md.table[target] if target in md.table else None
            if tcol is None:
                lab = np.full(n, -1, np.int8)
            elif tcol.kind == "str":
                dl = np.array([1 if str(t).strip() in pos else (0 if str(t).strip() in neg else -1)
                               for t in tcol.dictionary] + [-1], np.int8)
                lab = dl[np.where(tcol.values >= 0, tcol.values, len(tcol.dictionary))]
            else:
                st = np.asarray([str(t).strip() for t in tcol.strings()])
                lab = np.where(np.isin(st, list(pos)), 1, np.where(np.isin(st, list(neg)), 0, -1)).astype(np.int8)
            aps["lab"].append(lab)
            aps["w"].append(np.asarray(md.w, np.float64))
            for m in score_meta:
                aps["meta:" + m].append(md.table[m].numeric() if m in md.table else np.full(n, np.nan))
            n_local += n
    finally:
        lines.close()
        for a in aps.values():
            a.close()
    got = dist.all_gather_objects((n_local, cols))
    cols = next((c for _, c in got if c is not None), cols) or []
    sort = not nosort
    lib = _native.rt()
    if write and sort and n_local:
        key = np.load(os.path.join(pdir, "key.npy"), mmap_mode="r")
        k = np.asarray(key)
        k = np.where(np.isnan(k), -np.inf, k)          # NaN ranks with -inf; +-inf stay unclamped
        order = E.order_desc(k)
        blob = np.memmap(os.path.join(pdir, "lines.bin"), dtype=np.uint8, mode="r") if off else np.zeros(1, np.uint8)
        ends = np.ascontiguousarray(np.load(os.path.join(pdir, "ends.npy")))
        new_end = np.zeros(n_local, np.int64)
        rc = lib.shifu_gather_lines(blob.ctypes.data, ends.ctypes.data, order.ctypes.data, n_local,
                                    os.path.join(pdir, "sorted.bin").encode(), new_end.ctypes.data)
        if rc < 0:
            raise OSError("eval: writing the sorted score run failed")
        np.save(os.path.join(pdir, "sorted_ends.npy"), new_end)
        np.save(os.path.join(pdir, "sorted_key.npy"), np.ascontiguousarray(k[order]))
        del blob
    dist.barrier()
    counts = [g[0] for g in got]
    parts = [os.path.join(tmp, f"part-{r:05d}") for r in range(info.world_size)]
    if write and info.rank == 0:
        hdr = ["tag", "weight"] + cols + list(meta_cols) + list(score_meta)
        with open(path, "w") as f:
            f.write("|".join(hdr) + "\n")
        live = [(p_, c) for p_, c in zip(parts, counts) if c]
        if sort and live:
            import ctypes
            keep = []
            bl, en, ky = [], [], []
            for p_, c in live:
                b = np.memmap(os.path.join(p_, "sorted.bin"), dtype=np.uint8, mode="r")
                e = np.ascontiguousarray(np.load(os.path.join(p_, "sorted_ends.npy")))
                kk = np.ascontiguousarray(np.load(os.path.join(p_, "sorted_key.npy")))
                keep += [b, e, kk]
                bl.append(b.ctypes.data)
                en.append(e.ctypes.data)
                ky.append(kk.ctypes.data)
            R = len(live)
            rc = lib.shifu_merge_runs(R, (ctypes.c_void_p * R)(*bl), (ctypes.c_void_p * R)(*en),
                                      (ctypes.c_void_p * R)(*ky), (ctypes.c_long * R)(*[c for _, c in live]),
                                      path.encode())
            if rc != sum(c for _, c in live):
                raise OSError("eval: merging the score runs failed")
        else:
            with open(path, "ab") as f:
                for p_, c in live:
                    with open(os.path.join(p_, "lines.bin"), "rb") as src:
                        shutil.copyfileobj(src, f, 1 << 22)
        _log.info("eval %s: scored %d rows on %d rank(s) with %d models (streamed) -> %s", ev.get("name"),
                  sum(counts), info.world_size, len(runner.models), path)
    # metrics inputs on rank 0: the numeric parts, memory-mapped in rank order (local_metrics:
    # every rank its own part, for the collective EvalPerformance of algos/eval_dist.py)
    live = [p_ for p_, c in zip(parts, counts) if c] or parts[:1]
    if local_metrics:
        live = [pdir]
    elif info.rank != 0:
        return None

    def col(name):
        arrs = [np.load(os.path.join(p_, f"{name}.npy"), mmap_mode="r") for p_ in live]
        return arrs[0] if len(arrs) == 1 else RowParts(arrs)
    keyc, labc, wc = col("key"), col("lab"), col("w")
    metas = {m: np.asarray(col(meta_file[m])) for m in score_meta}
    view = _StreamedEval(len(keyc), np.asarray(wc), metas)
    res = {sel: np.asarray(keyc), "mean": np.asarray(keyc)}
    return view, res, None, np.asarray(labc), tmp


def score_eval(ms: ModelSet, ev, device=None, write: bool = True, nosort: bool = False):
    mc = ms.mc
    conv = ev.get("gbtScoreConvertStrategy") or "RAW"
    models_dir = ms.pf.eval_models_dir(ev)
    runner = ModelRunner(mc, ms.ccs, models_dir, device=device, gbt_convert=conv)
    meta_cols = _meta_names(ms, ev.dataSet, "metaColumnNameFile") if ev.dataSet else []
    score_meta = _meta_names(ms, ev, "scoreMetaColumnNameFile")
    md = _load_eval_data(ms, ev, runner.raw_columns(), list(meta_cols) + list(score_meta))
    scale = float(ev.get("scoreScale", 1000) or 1000)
    from ..parallel import dist
    info = dist.info()
    # data parallel: every rank parsed and scores only its byte range; the sorted EvalScore is a
    # merge of the ranks' locally sorted parts (Eval.pig's ORDER BY), the metrics come from a
    # tensor gather of (score, label, weight) only
    res = runner.score(md.table, scale)
    target = ev.dataSet.get("targetColumnName") or mc.dataSet.get("targetColumnName")
    tags = md.table[target].strings() if target in md.table else np.array([""] * md.n)
    if info.world_size > 1:
        if write:
            _write_scores_dp(ms, ev, md, res, tags, list(meta_cols) + list(score_meta), nosort)
        return _gather_eval_numeric(ms, ev, md, res, tags, score_meta) + (score_meta,)
    if write:
        d = ms.pf.eval_dir(ev.get("name"))
        os.makedirs(d, exist_ok=True)
        path = ms.pf.eval_score(ev)
        if os.path.isdir(path):
            path = os.path.join(path, "part-00000")
        cols = [k for k in res if k not in ("class_scores", "pred_class")]
        with open(path, "w") as f:
            hdr = ["tag", "weight"] + cols + list(meta_cols) + list(score_meta)
            f.write("|".join(hdr) + "\n")
            mats = [np.asarray(res[k]) for k in cols]
            metas = [md.table[m].strings() if m in md.table else np.array([""] * md.n)
                     for m in list(meta_cols) + list(score_meta)]
            # rows leave sorted by score, descending (Eval.pig ORDER BY), except for
            # classification or `eval -score -nosort` (EvalModelProcessor.java:432)
            order = range(md.n)
            if not (nosort or mc.is_multiclass()):
                sel = ev.get("performanceScoreSelector", "mean") or "mean"
                key = np.asarray(res.get(sel, res.get("mean")), dtype=np.float64)
                if key.ndim == 1 and len(key) == md.n:
                    order = E.order_desc(key)
            for i in order:
                row = [str(tags[i]), repr(float(md.w[i]))]
                row += [f"{float(m[i]):.6f}" if m.ndim == 1 else ",".join(f"{v:.6f}" for v in m[i]) for m in mats]
                row += [str(m[i]) for m in metas]
                f.write("|".join(row) + "\n")
        _log.info("eval %s: scored %d rows with %d models -> %s", ev.get("name"), md.n, len(runner.models), path)
    return md, res, tags, score_meta


class _GCol:
    def __init__(self, v):
        self.v = v

    def strings(self):
        return self.v

    def numeric(self):
        if isinstance(self.v, np.ndarray) and self.v.dtype.kind == "f":
            return self.v
        out = np.full(len(self.v), np.nan)
        for i, x in enumerate(self.v):
            try:
                out[i] = float(x)
            except (TypeError, ValueError):
                pass
        return out


class _GTable(dict):
    def __getitem__(self, k):
        return _GCol(dict.__getitem__(self, k))


class _GatheredEval:
    def __init__(self, n, w, cols):
        self.n, self.w, self.table = n, w, _GTable(cols)


def _score_rows(md, res, tags, metas, order):
    cols = [k for k in res if k not in ("class_scores", "pred_class")]
    mats = [np.asarray(res[k]) for k in cols]
    for i in order:
        row = [str(tags[i]), repr(float(md.w[i]))]
        row += [f"{float(m[i]):.6f}" if m.ndim == 1 else ",".join(f"{v:.6f}" for v in m[i]) for m in mats]
        row += [str(m[i]) for m in metas]
        yield "|".join(row)


def _write_scores_dp(ms, ev, md, res, tags, meta_names, nosort):
    """Every rank writes its rows sorted by score (full-precision key prefix) to a temp part; rank
    0 k-way merges the parts into EvalScore (stable: equal scores keep rank = row order, exactly the
    single-process stable sort) while streaming, then removes the parts."""
    import heapq
    from ..parallel import dist
    mc = ms.mc
    info = dist.info()
    d = ms.pf.eval_dir(ev.get("name"))
    os.makedirs(d, exist_ok=True)
    path = ms.pf.eval_score(ev)
    if os.path.isdir(path):
        path = os.path.join(path, "part-00000")
    metas = [md.table[m].strings() if m in md.table else np.array([""] * md.n) for m in meta_names]
    sort = not (nosort or mc.is_multiclass())
    key = None
    order = range(md.n)
    if sort:
        sel = ev.get("performanceScoreSelector", "mean") or "mean"
        key = np.asarray(res.get(sel, res.get("mean")), dtype=np.float64)
        if key.ndim == 1 and len(key) == md.n:
            order = E.order_desc(key)
        else:
            key = None
    part = f"{path}.rank{info.rank:05d}"
    with open(part, "w") as f:
        for i, line in zip(order, _score_rows(md, res, tags, metas, order)):
            f.write((f"{float(-key[i])!r}\t" if key is not None else "") + line + "\n")
    dist.barrier()
    if info.rank == 0:
        cols = [k for k in res if k not in ("class_scores", "pred_class")]
        hdr = ["tag", "weight"] + cols + list(meta_names)
        parts = [f"{path}.rank{r:05d}" for r in range(info.world_size)]
        fhs = [open(p_) for p_ in parts]
        with open(path, "w") as out:
            out.write("|".join(hdr) + "\n")
            if key is not None:
                merged = heapq.merge(*fhs, key=lambda l: float(l.split("\t", 1)[0]))
                for l in merged:
                    out.write(l.split("\t", 1)[1])
            else:
                for fh in fhs:
                    for l in fh:
                        out.write(l)
        for fh, p_ in zip(fhs, parts):
            fh.close()
            os.remove(p_)
        _log.info("eval %s: merged %d rank parts -> %s", ev.get("name"), info.world_size, path)
    dist.barrier()


def _gather_eval_numeric(ms, ev, md, res, tags, score_meta):
    """(score or predicted class, label code, weight, score-meta columns) of every rank -> rank 0
    as tensors (dist.gather_cat); rank 0 gets an eval view with synthetic tag strings carrying
    the same labels, the others their own shard."""
    import torch
    from ..parallel import dist
    mc = ms.mc
    info = dist.info()
    dev = dist.coll_device()
    tg = np.asarray([str(t).strip() for t in tags])
    if mc.is_multiclass():
        lab = np.array([next((i for i, g in enumerate(mc.tags()) if t in g), -1) for t in tg], np.int64)
        score = np.asarray(res["pred_class"], np.float64)
    else:
        pos = set(ev.dataSet.get("posTags") or mc.pos_tags)
        neg = set(ev.dataSet.get("negTags") or mc.neg_tags)
        lab = np.where(np.isin(tg, list(pos)), 1, np.where(np.isin(tg, list(neg)), 0, -1)).astype(np.int64)
        sel = ev.get("performanceScoreSelector", "mean") or "mean"
        score = np.asarray(res.get(sel, res["mean"]), np.float64)
    arrays = {"score": score, "lab": lab, "w": np.asarray(md.w, np.float64)}
    for m in score_meta:
        arrays["meta:" + m] = md.table[m].numeric() if m in md.table else np.full(md.n, np.nan)
    got = {k: dist.gather_cat(torch.as_tensor(np.ascontiguousarray(v)).to(dev)) for k, v in arrays.items()}
    if info.rank != 0:
        return md, res, tags
    got = {k: v.cpu().numpy() for k, v in got.items()}
    lab = got["lab"]
    if mc.is_multiclass():
        names = [str(g[0]) for g in mc.tags()]
        tags = np.array([names[k] if k >= 0 else "" for k in lab], dtype=object)
        res = {"pred_class": got["score"].astype(np.int64)}
    else:
        pos = list(ev.dataSet.get("posTags") or mc.pos_tags)
        neg = list(ev.dataSet.get("negTags") or mc.neg_tags)
        tags = np.where(lab == 1, str(pos[0]) if pos else "1", np.where(lab == 0, str(neg[0]) if neg else "0", ""))
        sel = ev.get("performanceScoreSelector", "mean") or "mean"
        res = {sel: got["score"], "mean": got["score"]}
    cols = {m: got["meta:" + m] for m in score_meta}
    return _GatheredEval(len(lab), got["w"], cols), res, tags


def perf_eval(ms: ModelSet, ev, md, res, tags, score_meta=(), device=None, lab=None, collective: bool = False):
    """``lab`` (optional, numeric labels of the streamed eval): binary 1 pos / 0 neg / -1 neither,
    multi-class the tag-group index; replaces the per-row tag strings.  ``collective``: every
    rank passes its own rows and the metrics are the exact global ones (algos/eval_dist.py,
    binary only); rank 0 writes the files."""
    from ..parallel import dist
    mc = ms.mc
    if collective:
        from ..algos import eval_dist
        perf_fn, writer = eval_dist.performance, dist.info().rank == 0
    else:
        perf_fn, writer = E.performance, True
    d = ms.pf.eval_dir(ev.get("name"))
    os.makedirs(d, exist_ok=True)
    pos = set(ev.dataSet.get("posTags") or mc.pos_tags)
    neg = set(ev.dataSet.get("negTags") or mc.neg_tags)
    nb = int(ev.get("performanceBucketNum", 10) or 10)
    scale = float(ev.get("scoreScale", 1000) or 1000)
    if mc.is_multiclass():
        truth = np.asarray(lab) if lab is not None else \
            np.array([next((i for i, g in enumerate(mc.tags()) if t in g), -1) for t in tags])
        ok = truth >= 0
        cm = E.multiclass_confusion(res["pred_class"][ok], truth[ok], len(mc.tags()))
        with open(ms.pf.eval_confusion_matrix(ev), "w") as f:
            f.write("\n".join("|".join(str(int(v)) for v in r) for r in cm) + "\n")
        acc = float(np.trace(cm) / max(cm.sum(), 1))
        _log.info("eval %s multi-class accuracy %.6f", ev.get("name"), acc)
        with open(ms.pf.eval_performance(ev), "w") as f:
            f.write(E.to_json({"version": "0.13.0", "accuracy": acc, "confusionMatrix": cm.tolist()}))
        return {"accuracy": acc}
    sel = ev.get("performanceScoreSelector", "mean") or "mean"
    score = np.asarray(res.get(sel, res["mean"]))
    if lab is not None:
        lab = np.asarray(lab)
        valid = lab >= 0
        is_pos = lab[valid] == 1
    else:
        tg = np.asarray([str(t).strip() for t in tags])
        valid = np.isin(tg, list(pos | neg))
        is_pos = np.isin(tg[valid], list(pos))
    w = np.asarray(md.w)[valid] if ev.dataSet.get("weightColumnName") else None
    perf = perf_fn(score[valid], is_pos, w, nb, max_score=scale, device=device)
    if writer:
        with open(ms.pf.eval_performance(ev), "w") as f:
            f.write(E.to_json(perf))
        _log.info("eval %s: AUC(ROC)=%.6f AUC(PR)=%.6f weighted AUC=%.6f", ev.get("name"), perf["areaUnderRoc"],
                  perf["areaUnderPr"], perf["weightedAreaUnderRoc"])
    # champion / meta score columns (EvalModelProcessor.runDistEval :911-935): each column's
    # performance goes to EvalMetaScore/<column>EvalPerformance.json
    champions = []
    for m in score_meta:
        if m in md.table:
            sv = md.table[m].numeric()[valid]
            okm = np.isfinite(sv)
            mx = float(np.nanmax(sv[okm])) if okm.any() else -math.inf
            if collective:
                mx = dist.all_reduce_max_scalar(mx)
            p2 = perf_fn(sv[okm], is_pos[okm], None if w is None else w[okm], nb,
                         max_score=mx if math.isfinite(mx) else 1.0, device=device)
            champions.append((m, p2))
            if writer:
                md_dir = os.path.join(d, "EvalMetaScore")
                os.makedirs(md_dir, exist_ok=True)
                with open(os.path.join(md_dir, f"{m}EvalPerformance.json"), "w") as f:
                    f.write(E.to_json(p2))
    if writer:
        # gain / PR / ROC pages and the per-series CSVs (ConfusionMatrix.java:543-596 without
        # champion columns, EvalModelProcessor.java:937-1001 with them)
        from ..algos.eval_reports import write_eval_reports
        evn = ev.get("name")
        model_name = mc.basic.get("name") or "model"
        series = ([(evn, perf)] if not champions else [(f"{model_name}-{evn}", perf)] + champions)
        write_eval_reports(d, evn, model_name, series, bool(ev.dataSet.get("weightColumnName")))
    return perf


def norm_eval(ms: ModelSet, ev, strict: bool = False):
    """``eval -norm [-strict]``: write the normalized eval data (NN inputs) for external scorers.
    ``-strict``: every selected column must be present in the eval data (otherwise the missing
    ones normalize as missing values)."""
    cols = ms.selected()
    if strict:
        from ..data.reader import read_header
        ds = ev.dataSet

        def _abs(x):
            return x if not x or os.path.isabs(x) else os.path.join(ms.root, x)
        hdr = set(read_header(_abs(ds.get("headerPath")), ds.get("headerDelimiter") or "|",
                              _abs(ds.get("dataPath")), ds.get("dataDelimiter") or "|"))
        if hdr:
            missing = [c.name for c in cols if c.name not in hdr]
            if missing:
                raise ValueError(f"eval -norm -strict: selected columns missing from {ev.get('name')}: {missing}")
    md = _load_eval_data(ms, ev, [c.name for c in cols])
    X, names, _ = normalize_table(ms.mc, ms.ccs, md.table, columns=cols)
    save_dataset(ms.pf.eval_normalized(ev), {"X": X, "y": md.y, "w": md.w.astype(np.float32)},
                 {"n": int(md.n), "input_names": names})
    return X


def _cuda_index(dev):
    import torch
    d = torch.device(dev)
    return d if d.index is not None else torch.device("cuda", torch.cuda.current_device())


def run_eval(root: str = ".", action: str = "run", name: str | None = None, device=None, nosort: bool = False,
             strict: bool = False) -> int:
    from ..parallel import dist
    if action in ("new", "list", "delete", "norm") and dist.info().world_size > 1:
        # model-set edits and the normalized eval export: rank 0 alone
        if dist.info().rank == 0:
            with dist.local_only():
                return run_eval(root, action, name, device, nosort, strict)
        return 0
    ms = ModelSet(root)
    if action == "new":
        new_eval(ms, name)
        return 0
    if action == "list":
        for e in ms.mc.evals:
            print(e.get("name"))
        return 0
    if action == "delete":
        delete_eval(ms, name)
        return 0
    ms.setup("EVAL", validate=False)
    for ev in _eval_confs(ms, name):
        if action == "norm":
            norm_eval(ms, ev, strict)
            continue
        from ..parallel import dist
        if _eval_streaming(ms, ev):
            runner = ModelRunner(ms.mc, ms.ccs, ms.pf.eval_models_dir(ev), device=device,
                                 gbt_convert=ev.get("gbtScoreConvertStrategy") or "RAW")
            meta_cols = _meta_names(ms, ev.dataSet, "metaColumnNameFile") if ev.dataSet else []
            score_meta = _meta_names(ms, ev, "scoreMetaColumnNameFile")
            from ..config import environment
            coll = dist.info().world_size > 1 and not ms.mc.is_multiclass() and \
                environment.get_bool("shifu.eval.distPerf", True)
            out = _score_eval_streamed(ms, ev, runner, meta_cols, score_meta,
                                       float(ev.get("scoreScale", 1000) or 1000), True, nosort, local_metrics=coll)
            if coll and action in ("run", "perf", "confmat"):
                view, res, _, lab, tmp = out          # this rank's rows: exact global metrics, no gather
                perf_eval(ms, ev, view, res, None, score_meta, device, lab=lab, collective=True)
            elif out is not None and action in ("run", "perf", "confmat"):
                view, res, _, lab, tmp = out
                with dist.local_only():
                    perf_eval(ms, ev, view, res, None, score_meta, device, lab=lab)
            dist.barrier()
            if dist.info().rank == 0 and out is not None:
                import shutil
                shutil.rmtree(out[4], ignore_errors=True)
            continue
        md, res, tags, score_meta = score_eval(ms, ev, device, nosort=nosort)
        if action in ("run", "perf", "confmat") and dist.info().rank == 0:
            with dist.local_only():
                perf_eval(ms, ev, md, res, tags, score_meta, device)
    return 0
