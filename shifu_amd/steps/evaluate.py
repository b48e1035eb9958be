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
                    order = np.argsort(-key, kind="stable")
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
            order = np.argsort(-key, kind="stable")
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
    dev = torch.device("cuda", torch.cuda.current_device()) if info.backend == "nccl" else torch.device("cpu")
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


def _gather_scores(md, res, tags, meta_names):
    """All ranks' (tags, weights, score arrays, meta columns) -> one row set on rank 0 (rank order
    = row order).  Other ranks get their own shard back."""
    import torch.distributed as tdist
    from ..parallel import dist
    payload = (np.asarray(tags), np.asarray(md.w), {k: np.asarray(v) for k, v in res.items()},
               {m: (md.table[m].strings() if m in md.table else np.array([""] * md.n)) for m in meta_names})
    # gathered on rank 0 only (the other ranks neither receive nor hold the full score set)
    parts = [None] * dist.info().world_size if dist.info().rank == 0 else None
    tdist.gather_object(payload, parts, dst=0)
    if dist.info().rank != 0:
        return md, res, tags
    tags = np.concatenate([p[0] for p in parts])
    w = np.concatenate([p[1] for p in parts])
    res = {k: np.concatenate([p[2][k] for p in parts]) for k in parts[0][2]}
    cols = {m: np.concatenate([p[3][m] for p in parts]) for m in meta_names}
    return _GatheredEval(len(tags), w, cols), res, tags


def perf_eval(ms: ModelSet, ev, md, res, tags, score_meta=(), device=None):
    mc = ms.mc
    d = ms.pf.eval_dir(ev.get("name"))
    os.makedirs(d, exist_ok=True)
    pos = set(ev.dataSet.get("posTags") or mc.pos_tags)
    neg = set(ev.dataSet.get("negTags") or mc.neg_tags)
    nb = int(ev.get("performanceBucketNum", 10) or 10)
    scale = float(ev.get("scoreScale", 1000) or 1000)
    if mc.is_multiclass():
        truth = np.array([next((i for i, g in enumerate(mc.tags()) if t in g), -1) for t in tags])
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
    tg = np.asarray([str(t).strip() for t in tags])
    valid = np.isin(tg, list(pos | neg))
    is_pos = np.isin(tg[valid], list(pos))
    w = md.w[valid] if ev.dataSet.get("weightColumnName") else None
    perf = E.performance(score[valid], is_pos, w, nb, max_score=scale, device=device)
    with open(ms.pf.eval_performance(ev), "w") as f:
        f.write(E.to_json(perf))
    E.write_gain_chart(ms.pf.eval_gain_chart(ev, "gainchart", "html"), ms.pf.eval_gain_chart(ev, "gainchart", "csv"),
                       perf, ev.get("name"))
    _log.info("eval %s: AUC(ROC)=%.6f AUC(PR)=%.6f weighted AUC=%.6f", ev.get("name"), perf["areaUnderRoc"],
              perf["areaUnderPr"], perf["weightedAreaUnderRoc"])
    # champion / meta score columns
    for m in score_meta:
        if m in md.table:
            sv = md.table[m].numeric()[valid]
            okm = np.isfinite(sv)
            p2 = E.performance(sv[okm], is_pos[okm], None if w is None else w[okm], nb,
                               max_score=float(np.nanmax(sv)) if okm.any() else 1.0, device=device)
            with open(os.path.join(d, f"{m}.EvalPerformance.json"), "w") as f:
                f.write(E.to_json(p2))
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
        md, res, tags, score_meta = score_eval(ms, ev, device, nosort=nosort)
        from ..parallel import dist
        if action in ("run", "perf", "confmat") and dist.info().rank == 0:
            with dist.local_only():
                perf_eval(ms, ev, md, res, tags, score_meta, device)
    return 0
