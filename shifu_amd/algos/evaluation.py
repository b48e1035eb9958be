"""Evaluation metrics (H14): confusion-matrix sweep, performance buckets, AUC, gain charts.

``ConfusionMatrix.bufferedComputeConfusionMatrixAndPerformance`` (J/core/ConfusionMatrix.java:276-507)
streams the score-sorted rows, moving one record at a time from FN->TP or TN->FP, and emits a
PerformanceObject whenever FPR / recall / action rate / weighted variants cross the next
``1/performanceBucketNum`` boundary (at most one bucket per row) and when the score drops below
the next score bin.  ``AreaUnderCurve`` (J/core/eval/AreaUnderCurve.java:56-117) integrates the
bucket points with trapezoids.

Here the whole sweep is a device sort + cumulative sums; the bucket boundaries are found with
``searchsorted`` over the monotone cumulative curves (``first i > prev with m[i] >= k/B``), which
reproduces the one-bucket-per-row rule exactly.
"""
from __future__ import annotations

import csv
import json
import math
from collections import OrderedDict

import numpy as np
import torch

from ..utils.trace import trace_range

PO_FIELDS = ("binNum", "binLowestScore", "actionRate", "weightedActionRate", "recall", "weightedRecall",
             "precision", "weightedPrecision", "fpr", "weightedFpr", "liftUnit", "weightLiftUnit",
             "scoreCount", "scoreWgtCount", "tp", "fp", "tn", "fn", "weightedTp", "weightedFp", "weightedTn",
             "weightedFn")


def _div(a, b):
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.where(b != 0, a / np.where(b != 0, b, 1), np.nan)


def _po(i, cm, bin_num=0, score_count=0.0, score_wcount=0.0, first=False):
    tp, fp, fn, tn, wtp, wfp, wfn, wtn, score = (float(cm[k][i]) for k in
                                                ("tp", "fp", "fn", "tn", "wtp", "wfp", "wfn", "wtn", "score"))
    tot, wtot = tp + fp + fn + tn, wtp + wfp + wfn + wtn
    f = lambda a, b: (a / b) if b != 0 else float("nan")
    po = OrderedDict(binNum=bin_num, binLowestScore=score,
                     actionRate=f(tp + fp, tot), weightedActionRate=f(wtp + wfp, wtot),
                     recall=f(tp, tp + fn), weightedRecall=f(wtp, wtp + wfn),
                     precision=f(tp, tp + fp), weightedPrecision=f(wtp, wtp + wfp),
                     fpr=f(fp, fp + tn), weightedFpr=f(wfp, wfp + wtn),
                     liftUnit=f(tp, (tp + fp) * (tp + fn) / tot) if tot else float("nan"),
                     weightLiftUnit=f(wtp, (wtp + wfp) * (wtp + wfn) / wtot) if wtot else float("nan"),
                     scoreCount=score_count, scoreWgtCount=score_wcount,
                     tp=tp, fp=fp, tn=tn, fn=fn, weightedTp=wtp, weightedFp=wfp, weightedTn=wtn, weightedFn=wfn)
    if first:
        po["precision"] = po["weightedPrecision"] = 1.0
        po["liftUnit"] = po["weightLiftUnit"] = 0.0
    return po


def _bucket_indices(metric, nb: int, start: int = 1) -> list:
    """Rows (>= start) where the k-th bucket is emitted: first row after the previous emission
    whose metric >= k/nb.  ``metric``: numpy array or (device) tensor.  The first row whose
    running max reaches k/nb is the first row whose value does (NaN never does), so each bucket
    is one compare + first-true argmax -- no running-max scan of the whole curve."""
    m = torch.as_tensor(metric)
    out, prev, k = [], start - 1, 1
    cap = 1.0 / nb
    n = m.numel()
    while True:
        hit = m >= k * cap
        j = int(torch.argmax(hit.to(torch.uint8)).item()) if n else 0
        if n == 0 or not bool(hit[j]):
            j = n
        j = max(j, prev + 1)
        if j >= n:
            break
        out.append((k, j))
        prev, k = j, k + 1
    return out


def order_desc(key, device=None):
    """Stable descending order of scores: ties keep row order, NaN ranks with -inf (last).  K16's
    radix sort on the GPU (ops/csrc/sort_kernels.hip) for a device tensor or, when a GPU is
    present, for a large host array; a stable argsort otherwise.  Returns the input's kind
    (device tensor / numpy int64)."""
    if torch.is_tensor(key):
        if key.device.type == "cuda":
            from ..ops.stats_ops import sort_desc
            return sort_desc(key).long()
        k = key.to(torch.float64)
        return torch.argsort(-torch.where(torch.isnan(k), torch.full_like(k, -math.inf), k), stable=True)
    dev = device or (torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
    k = np.asarray(key, dtype=np.float64)
    if torch.device(dev).type == "cuda" and k.size >= 4096:
        from ..ops.stats_ops import sort_desc
        return sort_desc(torch.from_numpy(np.ascontiguousarray(k)).to(dev)).long().cpu().numpy()
    return np.argsort(-np.where(np.isnan(k), -np.inf, k), kind="stable").astype(np.int64)


def _as_dev(x, dev):
    if torch.is_tensor(x):
        return x.to(dev, torch.float64)
    return torch.as_tensor(np.asarray(x, dtype=np.float64), device=dev)


def confusion_sweep_t(score, is_pos, weight=None, device=None, max_score: float | None = None) -> dict:
    """Sort descending by score and return cumulative confusion tensors of length N+1 on the
    device (index 0 = the initial matrix with every record predicted negative).  Inputs: numpy
    arrays or tensors (device-resident scores are not copied through the host)."""
    dev = device or (score.device if torch.is_tensor(score) else
                     (torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")))
    s = _as_dev(score, dev)
    p = _as_dev(is_pos, dev)
    w = torch.ones_like(s) if weight is None else _as_dev(weight, dev)
    with trace_range("eval.sort"):
        order = order_desc(s)
        s, p, w = s[order], p[order], w[order]
    with trace_range("eval.sweep"):
        z = torch.zeros(1, dtype=torch.float64, device=dev)
        tp = torch.cat([z, torch.cumsum(p, 0)])
        fp = torch.cat([z, torch.cumsum(1 - p, 0)])
        wtp = torch.cat([z, torch.cumsum(p * w, 0)])
        wfp = torch.cat([z, torch.cumsum((1 - p) * w, 0)])
    P, Nn, WP, WN = tp[-1], fp[-1], wtp[-1], wfp[-1]
    ms = float(s.max().item()) if max_score is None and s.numel() else (max_score or 0.0)
    sc = torch.cat([torch.tensor([ms], dtype=torch.float64, device=dev), s])
    return dict(tp=tp, fp=fp, fn=P - tp, tn=Nn - fp, wtp=wtp, wfp=wfp, wfn=WP - wtp, wtn=WN - wfp, score=sc,
                w=torch.cat([z, w]))


def confusion_sweep(score, is_pos, weight=None, device=None, max_score: float | None = None):
    """``confusion_sweep_t`` as host numpy arrays."""
    return {k: v.cpu().numpy() for k, v in confusion_sweep_t(score, is_pos, weight, device, max_score).items()}


def auc(points, xk, yk) -> float:
    if len(points) < 2:
        return 0.0
    a = 0.0
    for p0, p1 in zip(points, points[1:]):
        x1, y1, x2, y2 = p0[xk], p0[yk], p1[xk], p1[yk]
        if any(math.isnan(v) for v in (x1, y1, x2, y2)):
            continue
        a += (y2 + y1) * (x2 - x1) / 2.0
    return a


def performance(score, is_pos, weight=None, num_bucket: int = 10, max_score: float = 1000.0,
                min_score: float = 0.0, device=None, version: str = "0.13.0"):
    """-> PerformanceResult dict (EvalPerformance.json).  The sweep, the curves and the bucket
    searches stay on the device; only the emitted rows' confusion values come to the host."""
    cm = confusion_sweep_t(score, is_pos, weight, device, max_score)
    n = cm["tp"].numel() - 1

    def div(a, b):
        return torch.where(b != 0, a / torch.where(b != 0, b, torch.ones_like(b)), torch.full_like(a, math.nan))
    wtot = cm["wtp"] + cm["wfp"] + cm["wfn"] + cm["wtn"]
    curves = (("roc", div(cm["fp"], cm["fp"] + cm["tn"])), ("pr", div(cm["tp"], cm["tp"] + cm["fn"])),
              ("gains", torch.arange(n + 1, dtype=torch.float64, device=cm["tp"].device) / max(n, 1)),
              ("weightedRoc", div(cm["wfp"], cm["wfp"] + cm["wtn"])),
              ("weightedPr", div(cm["wtp"], cm["wtp"] + cm["wfn"])),
              ("weightedGains", div(cm["wtp"] + cm["wfp"], wtot)))
    marks = {key: _bucket_indices(metric, num_bucket) for key, metric in curves}
    del curves, wtot
    # score buckets: bucket k closes at the first row after the previous emission whose score
    # <= max_score - k * bin_score (binary searches on the descending scores)
    bin_score = (max_score - min_score) / num_bucket
    neg = -cm["score"][1:]                                           # ascending; NaN scores last
    neg = torch.where(torch.isnan(neg), torch.full_like(neg, math.inf), neg)
    wcum = torch.cumsum(cm["w"], 0)
    emits, k, last = [], 1, 0
    while last < n:
        thr = max_score - k * bin_score
        j = max(int(torch.searchsorted(neg, torch.tensor([-thr], dtype=neg.dtype, device=neg.device)).item()) + 1,
                last + 1)
        if j > n:
            break
        emits.append((k, j, last))
        k += 1
        last = j
    # one gather of every emitted row
    idx = sorted({0} | {j for v in marks.values() for _, j in v} | {j for _, j, _ in emits} |
                 {l for _, _, l in emits})
    it = torch.tensor(idx, dtype=torch.long, device=cm["tp"].device)
    keys = ("tp", "fp", "fn", "tn", "wtp", "wfp", "wfn", "wtn", "score")
    host = torch.stack([cm[c][it] for c in keys] + [wcum[it]]).cpu().numpy()
    pos = {j: q for q, j in enumerate(idx)}
    hcm = {c: host[r] for r, c in enumerate(keys)}
    hw = host[len(keys)]
    first = _po(0, hcm, first=True)
    lists = OrderedDict()
    for key in ("roc", "pr", "gains", "weightedRoc", "weightedPr", "weightedGains"):
        lists[key] = [first] + [_po(pos[j], hcm, kk) for kk, j in marks[key]]
    ms = [first] + [_po(pos[j], hcm, kk, float(j - l), float(hw[pos[j]] - hw[pos[l]])) for kk, j, l in emits]
    res = OrderedDict(version=version)
    res["areaUnderRoc"] = auc(lists["roc"], "fpr", "recall")
    res["weightedAreaUnderRoc"] = auc(lists["weightedRoc"], "weightedFpr", "weightedRecall")
    res["areaUnderPr"] = auc(lists["pr"], "recall", "precision")
    res["weightedAreaUnderPr"] = auc(lists["weightedPr"], "weightedRecall", "weightedPrecision")
    for key in ("pr", "weightedPr", "roc", "weightedRoc", "gains", "weightedGains"):
        res[key] = lists[key]
    res["modelScoreList"] = ms
    return res


def exact_auc(score, is_pos) -> float:
    """Rank-based ROC AUC (ties averaged) — a precise reference for tests."""
    s = np.asarray(score, dtype=np.float64)
    y = np.asarray(is_pos).astype(bool)
    from scipy.stats import rankdata
    r = rankdata(s)
    npos, nneg = y.sum(), (~y).sum()
    if npos == 0 or nneg == 0:
        return float("nan")
    return float((r[y].sum() - npos * (npos + 1) / 2) / (npos * nneg))


def multiclass_confusion(pred: np.ndarray, truth: np.ndarray, n_classes: int, weight=None) -> np.ndarray:
    """``computeConfusionMatixForMultipleClassification`` (J/core/ConfusionMatrix.java:625):
    rows = true class, cols = predicted class."""
    m = np.zeros((n_classes, n_classes))
    np.add.at(m, (truth.astype(int), pred.astype(int)), 1.0 if weight is None else weight)
    return m


def to_json(obj) -> str:
    def clean(v):
        if isinstance(v, float) and (math.isnan(v) or math.isinf(v)):
            return "NaN" if math.isnan(v) else ("Infinity" if v > 0 else "-Infinity")
        if isinstance(v, dict):
            return OrderedDict((k, clean(x)) for k, x in v.items())
        if isinstance(v, list):
            return [clean(x) for x in v]
        return v
    return json.dumps(clean(obj), indent=2)
