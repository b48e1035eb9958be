"""Eval report files (the reference's ``GainChart`` / ``ConfusionMatrix.generateChartAndJsonPerfFiles``
/ ``EvalModelProcessor.runDistEval`` outputs, J/core/eval/GainChart.java:39-1224,
J/core/ConfusionMatrix.java:543-596, J/core/processor/EvalModelProcessor.java:937-1001).

Per eval set ``<ev>``, in ``evals/<ev>/``:

* ``<ev>_gainchart.html`` -- seven charts (weighted / unit-wise operation point x weighted /
  unit-wise recall, model score x weighted / unit-wise recall, score distribution), every chart
  overlaying the model and every champion score column;
* ``<ev>_prroc.html`` -- weighted / unit-wise PR and ROC curves, same overlay;
* per series name ``<name>_unit_wise_{gainchart,pr,roc}.csv``, ``<name>_weighted_{gainchart,pr,roc}.csv``
  (when the eval set has a weight column) and ``<name>_modelscore_gainchart.csv``, in
  ``GainChart.generateCsv``'s layout (header, ``#.####`` values, ``Double.toString`` score).
  Series names: ``<ev>`` alone without champion columns; ``<model>-<ev>`` followed by every
  champion column with them.

The pages are self-contained (inline SVG; the reference loads Highcharts from a CDN) and carry
each series' points as ``var data_<j>`` arrays in the reference's order.
"""
from __future__ import annotations

import html
import json
import math
import os
from decimal import ROUND_HALF_EVEN, Decimal

CSV_HEADER = ("ActionRate,WeightedActionRate,Recall,WeightedRecall,Precision,WeightedPrecision,FPR,WeightedFPR,"
              "BinLowestScore\n")
COLORS = ["#1f77b4", "#d62728", "#2ca02c", "#ff7f0e", "#9467bd", "#8c564b", "#e377c2", "#7f7f7f", "#bcbd22",
          "#17becf"]
_Q4 = Decimal("0.0001")


def java_df(x) -> str:
    """``new DecimalFormat("#.####").format(x)``: HALF_EVEN on the exact binary value, at most four
    decimals, no trailing zeros, no leading-zero-less forms ("0.5", "12", "-0.0001", "-0")."""
    x = float(x)
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "∞" if x > 0 else "-∞"
    q = Decimal(x).quantize(_Q4, rounding=ROUND_HALF_EVEN)
    neg = q.is_signed()
    s = format(abs(q), "f")
    if "." in s:
        s = s.rstrip("0").rstrip(".")
    return ("-" if neg else "") + s


def java_double(x) -> str:
    """``Double.toString(x)``: plain decimal in [1e-3, 1e7), else ``d.dddE<exp>``; shortest
    round-trip digits (Python's repr digits)."""
    x = float(x)
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    if x == 0.0:
        return "-0.0" if math.copysign(1.0, x) < 0 else "0.0"
    a = abs(x)
    sign = "-" if x < 0 else ""
    if 1e-3 <= a < 1e7:
        s = repr(a)
        if "e" in s or "E" in s:                 # repr may use an exponent for some values here
            s = format(Decimal(s), "f")
        if "." not in s:
            s += ".0"
        return sign + s
    t = Decimal(repr(a)).as_tuple()              # shortest round-trip digits
    ds = "".join(map(str, t.digits)).rstrip("0") or "0"
    exp = len(t.digits) + t.exponent - 1
    mant = ds[0] + "." + (ds[1:] or "0")
    return f"{sign}{mant}E{exp}"


def write_perf_csv(path: str, pos: list) -> None:
    """``GainChart.generateCsv``: one row per PerformanceObject."""
    with open(path, "w") as f:
        f.write(CSV_HEADER)
        for po in pos:
            f.write(",".join([java_df(po["actionRate"]), java_df(po["weightedActionRate"]), java_df(po["recall"]),
                              java_df(po["weightedRecall"]), java_df(po["precision"]),
                              java_df(po["weightedPrecision"]), java_df(po["fpr"]), java_df(po["weightedFpr"]),
                              java_double(po["binLowestScore"])]) + "\n")


def _num(v):
    v = float(v)
    return None if (math.isnan(v) or math.isinf(v)) else v


# (panel title, y label, list key, x field, y field, x scale (100: percent))
GAIN_PANELS = [
    ("Weighted Operation Point", "Weighted Recall", "weightedGains", "weightedActionRate", "weightedRecall", 100),
    ("Weighted Operation Point", "Unit-wise Recall", "weightedGains", "weightedActionRate", "recall", 100),
    ("Unit-wise Operation Point", "Weighted Recall", "gains", "actionRate", "weightedRecall", 100),
    ("Unit-wise Operation Point", "Unit-wise Recall", "gains", "actionRate", "recall", 100),
    ("Model Score", "Weighted Recall", "modelScoreList", "binLowestScore", "weightedRecall", 1),
    ("Model Score", "Unit-wise Recall", "modelScoreList", "binLowestScore", "recall", 1),
    ("Score Distribution", "Score Count", "modelScoreList", "binLowestScore", "scoreCount", 1),
]
PRROC_PANELS = [
    ("Weighted PR Curve", "Weighted Precision", "weightedPr", "weightedRecall", "weightedPrecision", 100),
    ("Weighted PR Curve", "Unit-wise Precision", "weightedPr", "weightedRecall", "precision", 100),
    ("Unit-wise PR Curve", "Weighted Precision", "pr", "recall", "weightedPrecision", 100),
    ("Unit-wise PR Curve", "Unit-wise Precision", "pr", "recall", "precision", 100),
    ("Weighted ROC Curve", "Weighted Recall", "weightedRoc", "weightedFpr", "weightedRecall", 100),
    ("Weighted ROC Curve", "Unit-wise Recall", "weightedRoc", "weightedFpr", "recall", 100),
    ("Unit-wise ROC Curve", "Weighted Recall", "roc", "fpr", "weightedRecall", 100),
    ("Unit-wise ROC Curve", "Unit-wise Recall", "roc", "fpr", "recall", 100),
]


def _panel_svg(title, ylabel, series, xkey, ykey, lk, xscale):
    """One chart: every series' (x, y) polyline, shared axes scaled to the data."""
    W, H, L, T = 560, 340, 60, 30
    pts_all = []
    for _, perf in series:
        pts = []
        for po in perf.get(lk, []):
            x, y = _num(po.get(xkey, math.nan)), _num(po.get(ykey, math.nan))
            if x is None or y is None:
                continue
            ys = y if ykey == "scoreCount" else y * 100
            pts.append((x * xscale, ys))
        pts_all.append(pts)
    xs = [p[0] for ps in pts_all for p in ps] or [0.0, 1.0]
    ys = [p[1] for ps in pts_all for p in ps] or [0.0, 1.0]
    x0, x1 = min(xs), max(xs)
    y0, y1 = min(0.0, min(ys)), max(ys)
    x1 = x1 if x1 > x0 else x0 + 1
    y1 = y1 if y1 > y0 else y0 + 1
    pw, ph = W - L - 20, H - T - 40

    def px(x):
        return L + (x - x0) / (x1 - x0) * pw

    def py(y):
        return T + ph - (y - y0) / (y1 - y0) * ph
    out = [f'<svg width="{W}" height="{H}" xmlns="http://www.w3.org/2000/svg">',
           f'<text x="{L}" y="18" font-size="14">{html.escape(title)} &#8212; {html.escape(ylabel)}</text>',
           f'<rect x="{L}" y="{T}" width="{pw}" height="{ph}" fill="none" stroke="#999"/>']
    for k in range(5):
        gx, gy = x0 + (x1 - x0) * k / 4, y0 + (y1 - y0) * k / 4
        out.append(f'<text x="{px(gx):.1f}" y="{T + ph + 14}" font-size="10" text-anchor="middle">{gx:.4g}</text>')
        out.append(f'<text x="{L - 4}" y="{py(gy) + 3:.1f}" font-size="10" text-anchor="end">{gy:.4g}</text>')
    for j, pts in enumerate(pts_all):
        if not pts:
            continue
        path = " ".join(f"{px(x):.1f},{py(y):.1f}" for x, y in pts)
        out.append(f'<polyline fill="none" stroke="{COLORS[j % len(COLORS)]}" stroke-width="2" points="{path}"/>')
    for j, (name, _) in enumerate(series):
        out.append(f'<text x="{L + 8}" y="{T + 14 + 13 * j}" font-size="11" fill="{COLORS[j % len(COLORS)]}">'
                   f'{html.escape(name)}</text>')
    out.append("</svg>")
    return "".join(out)


def _page(path, heading, panels, series):
    data = []
    for j, (name, perf) in enumerate(series):
        data.append(f"  var data_{j} = " + json.dumps(
            {k: [{f: _num(po.get(f, math.nan)) for f in ("actionRate", "weightedActionRate", "recall",
                                                           "weightedRecall", "precision", "weightedPrecision",
                                                           "fpr", "weightedFpr", "binLowestScore", "scoreCount")}
                 for po in perf.get(k, [])]
             for k in ("gains", "weightedGains", "pr", "weightedPr", "roc", "weightedRoc", "modelScoreList")}) + ";")
    body = "".join(f"<div>{_panel_svg(t, yl, series, xk, yk, lk, xs)}</div>" for t, yl, lk, xk, yk, xs in panels)
    auc = "".join(f"<li>{html.escape(n)}: AUC(ROC) {java_df(p.get('areaUnderRoc', math.nan))}, "
                  f"weighted AUC(ROC) {java_df(p.get('weightedAreaUnderRoc', math.nan))}, "
                  f"AUC(PR) {java_df(p.get('areaUnderPr', math.nan))}</li>" for n, p in series)
    with open(path, "w") as f:
        f.write(f"<!DOCTYPE html>\n<html><head><meta charset=\"utf-8\"><title>{html.escape(heading)}</title></head>"
                f"<body><h2>{html.escape(heading)}</h2><ul>{auc}</ul>\n{body}\n<script>\n"
                + "\n".join(data) + "\n</script></body></html>\n")


def write_eval_reports(eval_dir: str, ev_name: str, model_name: str, series: list, has_weight: bool) -> list:
    """Write every report file of one eval set; ``series`` = [(name, performance dict)] with the
    model first.  Returns the written paths."""
    os.makedirs(eval_dir, exist_ok=True)
    title = f"{model_name}::{ev_name}"
    written = []
    p = os.path.join(eval_dir, f"{ev_name}_gainchart.html")
    _page(p, title + " gain chart", GAIN_PANELS, series)
    written.append(p)
    p = os.path.join(eval_dir, f"{ev_name}_prroc.html")
    _page(p, title + " PR / ROC", PRROC_PANELS, series)
    written.append(p)
    for name, perf in series:
        files = [("unit_wise_gainchart", "gains"), ("unit_wise_pr", "pr"), ("unit_wise_roc", "roc")]
        if has_weight:
            files += [("weighted_gainchart", "weightedGains"), ("weighted_pr", "weightedPr"),
                      ("weighted_roc", "weightedRoc")]
        files.append(("modelscore_gainchart", "modelScoreList"))
        for suffix, key in files:
            p = os.path.join(eval_dir, f"{name}_{suffix}.csv")
            write_perf_csv(p, perf.get(key, []))
            written.append(p)
    return written
