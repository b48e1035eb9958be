"""``export -t pmml|columnstats|woemapping|bagging|baggingpmml|corr|woe`` (B10).

``ExportModelProcessor.run`` (J/core/processor/ExportModelProcessor.java:109, types :76-88).
"""
from __future__ import annotations

import csv
import json
import os
import shutil

import numpy as np

from ..formats import nn_format, pmml, tree_format
from ..models import lr as lrmod
from ..scoring.model_runner import list_model_files
from ..utils.log import get_logger
from .base import ModelSet

_log = get_logger("steps.export")

TYPES = ("pmml", "columnstats", "woemapping", "bagging", "baggingpmml", "corr", "woe")


def _target(ms):
    t = [c for c in ms.ccs if c.is_target()]
    return t[0].name if t else "target"


def export_pmml(ms, concise=False):
    from ..config.column_config import model_input_columns
    cols = model_input_columns(ms.ccs, ms.mc.is_binary())
    out_dir = ms.pf.p("pmmls")
    os.makedirs(out_dir, exist_ok=True)
    cutoff = float(ms.mc.normalize.get("stdDevCutOff", 6.0))
    paths = []
    for p in list_model_files(ms.pf.models_dir, ms.mc.algorithm):
        name = os.path.splitext(os.path.basename(p))[0]
        if p.endswith(".nn"):
            net = nn_format.read_encog(p) if not nn_format.is_binary_nn(p) else nn_format.read_binary_nn(p)["networks"][0]
            doc = pmml.nn_pmml(net, cols, _target(ms), ms.mc.norm_type, cutoff, name)
        elif p.endswith(".lr"):
            doc = pmml.lr_pmml(lrmod.read_lr(p), cols, _target(ms), ms.mc.norm_type, cutoff, name)
        elif p.endswith((".gbt", ".rf")):
            doc = pmml.tree_pmml(tree_format.read_tree_model(p), cols, _target(ms), name)
        else:
            continue
        out = os.path.join(out_dir, f"{ms.mc.name}{name[len('model'):]}.pmml")
        pmml.write_pmml(doc, out)
        paths.append(out)
    _log.info("exported %d PMML files to %s", len(paths), out_dir)
    return paths


def export_bagging_pmml(ms):
    """``export -t baggingpmml`` (ExportModelProcessor :173-187): every NN bag in ONE PMML
    (``pmmls/<modelSetName>.pmml``, an averaging MiningModel); NN only, as in the reference."""
    if str(ms.mc.algorithm).upper() != "NN":
        _log.warning("Currently one bagging pmml model is only supported in NN algorithm.")
        return None
    from ..config.column_config import model_input_columns
    cols = model_input_columns(ms.ccs, ms.mc.is_binary())
    nets = []
    for p in list_model_files(ms.pf.models_dir, "NN"):
        if p.endswith(".nn"):
            nets.append(nn_format.read_encog(p) if not nn_format.is_binary_nn(p)
                        else nn_format.read_binary_nn(p)["networks"][0])
    if not nets:
        raise FileNotFoundError("no NN models to export")
    cutoff = float(ms.mc.normalize.get("stdDevCutOff", 6.0))
    doc = pmml.nn_bagging_pmml(nets, cols, _target(ms), ms.mc.norm_type, cutoff, ms.mc.name)
    out = ms.pf.p("pmmls", f"{ms.mc.name}.pmml")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    pmml.write_pmml(doc, out)
    _log.info("one bagging PMML (%d networks) -> %s", len(nets), out)
    return out


def export_bagging(ms):
    """Merge all NN bags into one binary ``.nn`` (BinaryNNSerializer with N networks)."""
    from ..config.column_config import model_input_columns
    from .train import nn_column_stats
    cols = model_input_columns(ms.ccs, ms.mc.is_binary())
    nets = []
    for p in list_model_files(ms.pf.models_dir, "NN"):
        if p.endswith(".nn"):
            nets.append(nn_format.read_encog(p) if not nn_format.is_binary_nn(p)
                        else nn_format.read_binary_nn(p)["networks"][0])
    if not nets:
        raise FileNotFoundError("no NN models to merge")
    out = ms.pf.p("onebaggingmodel", f"{ms.mc.name}.b.nn")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    nn_format.write_binary_nn(out, ms.mc.norm_type, nn_column_stats(ms.mc, cols),
                              {c.num: i for i, c in enumerate(cols)}, nets)
    return out


def export_column_stats(ms):
    path = ms.pf.column_stats_csv
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["columnNum", "columnName", "columnType", "columnFlag", "finalSelect", "ks", "iv", "woe",
                    "mean", "stdDev", "min", "max", "median", "totalCount", "missingCount", "missingPercentage",
                    "distinctCount", "skewness", "kurtosis", "psi", "numBins"])
        for c in ms.ccs:
            s = c.stats
            w.writerow([c.num, c.name, c.type, c.flag, c.final_select, s.get("ks"), s.get("iv"), s.get("woe"),
                        s.get("mean"), s.get("stdDev"), s.get("min"), s.get("max"), s.get("median"),
                        s.get("totalCount"), s.get("missingCount"), s.get("missingPercentage"),
                        s.get("distinctCount"), s.get("skewness"), s.get("kurtosis"), s.get("psi"),
                        c.n_bins() - 1])
    return path


def _java_double(v) -> str:
    """Java Double.toString-style text for the exported mapping files."""
    v = float(v)
    if v != v:
        return "NaN"
    if v in (float("inf"), float("-inf")):
        return "Infinity" if v > 0 else "-Infinity"
    return repr(v)


def export_woe_mapping(ms, request_vars=None, expected_bins: int = 0, iv_keep_ratio: float = 1.0,
                       min_inst_cnt: float = 0):
    """``export -t woemapping`` (ExportModelProcessor.java:190-206, rebinAndExportWoeMapping
    :263-304, generate*WoeMapping :306-350): every requested column is re-binned with the
    IV-keeping dynamic merge and written as a SQL ``case`` expression into ``woemapping.txt``."""
    from ..algos import stats as S
    from ..algos.dynamic_binning import dynamic_rebin
    texts = []
    for c in ms.ccs:
        if request_vars and c.name not in request_vars:
            continue
        cat = c.is_categorical()
        keys = (c.bin_category if cat else c.bin_boundary) or []
        if not keys or c.bin_count_pos is None:
            continue
        bins, miss = dynamic_rebin(cat, keys, c.bin_count_pos, c.bin_count_neg, c.bin_weighted_pos,
                                   c.bin_weighted_neg, expected_bins, iv_keep_ratio, min_inst_cnt)
        neg = np.array([b.neg for b in bins] + [miss.neg], float)
        pos = np.array([b.pos for b in bins] + [miss.pos], float)
        m = S.column_metrics(neg, pos)
        if m is None:
            continue
        woe = m[3]
        name = c.name
        lines = ["( case "]
        if cat:
            for i, b in enumerate(bins):
                vals = []
                for v in b.values:
                    vals += [f"'{x}'" for x in str(v).split("@^")]
                lines.append(f"\twhen {name} in ({','.join(vals)}) then {_java_double(woe[i])}")
            lines.append(f"\telse {_java_double(woe[-1])}")
        else:
            lines.append(f"\twhen {name} = . then {_java_double(woe[-1])}")
            for i, b in enumerate(bins):
                right = bins[i + 1].left if i + 1 < len(bins) else float("inf")
                cond = ""
                if b.left not in (float("inf"), float("-inf")):
                    cond += f"{_java_double(b.left)} <= "
                cond += name
                if right not in (float("inf"), float("-inf")):
                    cond += f" < {_java_double(right)}"
                lines.append(f"\twhen ({cond}) then {_java_double(woe[i])}")
        lines.append(f"  end ) as {name}_{len(bins)}")
        texts.append("\n".join(lines))
        _log.info("%s: %d bins, IV %.6f, KS %.6f", name, len(bins), m[1], m[0])
    path = ms.pf.p("woemapping.txt")
    with open(path, "w") as f:
        f.write(",\n".join(texts))
    return path


def export_var_woe(ms):
    """``export -t woe`` (ExportModelProcessor.java:207-220, generateWoeInfos :238-261):
    per column with more than one bin, its bin ranges / categories with their WOE, into
    ``varwoe_info.txt`` (blank line between columns)."""
    out = []
    for c in ms.ccs:
        woe = c.bin_count_woe
        if not woe:
            continue
        bb, cats = c.bin_boundary, c.bin_category
        if c.is_categorical():
            if not cats:
                continue
            out.append(c.name)
            out += [f"{cats[i]}\t{_java_double(woe[i])}" for i in range(len(cats))]
        else:
            if not bb or len(bb) <= 1:
                continue
            out.append(c.name)
            for i in range(len(bb)):
                if i == 0:
                    out.append(f"(-\u221e,{_java_double(bb[1])}]\t{_java_double(woe[i])}")
                elif i == len(bb) - 1:
                    out.append(f"({_java_double(bb[i])},+\u221e]\t{_java_double(woe[i])}")
                else:
                    out.append(f"({_java_double(bb[i])},{_java_double(bb[i + 1])}]\t{_java_double(woe[i])}")
        out.append(f"MISSING\t{_java_double(woe[-1])}")
        out.append("")
    path = ms.pf.p("varwoe_info.txt")
    with open(path, "w", encoding="utf-8") as f:
        f.write("\n".join(out) + ("\n" if out else ""))
    return path


def export_corr(ms):
    """``export -t corr`` (exportVariableCorr :481-524): every (good candidate or target, other
    non-meta non-target) pair of ``correlation.csv`` as ``left,right,corr,leftMetric,rightMetric``
    (names ordered, metric = varSelect.postCorrelationMetric IV|KS), sorted by correlation
    descending, into ``tmp/vars_corr.csv``."""
    from ..config.column_config import has_candidates
    metric = str(ms.mc.varSelect.get("postCorrelationMetric") or "IV").upper()
    hc = has_candidates(ms.ccs)
    binary = ms.mc.is_binary()

    def mval(c):
        v = c.stats.get("ks" if metric == "KS" else "iv")
        return float("nan") if v is None else float(v)
    pairs = {}
    with open(ms.pf.correlation_csv) as f:
        f.readline()
        f.readline()
        for line in f:
            parts = line.rstrip("\n").split(",")
            if len(parts) != len(ms.ccs) + 2:
                continue
            src = ms.ccs[int(parts[0])]
            if not (src.is_target() or src.is_good_candidate(hc, binary)):
                continue
            for i, v in enumerate(parts[2:]):
                dst = ms.ccs[i]
                if i == src.num or dst.is_target() or dst.is_meta():
                    continue
                a, b = (src, dst) if src.name < dst.name else (dst, src)
                pairs[(a.name, b.name)] = (float(v), mval(a), mval(b))
    rows = sorted(pairs.items(), key=lambda kv: -kv[1][0])
    path = ms.pf.ensure(ms.pf.p("tmp", "vars_corr.csv"))
    with open(path, "w") as f:
        for (a, b), (v, ma, mb) in rows:
            f.write(f"{a},{b},{_java_double(v)},{_java_double(ma)},{_java_double(mb)}\n")
    return path


def run_export(root: str = ".", etype: str = "pmml", concise: bool = False, request_vars=None,
               expected_bins: int = 0, iv_keep_ratio: float = 1.0, min_inst_cnt: float = 0) -> int:
    ms = ModelSet(root)
    t = (etype or "pmml").lower()
    if t not in TYPES:
        raise ValueError(f"unsupported export type {etype}; one of {TYPES}")
    if t == "pmml":
        export_pmml(ms, concise)
    elif t == "baggingpmml":
        export_bagging_pmml(ms)
    elif t == "bagging":
        _log.info("merged bagging model -> %s", export_bagging(ms))
    elif t == "columnstats":
        _log.info("column stats -> %s", export_column_stats(ms))
    elif t == "woemapping":
        _log.info("woe mapping -> %s", export_woe_mapping(ms, request_vars, expected_bins, iv_keep_ratio,
                                                          min_inst_cnt))
    elif t == "woe":
        _log.info("variable woe -> %s", export_var_woe(ms))
    elif t == "corr":
        if not os.path.exists(ms.pf.correlation_csv):
            _log.warning("The correlation file doesn't exist. Please make sure you have ran `shifu stats -c`.")
            return 2
        _log.info("correlations -> %s", export_corr(ms))
    return 0
