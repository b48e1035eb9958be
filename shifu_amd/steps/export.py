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


def export_woe_mapping(ms, weighted=False):
    """Per selected column the bin -> WOE mapping (numeric intervals / category groups)."""
    out = {}
    for c in ms.ccs:
        if not (c.final_select or c.is_force_select()) or c.is_target():
            continue
        woe = c.bin_weighted_woe if weighted else c.bin_count_woe
        if woe is None:
            continue
        if c.is_categorical():
            m = {str(cat): woe[i] for i, cat in enumerate(c.bin_category or [])}
        else:
            bb = list(c.bin_boundary or [])
            m = {f"[{bb[i]}, {bb[i + 1] if i + 1 < len(bb) else 'Infinity'})": woe[i] for i in range(len(bb))}
        m["<missing>"] = woe[-1]
        out[c.name] = m
    path = ms.pf.p("woemapping.json" if not weighted else "woemapping.weighted.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, default=float)
    return path


def run_export(root: str = ".", etype: str = "pmml", concise: bool = False) -> int:
    ms = ModelSet(root)
    t = (etype or "pmml").lower()
    if t not in TYPES:
        raise ValueError(f"unsupported export type {etype}; one of {TYPES}")
    if t in ("pmml", "baggingpmml"):
        export_pmml(ms, concise)
    elif t == "bagging":
        _log.info("merged bagging model -> %s", export_bagging(ms))
    elif t == "columnstats":
        _log.info("column stats -> %s", export_column_stats(ms))
    elif t in ("woemapping", "woe"):
        _log.info("woe mapping -> %s", export_woe_mapping(ms, weighted=False))
    elif t == "corr":
        if not os.path.exists(ms.pf.correlation_csv):
            raise FileNotFoundError("run `stats -c` first")
        dst = ms.pf.p("export.correlation.csv")
        shutil.copyfile(ms.pf.correlation_csv, dst)
        _log.info("correlation -> %s", dst)
    return 0
