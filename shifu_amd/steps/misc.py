"""Small verbs: ``save/switch/show/list`` (B12), ``encode`` (B13), ``test -filter`` (B14),
``convert -tozipb/-totreeb`` + ``analysis -fi`` (B15).

* ManageModelProcessor (J/core/processor/ManageModelProcessor.java:49-75): branches live under
  ``backup_models/<name>`` (ModelConfig/ColumnConfig/models); ``.HEAD`` names the current one.
* ModelDataEncodeProcessor (J/core/processor/ModelDataEncodeProcessor.java:77): encode each row of
  the training set (or an eval set) as the L/R leaf paths of a GBT/RF model, appended to the raw
  columns; output ``tmp/encodedTrainData`` (or ``tmp/encodedEval<name>``) as ``|`` text + header.
* ShifuTestProcessor (J/core/processor/ShifuTestProcessor.java:45-80): evaluate the filter
  expression of the training / eval data sets on the first N records and report kept counts.
* convert: binary ``.gbt`` <-> zip "readable spec" (``model.ini`` + one JSON per tree);
  analysis -fi: tree feature importance table.
"""
from __future__ import annotations

import io
import json
import os
import shutil
import zipfile

import numpy as np

from ..data.expr import Evaluator
from ..data.reader import first_line_is_header, read_header, read_table
from ..formats import tree_format
from ..scoring.tree_ensemble import TreeScorer
from ..utils.log import get_logger
from .base import ModelSet

_log = get_logger("steps.misc")
BACKUP = "backup_models"


# ---- save / switch / show / list ---------------------------------------------------------------------
def current_branch(root):
    p = os.path.join(root, ".HEAD")
    return open(p).read().strip() if os.path.exists(p) else "master"


def save_branch(root, name=None):
    name = name or current_branch(root)
    dst = os.path.join(root, BACKUP, name)
    os.makedirs(os.path.join(dst, "models"), exist_ok=True)
    for fn in ("ModelConfig.json", "ColumnConfig.json"):
        if os.path.exists(os.path.join(root, fn)):
            shutil.copyfile(os.path.join(root, fn), os.path.join(dst, fn))
    md = os.path.join(root, "models")
    if os.path.isdir(md):
        for fn in os.listdir(md):
            if fn.startswith("model") and os.path.isfile(os.path.join(md, fn)):
                shutil.copyfile(os.path.join(md, fn), os.path.join(dst, "models", fn))
    return dst


def switch_branch(root, name):
    save_branch(root, current_branch(root))
    src = os.path.join(root, BACKUP, name)
    if os.path.isdir(src):
        for fn in ("ModelConfig.json", "ColumnConfig.json"):
            if os.path.exists(os.path.join(src, fn)):
                shutil.copyfile(os.path.join(src, fn), os.path.join(root, fn))
        md = os.path.join(src, "models")
        if os.path.isdir(md):
            os.makedirs(os.path.join(root, "models"), exist_ok=True)
            for fn in os.listdir(md):
                shutil.copyfile(os.path.join(md, fn), os.path.join(root, "models", fn))
    with open(os.path.join(root, ".HEAD"), "w") as f:
        f.write(name)


def list_branches(root):
    b = os.path.join(root, BACKUP)
    return sorted(d for d in os.listdir(b) if os.path.isdir(os.path.join(b, d))) if os.path.isdir(b) else []


def run_manage(root=".", action="show", name=None) -> int:
    if action == "save":
        print(save_branch(root, name))
    elif action == "switch":
        switch_branch(root, name)
    elif action == "list":
        for b in list_branches(root):
            print(b)
    else:
        print(f"Current work model name is {current_branch(root)}")
    return 0


# ---- encode ------------------------------------------------------------------------------------------
def run_encode(root=".", target: str | None = None, ref_model: str | None = None, device=None) -> int:
    ms = ModelSet(root)
    mc = ms.mc
    mdir = ms.pf.models_dir if not ref_model else os.path.join(os.path.dirname(ms.root), ref_model, "models")
    paths = [os.path.join(mdir, f) for f in sorted(os.listdir(mdir)) if f.endswith((".gbt", ".rf"))]
    if not paths:
        raise FileNotFoundError(f"no GBT/RF model under {mdir}")
    scorer = TreeScorer(tree_format.read_tree_model(paths[0]), device or "cpu")
    depth = int((mc.train.get("params") or {}).get("MaxDepth", 0) or 0) or None
    confs = [("train", mc.dataSet)] if not target else [(e.get("name"), e.dataSet) for e in mc.evals
                                                         if target in ("*", e.get("name"))]
    for name, ds in confs:
        data_path = mc.resolve(ds.get("dataPath"))
        delim = ds.get("dataDelimiter") or "|"
        hp = ds.get("headerPath")
        header = read_header(mc.resolve(hp) if hp else None, ds.get("headerDelimiter") or "|", data_path, delim)
        t = read_table(data_path, header, delim, strings=header, missing=mc.missing_values,
                       skip_header_line=(not hp) and first_line_is_header(data_path, header, delim))
        m = scorer.model
        num = {m.names[c] for c in m.names if c not in m.categories}
        tab = read_table(data_path, header, delim, numeric=[h for h in header if h in num],
                         strings=[h for h in header if h not in num], missing=mc.missing_values,
                         skip_header_line=(not hp) and first_line_is_header(data_path, header, delim))
        codes = scorer.encode(tab, depth)
        out = ms.pf.encoded_train_data if name == "train" else ms.pf.encoded_eval_data(name)
        os.makedirs(out, exist_ok=True)
        enc_names = [f"tree_vars_{i}" for i in range(codes.shape[1])]
        raw = [t[h].strings() for h in header]
        with open(os.path.join(out, "part-00000"), "w") as f:
            for i in range(t.n):
                f.write("|".join([r[i] for r in raw] + list(codes[i])) + "\n")
        with open(os.path.join(out, ".pig_header"), "w") as f:
            f.write("|".join(list(header) + enc_names) + "\n")
        _log.info("encode %s: %d rows, %d tree features -> %s", name, t.n, len(enc_names), out)
    return 0


# ---- test -filter -----------------------------------------------------------------------------------
def run_filter_test(root=".", target: str | None = None, n: int = 100) -> int:
    ms = ModelSet(root)
    mc = ms.mc
    confs = []
    if not target:
        confs = [("train", mc.dataSet)]
    elif target == "*":
        confs = [("train", mc.dataSet)] + [(e.get("name"), e.dataSet) for e in mc.evals]
    else:
        for nm in target.split(","):
            es = [e for e in mc.evals if e.get("name") == nm.strip()]
            if not es:
                _log.error("Eval - %s doesn't exist!", nm)
                return 1
            confs.append((nm.strip(), es[0].dataSet))
    status = 0
    for name, ds in confs:
        expr = ds.get("filterExpressions") or ""
        data_path = mc.resolve(ds.get("dataPath"))
        delim = ds.get("dataDelimiter") or "|"
        hp = ds.get("headerPath")
        header = read_header(mc.resolve(hp) if hp else None, ds.get("headerDelimiter") or "|", data_path, delim)
        t = read_table(data_path, header, delim, strings=header, missing=mc.missing_values, max_rows=n,
                       skip_header_line=(not hp) and first_line_is_header(data_path, header, delim))
        if not expr.strip():
            print(f"[{name}] no filter expression; {t.n} records")
            continue
        try:
            ev = Evaluator(expr)
            # re-read referenced columns as numeric where they parse as numbers
            m = ev.mask(t)
            print(f"[{name}] filter `{expr}`: {int(m.sum())} of {t.n} records kept")
        except Exception as e:     # noqa: BLE001
            print(f"[{name}] filter `{expr}` failed: {e}")
            status = 1
    return status


# ---- convert / analysis -------------------------------------------------------------------------------
def _node_json(nd):
    if nd is None:
        return None
    d = {"id": nd.id, "gain": nd.gain, "wgtCnt": nd.wgt_cnt, "predict": nd.predict, "classValue": nd.class_value}
    if nd.split is not None:
        s = nd.split
        d["split"] = {"column": s.column, "type": "CONTINUOUS" if s.ftype == 1 else "CATEGORICAL",
                      "threshold": s.threshold, "isLeft": s.is_left,
                      "categories": sorted(s.categories) if s.categories else None}
        d["left"] = _node_json(nd.left)
        d["right"] = _node_json(nd.right)
    return d


def _node_from_json(d):
    if d is None:
        return None
    nd = tree_format.Node(d["id"], d.get("gain", 0.0), d.get("wgtCnt", 0.0), None, d.get("predict"),
                          d.get("classValue", 0))
    s = d.get("split")
    if s:
        nd.split = tree_format.Split(s["column"], 1 if s["type"] == "CONTINUOUS" else 2, s.get("threshold", 0.0),
                                     s.get("isLeft", True), set(s["categories"]) if s.get("categories") else None)
        nd.left, nd.right = _node_from_json(d.get("left")), _node_from_json(d.get("right"))
    return nd


def gbt_to_zip(src: str, dst: str):
    m = tree_format.read_tree_model(src)
    with zipfile.ZipFile(dst, "w", zipfile.ZIP_DEFLATED) as z:
        ini = {"version": m.version, "algorithm": m.algorithm, "loss": m.loss,
               "isClassification": m.is_classification, "isOneVsAll": m.is_one_vs_all,
               "inputCount": m.input_count, "numericalMeans": {str(k): v for k, v in m.numerical_means.items()},
               "columnNames": {str(k): v for k, v in m.names.items()},
               "categories": {str(k): v for k, v in m.categories.items()},
               "columnMapping": {str(k): v for k, v in m.column_mapping.items()}, "bags": len(m.bags)}
        z.writestr("model.ini", json.dumps(ini, indent=1))
        for b, bag in enumerate(m.bags):
            for t in bag:
                z.writestr(f"trees/bag{b}/tree{t.tree_id}.json",
                           json.dumps({"treeId": t.tree_id, "learningRate": t.learning_rate,
                                       "rootWgtCnt": t.root_wgt_cnt, "features": t.features,
                                       "nodeNum": t.node_num, "root": _node_json(t.root)}))


def zip_to_gbt(src: str, dst: str):
    with zipfile.ZipFile(src) as z:
        ini = json.loads(z.read("model.ini"))
        bags = [[] for _ in range(ini["bags"])]
        for nm in sorted(z.namelist()):
            if nm.startswith("trees/"):
                b = int(nm.split("/")[1][3:])
                d = json.loads(z.read(nm))
                bags[b].append(tree_format.TreeRecord(d["treeId"], d["nodeNum"], _node_from_json(d["root"]),
                                                      d["learningRate"], d.get("rootWgtCnt", 0.0),
                                                      d.get("features", [])))
        for bag in bags:
            bag.sort(key=lambda t: t.tree_id)
    ik = lambda dct: {int(k): v for k, v in dct.items()}   # noqa: E731
    m = tree_format.TreeModelFile(ini["algorithm"], ini["loss"], ini["isClassification"], ini["isOneVsAll"],
                                  ini["inputCount"], ik(ini["numericalMeans"]), ik(ini["columnNames"]),
                                  ik(ini["categories"]), ik(ini["columnMapping"]), bags)
    tree_format.write_tree_model(dst, m)


def run_convert(mode: str, src: str, dst: str) -> int:
    if mode in ("tozipb", "-tozipb"):
        gbt_to_zip(src, dst)
    elif mode in ("totreeb", "-totreeb"):
        zip_to_gbt(src, dst)
    else:
        raise ValueError("convert mode must be -tozipb or -totreeb")
    return 0


def run_analysis_fi(model_path: str, out: str | None = None) -> int:
    m = tree_format.read_tree_model(model_path)
    fi = tree_format.feature_importance(m)
    lines = [f"{k}\t{m.names.get(k, k)}\t{v:.6f}" for k, v in fi.items()]
    text = "\n".join(lines) + "\n"
    if out:
        with open(out, "w") as f:
            f.write(text)
    print(text, end="")
    return 0
