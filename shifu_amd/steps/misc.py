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
from ..formats.javaio import JavaIn, JavaOut
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
    import torch
    from ..data.join import stream_join
    from ..data.purifier import plan_dataset
    from ..data.reader import column_kinds
    from ..parallel import dist
    dev = device or ("cuda" if torch.cuda.is_available() and not os.environ.get("SHIFU_FORCE_CPU") else "cpu")
    scorer = TreeScorer(tree_format.read_tree_model(paths[0]), dev)
    m = scorer.model
    depth = int((mc.train.get("params") or {}).get("MaxDepth", 0) or 0) or None
    confs = [("train", mc.dataSet)] if not target else [(e.get("name"), e.dataSet) for e in mc.evals
                                                         if target in ("*", e.get("name"))]
    ntrees = sum(len(b) for b in m.bags)
    enc_names = [f"tree_vars_{i}" for i in range(ntrees)]
    info = dist.info()
    for name, ds in confs:
        # the trees' inputs only: numeric columns parsed as numbers, categorical ones as strings
        num = [m.names[c] for c in m.names if c not in m.categories]
        cat = [m.names[c] for c in m.names if c in m.categories]
        plan = plan_dataset(mc, ds, num, cat)
        kinds = column_kinds(plan.header, plan.nums, plan.strs)
        out = ms.pf.encoded_train_data if name == "train" else ms.pf.encoded_eval_data(name)
        rows = stream_join(plan, out, enc_names, kinds, lambda t, n: scorer.encode_fields(t, depth),
                           info.rank, info.world_size)
        _log.info("encode %s: %d rows (rank %d), %d tree features -> %s", name, rows, info.rank, len(enc_names), out)
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
def gbt_to_zip(src: str, dst: str):
    """Binary ``.gbt``/``.rf`` -> readable zip spec in the reference layout
    (IndependentTreeModelUtils.convertBinaryToZipSpec, J/util/IndependentTreeModelUtils.java:38-70):
    ``model.ini`` = the IndependentTreeModel bean as JSON with ``trees: null``, ``trees`` = int
    #bags, per bag int #trees + ``TreeNode.write`` records (Java big-endian)."""
    m = tree_format.read_tree_model(src)
    ini = {
        "numNameMapping": {str(k): v for k, v in m.names.items()},
        "categoricalColumnNameNames": {str(k): list(v) for k, v in m.categories.items()},
        "columnCategoryIndexMapping": {str(k): {c: j for j, c in enumerate(v)} for k, v in m.categories.items()},
        "columnNumIndexMapping": {str(k): v for k, v in m.column_mapping.items()},
        "trees": None,
        "weights": [[t.learning_rate for t in bag] for bag in m.bags],
        "lossStr": m.loss,
        "algorithm": m.algorithm,
        "inputNode": m.input_count,
        "numericalMeanMapping": {str(k): v for k, v in m.numerical_means.items()},
        "gbtScoreConvertStrategy": "RAW",
        "gbdt": m.algorithm.upper() == "GBT",
        "classification": m.is_classification,
        "convertToProb": False,
    }
    o = JavaOut()
    tree_format.write_bags(o, m.bags)
    with zipfile.ZipFile(dst, "w", zipfile.ZIP_DEFLATED) as z:
        z.writestr("model.ini", json.dumps(ini, indent=2))
        z.writestr("trees", o.bytes())


def zip_to_gbt(src: str, dst: str):
    """Readable zip spec -> binary ``.gbt`` (convertZipSpecToBinary, :74-125)."""
    with zipfile.ZipFile(src) as z:
        ini = json.loads(z.read("model.ini"))
        bags = tree_format.read_bags(JavaIn(z.read("trees")))
    if not bags or not any(bags):
        raise ValueError(f"{src}: no trees in the zip spec")
    ik = lambda dct: {int(k): v for k, v in (dct or {}).items()}   # noqa: E731
    m = tree_format.TreeModelFile(ini["algorithm"], ini.get("lossStr", "squared"), bool(ini.get("classification")),
                                  bool(ini.get("oneVsAll", False)), int(ini["inputNode"]),
                                  ik(ini.get("numericalMeanMapping")), ik(ini.get("numNameMapping")),
                                  ik(ini.get("categoricalColumnNameNames")), ik(ini.get("columnNumIndexMapping")), bags)
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
