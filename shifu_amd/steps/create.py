"""``new`` (B2) and ``init`` (B3) steps.

* new: ``CreateModelProcessor.run`` (J/core/processor/CreateModelProcessor.java:71-108) — model-set
  folder, default ModelConfig.json for the algorithm, ``.HEAD``, empty column-name files.
* init: ``InitModelProcessor.initColumnConfigList`` (J/core/processor/InitModelProcessor.java:424-502)
  — one ColumnConfig per header field (or per index without a header), flags from the column
  files; optional auto-type (:289-376 + :143-254): distinct count (exact, on the parsed
  dictionary instead of HyperLogLog), valid-number ratio > autoTypeThreshold% -> numeric,
  0/1 columns -> numeric.  (The reference's ``isDoubleFrequentVariable`` only rejects blank
  sampled items, which makes its threshold branch a no-op; we implement the documented
  ratio rule.)
"""
from __future__ import annotations

import os

import numpy as np

from ..config.column_config import ColumnConfig, save_column_configs
from ..config.model_config import create_init_model_config
from ..config.updater import update_column_flags
from ..data.reader import first_line_is_header, list_data_files, read_header, read_table
from ..utils.log import get_logger
from .base import ModelSet

_log = get_logger("steps.init")

COLUMN_FILES = ("meta.column.names", "categorical.column.names", "forceselect.column.names",
                "forceremove.column.names", "Eval1.meta.column.names", "Eval1score.meta.column.names")


def create_model_set(name: str, alg: str = "NN", description: str | None = None, parent: str = ".") -> str:
    root = os.path.abspath(os.path.join(parent, name))
    if os.path.exists(os.path.join(root, "ModelConfig.json")):
        raise FileExistsError(f"model set {root} already exists")
    os.makedirs(os.path.join(root, "columns"), exist_ok=True)
    mc = create_init_model_config(name, alg, description)
    mc.save(os.path.join(root, "ModelConfig.json"))
    for fn in COLUMN_FILES:
        p = os.path.join(root, "columns", fn)
        if not os.path.exists(p):
            open(p, "w").close()
    with open(os.path.join(root, ".HEAD"), "w") as f:
        f.write("master")
    _log.info("created model set %s (%s)", root, alg)
    return root


def norm_column_name(n: str) -> str:
    """``CommonUtils.normColumnName``: trim, and replace characters Pig cannot take."""
    n = (n or "").strip()
    for ch in ("-", "/", " ", ".", ":"):
        n = n.replace(ch, "_")
    return n


def init_column_configs(ms: ModelSet, auto_type: bool | None = None):
    mc = ms.mc
    ds = mc.dataSet
    data_path = mc.resolve(ds.get("dataPath"))
    delim = ds.get("dataDelimiter") or "|"
    hpath = ds.get("headerPath")
    target = ds.get("targetColumnName")
    if hpath:
        fields = read_header(mc.resolve(hpath), ds.get("headerDelimiter") or "|")
        schema = True
    else:
        fields = read_header(None, ds.get("headerDelimiter") or delim, data_path, delim)
        schema = target is not None and target in "".join(fields)
        if not schema:
            fields = [str(i) for i in range(len(fields))]
    first = list_data_files(data_path)
    if hpath and first:
        with open(first[0], "rb") as f:
            line = f.readline().decode("utf-8", "replace").rstrip("\r\n")
        if line and len(line.split(delim)) != len(fields):
            raise ValueError(f"header length {len(fields)} != data length {len(line.split(delim))}")
    ccs = []
    for i, fld in enumerate(fields):
        c = ColumnConfig()
        c.num = i
        c.name = norm_column_name(fld) if schema else str(i)
        ccs.append(c)
    segs = mc.segment_filter_expressions()
    base = list(ccs)
    for k in range(1, len(segs) + 1):          # segment copies: num = k * size + i, name "<col>_<k>"
        for c0 in base:
            c = ColumnConfig()
            c.num = k * len(base) + c0.num
            c.name = f"{c0.name}_{k}"
            ccs.append(c)
    update_column_flags(mc, ccs, "INIT")
    if not any(c.is_target() for c in ccs):
        raise ValueError(f"target column {target!r} not found in header")
    ms.ccs = ccs
    if auto_type if auto_type is not None else bool(ds.get("autoType", False)):
        auto_type_columns(ms, fields)
    return ccs


def auto_type_columns(ms: ModelSet, header=None, max_rows: int | None = None):
    mc = ms.mc
    ds = mc.dataSet
    data_path = mc.resolve(ds.get("dataPath"))
    delim = ds.get("dataDelimiter") or "|"
    hpath = ds.get("headerPath")
    header = header or read_header(mc.resolve(hpath) if hpath else None, ds.get("headerDelimiter") or "|",
                                   data_path, delim)
    skip = (not hpath) and first_line_is_header(data_path, header, delim)
    todo = [c for c in ms.ccs if not c.is_target() and not c.is_meta() and not c.is_weight()]
    t = read_table(data_path, header, delim, strings=[header[c.num] for c in todo],
                   missing=mc.missing_values, skip_header_line=skip, max_rows=max_rows)
    thr = float(ds.get("autoTypeThreshold", 0) or 0)
    n_cat = 0
    for c in todo:
        col = t[header[c.num]]
        d = col.dictionary
        counts = np.bincount(col.values[col.values >= 0], minlength=len(d)) if len(d) else np.zeros(0, np.int64)
        c.stats["distinctCount"] = int(len(d))
        if thr <= 0 or c.is_categorical() and c.name in set(mc.categorical_column_names()):
            continue
        valid = 0
        nums = []
        for s, k in zip(d, counts):
            try:
                nums.append(float(s))
                valid += int(k)
            except ValueError:
                pass
        nonmiss = int(counts.sum())
        ratio = valid / nonmiss if nonmiss else 1.0
        if len(d) == 2 and set(nums) <= {0.0, 1.0} and len(nums) == 2:
            c.type = "N"
        elif ratio > thr / 100.0:
            c.type = "N"
        else:
            c.type = "C"
            n_cat += 1
    _log.info("auto type: %d categorical columns", n_cat)
    return n_cat


def run_new(name: str, alg: str = "NN", description: str | None = None, parent: str = ".") -> int:
    create_model_set(name, alg, description, parent)
    return 0


def run_init(root: str = ".", auto_type: bool | None = None) -> int:
    ms = ModelSet(root).setup("INIT", update_flags=False)
    init_column_configs(ms, auto_type)
    save_column_configs(ms.ccs, ms.pf.column_config)
    _log.info("init: %d columns -> %s", len(ms.ccs), ms.pf.column_config)
    return 0


def copy_model_set(src: str, dst: str) -> int:
    """``shifu cp <src> <dst>`` (BasicModelProcessor.copyModelFiles :357-369): the source's
    ModelConfig.json is written into ``dst`` with the model-set name = basename(dst) and the
    creator = the current user."""
    import getpass
    from ..config.model_config import ModelConfig
    mc = ModelConfig.load(os.path.join(src, "ModelConfig.json"))
    os.makedirs(dst, exist_ok=True)
    mc.basic["name"] = os.path.basename(os.path.normpath(dst))
    try:
        mc.basic["author"] = getpass.getuser()
    except Exception:                     # noqa: BLE001 - no passwd entry in some containers
        pass
    mc.save(os.path.join(dst, "ModelConfig.json"))
    _log.info("Model set %s copied to %s", src, dst)
    return 0


def init_model_params(root: str = ".") -> int:
    """``shifu init -model`` (ShifuCLI.initializeModelParam :632-635 ->
    checkAlgorithmParam): fill the default train.params of the configured algorithm."""
    from .base import ModelSet, check_algorithm_params
    ms = ModelSet(root)
    check_algorithm_params(ms.mc)
    ms.save_mc()
    return 0
