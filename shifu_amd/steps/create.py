"""``new`` (B2) and ``init`` (B3) steps.

* new: ``CreateModelProcessor.run`` (J/core/processor/CreateModelProcessor.java:71-108) — model-set
  folder, default ModelConfig.json for the algorithm, ``.HEAD``, empty column-name files.
* init: ``InitModelProcessor.initColumnConfigList`` (J/core/processor/InitModelProcessor.java:424-502)
  — one ColumnConfig per header field (or per index without a header), flags from the column
  files; optional auto-type (:105-120, 143-254 + the AutoTypeDistinctCount MapReduce job): one
  data-parallel streamed pass (algos/autotype.py), see ``auto_type_columns``.
"""
from __future__ import annotations

import os

import numpy as np

from ..config.column_config import ColumnConfig, save_column_configs
from ..config.model_config import create_init_model_config
from ..config.updater import update_column_flags
from ..data.reader import list_data_files, read_header
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


def _is_binary(distinct: int, items: list) -> bool:
    """``InitModelProcessor.isBinaryVariable`` (:229-246): two distinct values, both 0 or 1."""
    if distinct != 2 or len(items) > 2:
        return False
    for s in items:
        v = _java_double(s)
        if v is None or v not in (0.0, 1.0):
            return False
    return True


def _java_double(s: str):
    """Double.valueOf: surrounding whitespace trimmed, an optional d/D/f/F suffix, NaN / Infinity;
    None when it would throw NumberFormatException."""
    t = str(s).strip()
    if t[-1:] in ("d", "D", "f", "F") and not t.endswith(("Infinity", "NaN")):
        t = t[:-1]
    u = t.lstrip("+-")
    if u in ("NaN", "Infinity"):
        return float(t.replace("Infinity", "inf"))
    if not t or any(ch in u.lower() for ch in ("n", "x", "_", "i")):
        return None
    try:
        return float(t)
    except ValueError:
        return None


def auto_type_columns(ms: ModelSet, header=None, max_rows: int | None = None):
    """Distinct counts (+ the column type when autoTypeThreshold > 0) from one data-parallel pass
    over the training data (algos/autotype.py: every rank streams its byte ranges; counts,
    hash sets / HyperLogLog registers and frequent items merged over the ranks).

    Type rule (``shifu.autoType.rule``):

    * ``reference`` (default) -- exactly InitModelProcessor.setCategoricalColumnsAndDistinctAccount
      (:181-219): a 0/1 column is numeric (isBinaryVariable :221-241); otherwise
      isDoubleFrequentVariable (:243-254) decides, and as written it tries Double.parseDouble only
      on BLANK sampled items, so a column is categorical exactly when one of its sampled items is
      whitespace-only, numeric otherwise; user categorical columns are re-typed too, as there;
    * ``ratio`` -- the intent documented beside it: numeric when more than autoTypeThreshold % of
      the non-missing values parse as doubles (setCategoricalColumnsByCountInfo :143-179's test),
      columns listed in categorical.column.names kept categorical."""
    from ..algos import autotype
    from ..config import environment
    from ..parallel import dist
    mc = ms.mc
    ds = mc.dataSet
    data_path = mc.resolve(ds.get("dataPath"))
    delim = ds.get("dataDelimiter") or "|"
    hpath = ds.get("headerPath")
    header = header or read_header(mc.resolve(hpath) if hpath else None, ds.get("headerDelimiter") or "|",
                                   data_path, delim)
    todo = [c for c in ms.ccs if not c.is_target() and not c.is_meta() and not c.is_weight() and c.num < len(header)]
    info = dist.info()
    st = autotype.scan(mc, header, [c.num for c in todo], info.rank, info.world_size)
    thr = float(ds.get("autoTypeThreshold", 0) or 0)
    rule = str(environment.get("shifu.autoType.rule", "reference")).lower()
    user_cat = set(mc.categorical_column_names())
    n_cat = 0
    for c in todo:
        s = st[c.num]
        c.stats["distinctCount"] = int(s.distinct)
        if thr <= 0:
            continue
        if rule == "ratio":
            if c.is_categorical() and c.name in user_cat:
                continue
            nonmiss = s.count - s.invalid
            ratio = s.validnum / nonmiss if nonmiss else 1.0
            numeric = _is_binary(s.distinct, s.items) or ratio > thr / 100.0
        else:
            numeric = _is_binary(s.distinct, s.items) or not any(not str(it).strip() for it in s.items)
        if numeric:
            c.type = "N"
        else:
            c.type = "C"
            n_cat += 1
    _log.info("auto type (%s rule): %d categorical columns", "ratio" if rule == "ratio" else "reference", n_cat)
    return n_cat


def run_new(name: str, alg: str = "NN", description: str | None = None, parent: str = ".") -> int:
    create_model_set(name, alg, description, parent)
    return 0


def run_init(root: str = ".", auto_type: bool | None = None) -> int:
    """Every rank builds the ColumnConfig (the auto-type pass is data parallel); rank 0 writes it."""
    from ..parallel import dist
    ms = ModelSet(root).setup("INIT", update_flags=False)
    init_column_configs(ms, auto_type)
    if dist.info().rank == 0:
        save_column_configs(ms.ccs, ms.pf.column_config)
        _log.info("init: %d columns -> %s", len(ms.ccs), ms.pf.column_config)
    dist.barrier()
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
    from ..parallel import dist
    from .base import ModelSet, check_algorithm_params
    if dist.info().rank == 0:          # one writer of ModelConfig.json under torchrun
        ms = ModelSet(root)
        check_algorithm_params(ms.mc)
        ms.save_mc()
    dist.barrier()
    return 0
