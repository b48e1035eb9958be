"""Shared step lifecycle (B1) and the columnar dataset cache (D5).

``BasicModelProcessor.setUp`` (J/core/processor/BasicModelProcessor.java:104-156): load
ModelConfig/ColumnConfig, validate for the step, refresh column flags, save; ``checkAlgorithmParam``
(:404-494) fills default algorithm params; ``runDataClean`` (:584-634) produces un-normalized
bin codes for trees.

Data artifacts are not Pig text part-files: ``norm`` writes a columnar cache of ``.npy`` arrays
(``X`` float32 [N, F'], ``y``, ``w``, tree ``codes`` uint8/int16 [N, F]) plus ``meta.json``.
Training memory-maps them and streams row chunks straight into HBM, so a 100M x 1k table never
needs a second host copy.
"""
from __future__ import annotations

import json
import os
import shutil
import time

import numpy as np

from ..config import validator
from ..config.column_config import load_column_configs, save_column_configs
from ..config.errors import ShifuErrorCode, ShifuException
from ..config.model_config import ModelConfig, create_params_by_alg
from ..config.path_finder import PathFinder
from ..config.updater import update_column_flags
from ..utils.log import get_logger

_log = get_logger("steps")


class ModelSet:
    """A model-set directory: ModelConfig.json + ColumnConfig.json + artifacts."""

    def __init__(self, root: str = ".", mc: ModelConfig | None = None, ccs=None):
        self.root = os.path.abspath(root)
        mcp = os.path.join(self.root, "ModelConfig.json")
        if mc is None:
            if not os.path.exists(mcp):
                raise ShifuException(ShifuErrorCode.ERROR_MODELCONFIG_NOT_EXIST, mcp)
            mc = ModelConfig.load(mcp)
        if mc.path is None:
            mc.path = mcp
        self.mc = mc
        self.pf = PathFinder(mc, self.root)
        if ccs is None and os.path.exists(self.pf.column_config):
            ccs = load_column_configs(self.pf.column_config)
        self.ccs = ccs or []

    # ---- lifecycle -----------------------------------------------------------------------
    def setup(self, step: str, validate: bool = True, update_flags: bool = True):
        if validate:
            r = validator.probe(self.mc, step)
            if not r:
                raise ShifuException(ShifuErrorCode.ERROR_MODELCONFIG_NOT_VALIDATION, "; ".join(r.causes))
        check_algorithm_params(self.mc)
        if step in ("NORMALIZE", "VARSELECT", "TRAIN", "EVAL") and self.mc.segment_filter_expressions() \
                and self.mc.algorithm not in ("NN", "LR"):
            raise ValueError("Segment expression is only supported in NN or LR model "
                             "(BasicModelProcessor.setUp :140-155)")
        if update_flags and self.ccs:
            update_column_flags(self.mc, self.ccs, step)
        return self

    def save_mc(self):
        if not _writer():
            return
        self.mc.save(self.pf.model_config)

    def save_cc(self, backup: bool = False):
        if not _writer():
            return
        if backup and os.path.exists(self.pf.column_config):
            dst = self.pf.ensure(self.pf.backup_column_config(time.strftime("%Y%m%d%H%M%S")))
            shutil.copyfile(self.pf.column_config, dst)
        save_column_configs(self.ccs, self.pf.column_config)

    # ---- column helpers ----------------------------------------------------------------------
    def selected(self):
        return [c for c in self.ccs if c.final_select and not c.is_target() and not c.is_meta()]

    def candidates(self):
        from ..config.column_config import has_candidates
        hc = has_candidates(self.ccs)
        return [c for c in self.ccs if c.is_candidate(hc)]

    def stats_columns(self):
        return [c for c in self.ccs if not c.is_target() and not c.is_meta() and not c.is_weight()
                and not c.is_force_remove()]

    def input_columns(self):
        from ..config.column_config import model_input_columns
        return model_input_columns(self.ccs, self.mc.is_binary())

    def norm_columns(self):
        """Columns written by ``norm``: every good candidate plus force/final-selected ones
        (Normalize.pig keeps candidates so varsel may run after norm; train then picks the
        final-selected subset from the cache)."""
        from ..config.column_config import has_candidates
        hc = has_candidates(self.ccs)
        return [c for c in self.ccs if not c.is_target() and not c.is_meta() and
                (c.final_select or c.is_force_select() or c.is_good_candidate(hc, self.mc.is_binary()))]

    def load_raw(self, columns, data_conf=None, sample_rate=1.0, sample_neg_only=False, seed=0,
                 extra_filter=None, require_target=True):
        from ..data.purifier import load_dataset
        nums = [c.name for c in columns if not c.is_categorical()]
        strs = [c.name for c in columns if c.is_categorical()]
        return load_dataset(self.mc, data_conf or self.mc.dataSet, nums, strs, sample_rate, sample_neg_only,
                            seed, require_target, extra_filter)


def _writer() -> bool:
    """Only rank 0 writes model-set files (every rank holds the same replicated state)."""
    from ..parallel import dist
    return dist.info().rank == 0


def shard_model_data(md):
    """This rank's contiguous row range of ``md`` (all of it for a single process)."""
    from dataclasses import replace
    from ..parallel import dist
    i = dist.info()
    if i.world_size <= 1:
        return md
    lo, hi = md.n * i.rank // i.world_size, md.n * (i.rank + 1) // i.world_size
    idx = np.arange(lo, hi)
    return replace(md, table=md.table.take(idx), y=md.y[idx], w=md.w[idx], tag_index=md.tag_index[idx])


def check_algorithm_params(mc):
    """Fill default params for the algorithm (``checkAlgorithmParam``)."""
    alg = mc.algorithm
    params = mc.train.get("params")
    if params is None:
        mc.train["params"] = create_params_by_alg(alg)
        return
    for k, v in create_params_by_alg(alg).items():
        if k not in params:
            params[k] = v


# ---- columnar dataset cache ---------------------------------------------------------------------
def save_dataset(path: str, arrays: dict, meta: dict):
    if os.path.isdir(path):
        shutil.rmtree(path)
    os.makedirs(path, exist_ok=True)
    for k, v in arrays.items():
        if v is not None:
            np.save(os.path.join(path, f"{k}.npy"), np.ascontiguousarray(v))
    with open(os.path.join(path, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1)


def load_dataset_cache(path: str, mmap: bool = True):
    if not os.path.exists(os.path.join(path, "meta.json")):
        return None
    with open(os.path.join(path, "meta.json")) as f:
        meta = json.load(f)
    if meta.get("parts"):           # streamed per-rank parts (data/rowstore.py)
        from ..data.rowstore import Bf16Rows, load_parts
        arrs = load_parts(path, meta, mmap)
        if "Xb" in arrs and "X" not in arrs:        # bf16 GEMM-ready rows (shifu.norm.dtype=bf16)
            arrs["X"] = Bf16Rows(arrs.pop("Xb"), meta["x_width"])
        return meta, arrs
    arrs = {}
    for fn in os.listdir(path):
        if fn.endswith(".npy"):
            arrs[fn[:-4]] = np.load(os.path.join(path, fn), mmap_mode="r" if mmap else None)
    return meta, arrs


def tag_targets(mc, md):
    """ModelData -> training target: binary 0/1, multi-class index, or regression value."""
    return md.y.astype(np.float32)
