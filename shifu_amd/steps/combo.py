"""``combo -new/-init/-run/-eval`` (B11, H16): stacking of sub-models.

``ComboModelProcessor.run`` (J/core/processor/ComboModelProcessor.java:80, ``runComboModels``
:278-356): N sub-model sets with different algorithms train on the same data; their scores are
joined to the raw rows; an assemble model set force-selects the sub-model score columns and runs
the normal pipeline (init, stats, norm, varsel, train).  ``-eval`` scores the eval sets with every
sub-model and evaluates the assemble model on the joined rows.

Layout (under the parent model set): ``ComboTrain.json``, ``<name>_<ALG>_<i>/`` sub model sets,
``<name>_assemble/`` with ``data/`` (training rows + score columns) and ``evaldata/<eval>/``.
"""
from __future__ import annotations

import json
import os
import shutil

import numpy as np

from ..config.model_config import ModelConfig, create_params_by_alg
from ..scoring.model_runner import ModelRunner
from ..utils.log import get_logger
from .base import ModelSet

_log = get_logger("steps.combo")


def combo_new(root: str, algs: str, assemble_alg: str | None = None):
    ms = ModelSet(root)
    parts = [a.strip().upper() for a in algs.split(",") if a.strip()]
    if assemble_alg is None:
        assemble_alg = parts[-1] if len(parts) > 1 else "LR"
        parts = parts[:-1] if len(parts) > 1 else parts
    cfg = {"subTrains": [{"modelName": f"{ms.mc.name}_{a}_{i}", "algorithm": a} for i, a in enumerate(parts)],
           "assemble": {"modelName": f"{ms.mc.name}_assemble", "algorithm": assemble_alg.upper()}}
    with open(ms.pf.combo_config, "w") as f:
        json.dump(cfg, f, indent=2)
    return cfg


def _load_cfg(ms):
    with open(ms.pf.combo_config) as f:
        return json.load(f)


def _sub_dir(ms, name):
    return os.path.join(ms.root, name)


def combo_init(root: str):
    ms = ModelSet(root)
    cfg = _load_cfg(ms)
    for sub in cfg["subTrains"] + [cfg["assemble"]]:
        d = _sub_dir(ms, sub["modelName"])
        os.makedirs(os.path.join(d, "columns"), exist_ok=True)
        mc = ModelConfig.load(ms.pf.model_config)
        mc.basic["name"] = sub["modelName"]
        mc.train["algorithm"] = sub["algorithm"]
        mc.train["params"] = create_params_by_alg(sub["algorithm"])
        for k in ("dataPath", "headerPath"):       # absolute paths: sub sets live one level down
            if mc.dataSet.get(k):
                mc.dataSet[k] = mc.resolve(mc.dataSet.get(k))
        for key in ("metaColumnNameFile", "categoricalColumnNameFile"):
            v = mc.dataSet.get(key)
            if v and os.path.exists(mc.resolve(v)):
                mc.dataSet[key] = mc.resolve(v)
        for ev in mc.evals:
            for k in ("dataPath", "headerPath"):
                if ev.dataSet.get(k):
                    ev.dataSet[k] = mc.resolve(ev.dataSet.get(k))
        for key in ("forceSelectColumnNameFile", "forceRemoveColumnNameFile", "candidateColumnNameFile"):
            v = mc.varSelect.get(key)
            if v and os.path.exists(mc.resolve(v)):
                mc.varSelect[key] = mc.resolve(v)
        mc.save(os.path.join(d, "ModelConfig.json"))
        if os.path.exists(ms.pf.column_config) and sub is not cfg["assemble"]:
            shutil.copyfile(ms.pf.column_config, os.path.join(d, "ColumnConfig.json"))
    return cfg


def _pipeline(root, steps=("init", "stats", "norm", "varsel", "train"), skip_init_if_cc=True, shuffle=False):
    from .create import run_init
    from .norm import run_norm
    from .stats import run_stats
    from .train import run_train
    from .varsel import run_varsel
    from ..parallel import dist
    # under torchrun every step ends with a barrier: rank 0 writes the step's outputs (ColumnConfig,
    # models) that the next step -- or the score join -- reads on every rank
    if "init" in steps and not (skip_init_if_cc and os.path.exists(os.path.join(root, "ColumnConfig.json"))):
        run_init(root)
        dist.barrier()
    if "stats" in steps:
        run_stats(root)
        dist.barrier()
    if "norm" in steps:
        run_norm(root, shuffle=shuffle)
        dist.barrier()
    if "varsel" in steps:
        run_varsel(root)
        dist.barrier()
    if "train" in steps:
        if shuffle:
            run_norm(root, shuffle=True)        # `train -shuffle` re-shuffles the normalized data
            dist.barrier()
        run_train(root)
        dist.barrier()


def _join_scores(subs, confs, out_dir: str) -> str:
    """Every sub model's mean score (x1000, ``%.6f``) appended to the raw rows of a data set
    (``confs[i]``: sub model i's view of it), streamed per rank into ``out_dir/part-<rank>``
    (``data/join.stream_join``) -> the data delimiter (also the ``.pig_header`` delimiter)."""
    from ..data.join import FIXED6, stream_join
    from ..data.purifier import plan_dataset
    from ..data.reader import column_kinds
    from ..parallel import dist
    runners = [(f"{name}_score", ModelRunner(sms.mc, sms.ccs, sms.pf.models_dir)) for name, sms in subs]
    cats = set()
    need = set()
    for (_, sms), (_, r) in zip(subs, runners):
        cats |= {c.name for c in sms.ccs if c.is_categorical()}
        need |= set(r.raw_columns())
    mc0 = subs[0][1].mc
    plan = plan_dataset(mc0, confs[0], [h for h in need if h not in cats], [h for h in need if h in cats])
    kinds = column_kinds(plan.header, plan.nums, plan.strs)

    def compute(table, n):
        return [(FIXED6, np.asarray(r.score(table, 1000.0)["mean"], dtype=np.float64)) for _, r in runners]
    info = dist.info()
    stream_join(plan, out_dir, [k for k, _ in runners], kinds, compute, info.rank, info.world_size)
    return plan.delim or "|"


def _has_models(d: str) -> bool:
    md = os.path.join(d, "models")
    return os.path.isdir(md) and any(not f.startswith(".") for f in os.listdir(md))


def combo_run(root: str, shuffle: bool = False, resume: bool = False):
    """Under torchrun (world > 1) every sub model's pipeline runs data parallel over all ranks, one
    after the other -- the reference runs one distributed Guagua job per sub model
    (ComboModelProcessor.java:278-356) -- then the score join (each rank joins its byte ranges) and
    the assemble pipeline.  In one process, ``shifu.combo.parallel > 1`` runs sub models side by side
    as child processes, each pinned to a GPU of its own (``DevicePool``; at most one child per GPU)."""
    from ..config import environment
    from ..parallel import dist
    from ..runtime.executor import DevicePool, ExecutorManager, cli_task
    ms = ModelSet(root)
    cfg = _load_cfg(ms)
    # sub models train with retries (ExecutorManager); shifu.combo.parallel > 1 runs them side by
    # side as child processes (ProcessManager), each with its own log under the sub model set
    parallel = int(environment.get("shifu.combo.parallel", 1) or 1)
    retries = int(environment.get("shifu.combo.retries", 1) or 0)
    dirs = [_sub_dir(ms, sub["modelName"]) for sub in cfg["subTrains"]]
    for sub in cfg["subTrains"]:
        _log.info("combo: training sub model %s (%s)", sub["modelName"], sub["algorithm"])
    # -resume: sub models that already hold trained models are not trained again
    todo = [(sub, d) for sub, d in zip(cfg["subTrains"], dirs) if not (resume and _has_models(d))]
    if resume and len(todo) < len(dirs):
        _log.info("combo -resume: %d of %d sub models already trained", len(dirs) - len(todo), len(dirs))
    info = dist.info()
    if info.world_size > 1:
        if parallel > 1:
            _log.info("combo: %d ranks -- sub models run data parallel in turn (shifu.combo.parallel unused)",
                      info.world_size)
        for sub, d in todo:          # a failure on one rank must stop every rank: no retries here
            _pipeline(d, shuffle=shuffle)
    elif parallel > 1:
        steps = ["init", "stats", "norm -shuffle" if shuffle else "norm", "varsel",
                 "train -shuffle" if shuffle else "train"]
        devices = DevicePool.for_node()
        workers = min(parallel, len(devices)) if devices is not None else parallel
        tasks = [cli_task([s for s in steps if not (s == "init" and os.path.exists(os.path.join(d, "ColumnConfig.json")))],
                          d, os.path.join(d, "combo_sub.log"), devices=devices) for _, d in todo]
        ExecutorManager(workers, retries).run(tasks, [sub["modelName"] for sub, _ in todo])
    else:
        tasks = [(lambda d=d: _pipeline(d, shuffle=shuffle)) for _, d in todo]
        ExecutorManager(1, retries).run(tasks, [sub["modelName"] for sub, _ in todo])
    subs = [(sub["modelName"], ModelSet(d)) for sub, d in zip(cfg["subTrains"], dirs)]
    asm = cfg["assemble"]
    ad = _sub_dir(ms, asm["modelName"])
    data_dir = os.path.join(ad, "data")
    delim = _join_scores(subs, [sms.mc.dataSet for _, sms in subs], data_dir)
    if info.rank == 0:
        ams = ModelSet(ad)
        ams.mc.dataSet["dataPath"] = data_dir
        ams.mc.dataSet["headerPath"] = os.path.join(data_dir, ".pig_header")
        ams.mc.dataSet["headerDelimiter"] = delim
        fs = os.path.join(ad, "columns", "forceselect.column.names")
        with open(fs, "w") as f:
            f.write("\n".join(f"{name}_score" for name, _ in subs) + "\n")
        ams.mc.varSelect["forceSelectColumnNameFile"] = fs
        ams.mc.varSelect["forceEnable"] = True
        ams.save_mc()
    dist.barrier()
    _pipeline(ad, skip_init_if_cc=False, shuffle=True)   # assemble model: norm -shuffle / train -shuffle
    return 0


def combo_eval(root: str):
    from ..parallel import dist
    from .evaluate import run_eval
    ms = ModelSet(root)
    cfg = _load_cfg(ms)
    asm = cfg["assemble"]
    ad = _sub_dir(ms, asm["modelName"])
    ams = ModelSet(ad)
    subs = [(sub["modelName"], ModelSet(_sub_dir(ms, sub["modelName"]))) for sub in cfg["subTrains"]]
    for ev in ams.mc.evals:
        confs = [[e for e in sms.mc.evals if e.get("name") == ev.get("name")][0].dataSet for _, sms in subs]
        out = os.path.join(ad, "evaldata", ev.get("name"))
        delim = _join_scores(subs, confs, out)
        ev.dataSet["dataPath"] = out
        ev.dataSet["headerPath"] = os.path.join(out, ".pig_header")
        ev.dataSet["headerDelimiter"] = delim
    if dist.info().rank == 0:
        ams.save_mc()
    dist.barrier()
    return run_eval(ad)


def run_combo(root=".", action="run", algs: str | None = None, shuffle: bool = False, resume: bool = False) -> int:
    from ..parallel import dist
    if action in ("new", "init"):      # config writes: rank 0 alone, the others wait for it
        if dist.info().rank == 0:
            with dist.local_only():
                combo_new(root, algs or "NN,LR") if action == "new" else combo_init(root)
        dist.barrier()
    elif action == "run":
        combo_run(root, shuffle=shuffle, resume=resume)
    elif action == "eval":
        combo_eval(root)
    else:
        raise ValueError(f"unknown combo action {action}")
    return 0
