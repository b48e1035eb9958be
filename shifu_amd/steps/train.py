"""``train`` step (B7): NN / LR / GBT / RF / WDL with bagging, k-fold, grid search, one-vs-all,
continuous training, checkpoints, early stop, progress log.

Reference flow: ``TrainModelProcessor.run`` (J/core/processor/TrainModelProcessor.java:167-218) ->
``runDistributedTrain`` (:661-1029) launching one Guagua master/worker job per bag / grid point /
fold; ``NNMaster``/``NNWorker``, ``LogisticRegressionMaster``/``Worker``, ``DTMaster``/``DTWorker``
iterate; ``NNOutput``/``DTOutput`` write progress (``    Trainer i Epoch #e Training Error:..
Validation Error:..``), tmp models every ``max(epochs/25, 20)`` epochs and the final models.

MI355X design: there is no master.  Every rank (one per GPU, ``torchrun``) owns a contiguous row
shard resident in HBM; each epoch is a fused HIP gradient pass + ONE RCCL all-reduce of the flat
gradient buffer (error/count folded into its tail) + an identical replicated optimizer update.
Bags / folds / grid points run one after another over the same resident shard (the data are
loaded once), which replaces the reference's "three-level parallel" job fan-out.
"""
from __future__ import annotations

import itertools
import json
import math
import os
import time

import numpy as np
import torch

from ..formats import nn_format, tree_format
from ..models import lr as lrmod
from ..models.nn import MLPSpec, MLPTrainer, can_grow, grow_weights
from ..parallel import dist
from ..runtime.fault import IterationWatchdog, check_finite, iteration_limit, maybe_fault
from ..utils.log import get_logger
from ..utils.trace import trace_range
from ..utils.metrics import MetricsWriter
from .base import ModelSet, load_dataset_cache
from .norm import TREE_ALGS, _norm_one

_log = get_logger("steps.train")

LIST_PARAMS = {"NumHiddenNodes", "ActivationFunc", "FixedLayers", "NumEmbedColumnIds"}


# ---- grid search (GridSearch J/core/dtrain/gs/GridSearch.java:76-246) ----------------------------
def flatten_grid(params: dict, grid_file_lines=None):
    if grid_file_lines:
        out = []
        for line in grid_file_lines:
            line = line.strip()
            if not line or line.startswith("#"):
                continue
            p = dict(params)
            for kv in line.split(";"):
                if ":" not in kv:
                    raise ValueError(f"grid config line must be k:v;k:v -> {line!r}")
                k, v = kv.split(":", 1)
                p[k.strip()] = _parse_value(v.strip())
            out.append(p)
        return out
    keys, vals = [], []
    for k, v in params.items():
        if isinstance(v, list) and v and ((k in LIST_PARAMS and isinstance(v[0], list)) or k not in LIST_PARAMS):
            keys.append(k)
            vals.append(v)
    if not keys:
        return [dict(params)]
    out = []
    for combo in itertools.product(*vals):
        p = dict(params)
        p.update(zip(keys, combo))
        out.append(p)
    return out


def _parse_value(s):
    try:
        return json.loads(s)
    except ValueError:
        if s.startswith("[") and s.endswith("]"):
            return [_parse_value(x.strip()) for x in s[1:-1].split(",") if x.strip()]
        return s


def checkpoint_interval(params: dict, default: int) -> int:
    """``CheckpointInterval`` param or ``-Dshifu.train.checkpoint.interval``; default = the
    reference's tmp-model cadence max(epochs/25, 20) (DTrainUtils.tmpModelFactor :293-295)."""
    from ..config import environment
    v = params.get("CheckpointInterval") or environment.get("shifu.train.checkpoint.interval")
    try:
        v = int(float(v))
    except (TypeError, ValueError):
        v = 0
    return v if v > 0 else default


def _num(v, default):
    if v is None:
        return default
    if isinstance(v, str):
        try:
            return float(v)
        except ValueError:
            return default
    return v


# ---- data ---------------------------------------------------------------------------------------------
class TrainSet:
    """Host-side (memory-mapped) training arrays of this rank's shard."""

    def __init__(self, X=None, codes=None, y=None, w=None, meta=None, vX=None, vcodes=None, vy=None, vw=None,
                 row0: int = 0):
        self.X, self.codes, self.y, self.w, self.meta = X, codes, y, w, meta or {}
        self.vX, self.vcodes, self.vy, self.vw = vX, vcodes, vy, vw
        self.row0 = int(row0)          # global index of this shard's first row (per-row draws)

    @property
    def n(self):
        return len(self.y)


def _shard(a, info):
    if a is None or info.world_size == 1:
        return a
    n = len(a)
    lo, hi = n * info.rank // info.world_size, n * (info.rank + 1) // info.world_size
    return a[lo:hi]


def _subset_cache(meta, arr, want, is_tree):
    """Column subset of a Normalized/CleanedData cache for the model inputs ``want`` (column
    nums in ColumnConfig order); None if some wanted column is missing from the cache."""
    if is_tree:
        nums = meta["column_nums"]
        pos = {n: i for i, n in enumerate(nums)}
        if any(n not in pos for n in want):
            return None
        idx = [pos[n] for n in want]
        if idx == list(range(len(nums))):
            return meta, arr
        meta = dict(meta, column_nums=list(want), nbins=[meta["nbins"][i] for i in idx],
                    is_cat=[meta["is_cat"][i] for i in idx])
        return meta, dict(arr, codes=np.asarray(arr["codes"])[:, idx])
    inums = meta["input_nums"]
    have = set(inums)
    if any(n not in have for n in want):
        return None
    wanted = set(want)
    idx = [i for i, n in enumerate(inums) if n in wanted]
    if len(idx) == len(inums):
        return meta, arr
    meta = dict(meta, input_nums=[inums[i] for i in idx], input_names=[meta["input_names"][i] for i in idx])
    from ..data.rowstore import Bf16Rows
    if isinstance(arr["X"], Bf16Rows):          # bf16 cache: a column view, nothing expanded on the host
        return meta, dict(arr, X=arr["X"].subset(idx))
    return meta, dict(arr, X=np.asarray(arr["X"])[:, idx])


def load_train_set(ms: ModelSet, is_tree: bool) -> TrainSet:
    info = dist.info()
    want = [c.num for c in ms.input_columns()]
    cache = load_dataset_cache(ms.pf.cleaned_data if is_tree else ms.pf.normalized_data)
    if cache is not None:
        cache = _subset_cache(*cache, want, is_tree)
    if cache is None:
        _log.info("no usable %s cache; normalizing in memory", "CleanedData" if is_tree else "NormalizedData")
        cols = ms.input_columns()
        tmp_x, tmp_t = ms.pf.p("tmp", "_mem_norm"), ms.pf.p("tmp", "_mem_clean")
        if info.rank == 0:
            _norm_one(ms, cols, ms.mc.dataSet, tmp_x, tmp_t, 1.0, False, False, 0, is_tree)
        dist.barrier()
        cache = load_dataset_cache(tmp_t if is_tree else tmp_x)
    meta, arr = cache
    ntot = len(arr["y"])
    ts = TrainSet(X=_shard(arr.get("X"), info), codes=_shard(arr.get("codes"), info), y=_shard(arr["y"], info),
                  w=_shard(arr["w"], info), meta=meta, row0=ntot * info.rank // info.world_size)
    vc = load_dataset_cache(ms.pf.cleaned_validation_data if is_tree else ms.pf.normalized_validation_data)
    if vc is not None:
        vc = _subset_cache(*vc, want, is_tree)
    if vc is not None:
        vm, va = vc
        ts.vX, ts.vcodes = _shard(va.get("X"), info), _shard(va.get("codes"), info)
        ts.vy, ts.vw = _shard(va["y"], info), _shard(va["w"], info)
    return ts


def _poisson_from_uniform(u: np.ndarray, lam: float) -> np.ndarray:
    """Poisson(lam) draws by inversion of the given uniforms (per-row, counter-based)."""
    k = np.zeros(len(u), np.float32)
    p = np.full(len(u), np.exp(-lam))
    c = p.copy()
    for i in range(1, 64):
        more = u > c
        if not more.any():
            break
        k += more
        p = p * lam / i
        c = c + p
    return k


# Version of the train / validation / bagging draws stored in checkpoints: 2 = counter-based per
# global row (row_uniform); 1 (absent) = the per-rank default_rng draws of rounds <= 4.  A resume
# across versions keeps training but warns: rows may have moved between the two sets.
SPLIT_SCHEME = 2


def _check_split_scheme(st: dict, what: str) -> None:
    v = int(st.get("split_scheme", 1)) if isinstance(st, dict) else 1
    if v != SPLIT_SCHEME:
        _log.warning("%s: checkpoint written with train/validation split scheme %d, resuming with scheme %d "
                     "(counter-based per-row draws): some rows move between the training and the validation "
                     "set", what, v, SPLIT_SCHEME)


def split_masks(mc, ts: TrainSet, bag: int, n_kfold: int, seed: int):
    """-> (train_mask, valid_mask, sample_weight) for one bag (AbstractNNWorker :667-800).  Every
    per-row draw (validation split, bagging) is a counter-based function of the row's GLOBAL index
    (``purifier.row_uniform``), so the split is the same in one process and over any number of
    data-parallel ranks (each rank holds rows [ts.row0, ts.row0 + n))."""
    from ..data.purifier import row_uniform
    n = ts.n
    tr = mc.train
    base = (seed * 7919 + bag) * 4
    y = np.asarray(ts.y)
    if n_kfold and n_kfold > 0:
        gid = np.arange(ts.row0, ts.row0 + n, dtype=np.uint64)
        fold = ((gid * np.uint64(2654435761)) % np.uint64(1 << 32)) % np.uint64(n_kfold)   # row-hash fold id
        valid = fold == bag
    elif ts.vy is not None:
        valid = np.zeros(n, dtype=bool)
    else:
        # stratifiedSample: a per-row draw at the same rate keeps every class's share in
        # expectation, which is what the reference's per-class sampling does
        rate = float(tr.get("validSetRate", 0.2) or 0.0)
        valid = row_uniform(base, ts.row0, n) < rate
    train = ~valid
    rate = float(tr.get("baggingSampleRate", 1.0))
    if n_kfold and n_kfold > 0:
        sw = np.ones(n, np.float32)
    elif bool(tr.get("baggingWithReplacement", False)):
        sw = _poisson_from_uniform(row_uniform(base + 1, ts.row0, n), rate)
    else:
        sw = (row_uniform(base + 2, ts.row0, n) <= rate).astype(np.float32) if rate < 1.0 else np.ones(n, np.float32)
    if bool(tr.get("sampleNegOnly", False)) and mc.is_binary():
        sw = np.where(y > 0.5, 1.0, sw).astype(np.float32)
    up = float(tr.get("upSampleWeight", 1.0) or 1.0)
    if up != 1.0 and mc.is_binary():
        sw = np.where(y > 0.5, sw * up, sw).astype(np.float32)
    return train, valid, sw


# ---- early stop (WindowEarlyStop / ConvergeAndValidToleranceEarlyStop) ---------------------------
class EarlyStop:
    def __init__(self, enabled: bool, window: int = 20, tolerance: float = 0.0, converge: float = 0.0,
                 min_epochs: int = 0):
        self.enabled, self.window, self.tol, self.conv, self.min_epochs = enabled, window, tolerance, converge, \
            min_epochs
        self.best, self.best_epoch = math.inf, -1

    def update(self, epoch: int, train_err: float, valid_err: float) -> bool:
        if self.conv > 0 and train_err <= self.conv:
            return True
        if self.tol > 0 and not math.isnan(valid_err) and valid_err <= self.tol:
            return True
        if not self.enabled or math.isnan(valid_err):
            return False
        if valid_err < self.best:
            self.best, self.best_epoch = valid_err, epoch
            return False
        return epoch >= self.min_epochs and epoch - self.best_epoch >= self.window


# ---- the step -----------------------------------------------------------------------------------------
class TrainStep:
    """Programmatic Step API (A5): ``TrainStep(ModelSet(path)).process()``."""

    def __init__(self, ms: ModelSet, dry: bool = False, device=None, resume: bool = True):
        self.ms = ms
        self.mc = ms.mc
        self.dry = dry
        from ..utils.device import default_device
        self.dev = torch.device(device) if device is not None else default_device()
        self.resume = resume
        self.info = dist.info()
        self.progress = None
        self.metrics = None

    # -- logging --
    def _log_epoch(self, trainer_id, epoch, terr, verr, extra=None):
        line = f"    Trainer {trainer_id} Epoch #{epoch} Training Error:{terr:.10f} Validation Error:{verr:.10f}"
        _log.info(line.strip())
        if self.progress is not None:
            self.progress.write(line + "\n")
            self.progress.flush()
        if self.metrics is not None:
            self.metrics.write(trainer=trainer_id, epoch=epoch, train_error=terr, valid_error=verr, **(extra or {}))

    def _epoch_extra(self, tr, rows: float, secs: float) -> dict:
        """Per-epoch throughput fields of the metrics stream: whole-job training rows
        per second, gradient all-reduce milliseconds, HBM in use / peak on this rank."""
        ar = 0.0
        for e0, e1 in tr.comm_events or []:
            if isinstance(e0, float):
                ar += (e1 - e0) * 1e3
            else:
                e1.synchronize()
                ar += e0.elapsed_time(e1)
        if tr.comm_events is not None:
            tr.comm_events.clear()
        out = {"rows_per_s": round(rows / secs, 1) if secs > 0 else None, "epoch_ms": round(secs * 1e3, 3),
               "allreduce_ms": round(ar, 3)}
        if tr.device.type == "cuda":
            out["hbm_gb"] = round(torch.cuda.memory_allocated(tr.device) / 1e9, 3)
            out["hbm_peak_gb"] = round(torch.cuda.max_memory_allocated(tr.device) / 1e9, 3)
        return out

    def _train_tensorflow(self) -> int:
        """``algorithm: TENSORFLOW`` (TensorflowTrainer + train.py): a mini-batch DNN trained on the
        MLP engine's MFMA kernels, gradients all-reduced per batch over RCCL; saved as a generic model under
        ``models/<ModelSetName>/`` (+ ``-checkpoint-<epoch>`` copies)."""
        from ..models.dnn_sgd import save_generic, train_dnn
        ms, mc = self.ms, self.mc
        ts = load_train_set(ms, False)
        if ts.X is None:
            raise ValueError("TENSORFLOW training needs the normalized data (run `shifu norm`)")
        params = dict(mc.train.get("params") or {})
        seed = max(0, int(mc.train.get("baggingSampleSeed", -1)))
        _, valid, sw = split_masks(mc, ts, 0, -1, seed)
        dev = self.dev
        names = [c.name for c in ms.input_columns()]
        name = mc.basic.get("name") or "model"
        out = os.path.join(ms.pf.models_dir, name)
        rank0 = self.info.rank == 0
        if rank0:
            os.makedirs(ms.pf.models_dir, exist_ok=True)

        def log_fn(ep, terr, verr):
            if rank0:
                _log.info("Epoch %d avg train error %.8f, avg validation error is %.8f.", ep, terr, verr)

        def ckpt_fn(model, ep):
            if rank0:
                save_generic(model, f"{out}-checkpoint-{ep}", names, {"epoch": ep})
        model, hist = train_dnn(ts.X, np.asarray(ts.y), np.asarray(sw), valid, params,
                                int(mc.train.get("numTrainEpochs", 100) or 100), dev, seed, log_fn, ckpt_fn)
        if rank0:
            path = save_generic(model, out, names, {"epochs": len(hist),
                                                    "trainError": hist[-1][1] if hist else None})
            _log.info("TENSORFLOW model -> %s", path)
        dist.barrier()
        return 0

    def process(self) -> int:
        ms, mc = self.ms, self.mc
        ms.setup("TRAIN")
        alg = mc.algorithm
        if alg == "GENERIC":
            raise ValueError(f"algorithm {alg}: generic models are trained outside shifu; put their "
                             "GenericModelConfig JSON (+ artifacts) under models/ and run eval/export "
                             "(scoring/generic.py)")
        if alg == "TENSORFLOW":
            return self._train_tensorflow()
        if alg not in ("NN", "LR", "GBT", "RF", "WDL", "SVM"):
            raise ValueError(f"unsupported algorithm {alg}")
        is_tree = alg in TREE_ALGS
        if self.info.rank == 0:
            for d in (ms.pf.models_dir, ms.pf.tmp_models_dir, ms.pf.tmp_dir, ms.pf.valerr_dir):
                os.makedirs(d, exist_ok=True)
            if alg == "NN":
                os.makedirs(ms.pf.bmodels_dir, exist_ok=True)
            self.progress = open(ms.pf.progress_log, "a")
            self.metrics = MetricsWriter(ms.pf.metrics_jsonl)
        params = dict(mc.train.get("params") or {})
        grid_file = mc.train.get("gridConfigFile")
        lines = open(mc.resolve(grid_file)).read().splitlines() if grid_file else None
        grid = flatten_grid(params, lines)
        n_kfold = int(mc.train.get("numKFold", -1) or -1)
        seed = int(mc.train.get("baggingSampleSeed", -1))
        seed = 0 if seed < 0 else seed
        jobs = []
        if len(grid) > 1:
            th = 30
            if len(grid) > th:       # shifu.gridsearch.threshold: random subsample of the grid
                idx = np.random.default_rng(seed).choice(len(grid), th, replace=False)
                grid = [grid[i] for i in sorted(idx)]
            jobs = [(i, p, i, None) for i, p in enumerate(grid)]
        elif n_kfold > 0:
            jobs = [(i, grid[0], i, None) for i in range(n_kfold)]
        elif mc.is_multiclass() and mc.is_one_vs_all():
            tags = mc.tags()
            jobs = [(i, grid[0], i, i) for i in range(len(tags))]
        else:
            jobs = [(i, grid[0], i, None) for i in range(int(mc.train.get("baggingNum", 1) or 1))]
        if self.dry:
            _log.info("dry run: %d jobs %s", len(jobs), [j[1] for j in jobs][:3])
            return 0
        t_start = time.time()
        if self._job_parallel(len(jobs), is_tree):
            val_errors = self._run_jobs_parallel(jobs, is_tree, n_kfold, seed)
        else:
            with trace_range("train.load_data"):
                ts = load_train_set(ms, is_tree)
            val_errors = self._run_jobs(jobs, ts, n_kfold, seed)
        if self.info.rank == 0:
            if len(grid) > 1:
                best = int(np.nanargmin(val_errors))
                _log.info("grid search: the %d-th params are selected (validation error %.8f): %s", best,
                          val_errors[best], grid[best])
                with open(ms.pf.p("tmp", "gridsearch.best.json"), "w") as f:
                    json.dump({"index": best, "valid_error": val_errors[best], "params": grid[best]}, f, indent=1)
            if n_kfold > 0:
                _log.info("k-fold CV: mean validation error %.8f over %d folds", float(np.nanmean(val_errors)),
                          n_kfold)
            if self.progress:
                self.progress.close()
            if self.metrics:
                self.metrics.close()
            _log.info("train: %d model(s) in %.1fs", len(jobs), time.time() - t_start)
        return 0

    # -- jobs -------------------------------------------------------------------------------
    def _run_jobs(self, jobs, ts, n_kfold, seed):
        mc, alg = self.mc, self.mc.algorithm
        val_errors = []
        for trainer_id, p, bag, ova_class in jobs:
            train_m, valid_m, sw = split_masks(mc, ts, bag, n_kfold, seed)
            y = np.asarray(ts.y, dtype=np.float32)
            if ova_class is not None:
                y = (np.rint(y) == ova_class).astype(np.float32)
            if alg == "NN":
                verr = self._train_nn(trainer_id, p, ts, y, train_m, valid_m, sw, ova_class)
            elif alg == "LR":
                verr = self._train_lr(trainer_id, p, ts, y, train_m, valid_m, sw)
            elif alg == "WDL":
                verr = self._train_wdl(trainer_id, p, ts, y, train_m, valid_m, sw)
            elif alg == "SVM":
                verr = self._train_svm(trainer_id, p, ts, y, train_m, valid_m, sw)
            else:
                verr = self._train_tree(trainer_id, p, ts, y, train_m, valid_m, sw)
            val_errors.append(verr)
            if self.info.rank == 0:
                with open(os.path.join(self.ms.pf.valerr_dir, f"val_error_{trainer_id}"), "w") as f:
                    f.write(repr(float(verr)) + "\n")
        return val_errors

    def _job_parallel(self, n_jobs: int, is_tree: bool) -> bool:
        """F6: bags / folds / grid points dealt over the ranks (``shifu.train.jobParallel``):
        ``true`` / ``false``, or ``auto`` (default) = on when there are at least as many jobs as
        ranks and the whole training cache fits in a quarter of one GPU's memory (every rank
        then holds the full table and trains its jobs with no collectives -- the reference runs
        one Guagua job per bag, TrainModelProcessor.runDistributedTrain :661-1029)."""
        from ..config import environment
        if self.info.world_size <= 1 or n_jobs <= 1:
            return False
        mode = str(environment.get("shifu.train.jobParallel", "auto")).lower()
        if mode in ("false", "0", "off"):
            return False
        cache = load_dataset_cache(self.ms.pf.cleaned_data if is_tree else self.ms.pf.normalized_data)
        if cache is None:                  # in-memory normalization is a collective path
            return False
        if mode in ("true", "1", "on"):
            return True
        if n_jobs < self.info.world_size:
            return False
        arr = cache[1]
        nbytes = sum(int(np.asarray(arr[k]).nbytes) for k in ("X", "codes", "y", "w") if arr.get(k) is not None)
        budget = (torch.cuda.get_device_properties(self.dev).total_memory if self.dev.type == "cuda"
                  else 64 << 30) // 4
        return nbytes <= budget

    def _run_jobs_parallel(self, jobs, is_tree, n_kfold, seed):
        """Every rank loads the whole training set and runs jobs rank, rank + R, ... alone
        (``dist.local_only``: a world of one, so each job is exactly the single-process job and
        its model / val_error files are written by the rank that trained it); the validation
        errors are then gathered so rank 0 can pick the grid-search winner."""
        info = self.info
        mine = [j for k, j in enumerate(jobs) if k % info.world_size == info.rank]
        _log.info("job-parallel training: rank %d runs %d of %d jobs", info.rank, len(mine), len(jobs))
        # ranks > 0 log their jobs' epochs to per-rank files that rank 0 appends to the progress
        # log / metrics stream afterwards (the logs then cover every job, as in the sequential path)
        pf = self.ms.pf
        if info.rank:
            self.progress = open(pf.progress_log + f".rank{info.rank:05d}", "w")
            self.metrics = MetricsWriter(pf.metrics_jsonl + f".rank{info.rank:05d}")
        with dist.local_only():
            self.info = dist.info()
            try:
                ts = load_train_set(self.ms, is_tree)
                errs = self._run_jobs(mine, ts, n_kfold, seed)
            finally:
                self.info = info
                if info.rank:
                    self.progress.close()
                    self.metrics.close()
                    self.progress = self.metrics = None
        got = {}
        for part in dist.all_gather_objects([(j[0], e) for j, e in zip(mine, errs)]):
            got.update(dict(part))
        if info.rank == 0:
            for r in range(1, info.world_size):
                for path, fh in ((pf.progress_log, self.progress), (pf.metrics_jsonl, self.metrics)):
                    src = path + f".rank{r:05d}"
                    if not os.path.exists(src) or fh is None:
                        continue
                    with open(src) as f:
                        data = f.read()
                    if isinstance(fh, MetricsWriter):
                        fh.write_raw(data)
                    else:
                        fh.write(data)
                    os.remove(src)
            if self.progress is not None:
                self.progress.flush()
        return [got[j[0]] for j in jobs]

    # -- NN ---------------------------------------------------------------------------------
    def _nn_spec(self, p, n_in, n_out):
        hidden = [int(h) for h in (p.get("NumHiddenNodes") or [50])][: int(_num(p.get("NumHiddenLayers"), 1))]
        acts = list(p.get("ActivationFunc") or ["tanh"])
        out_act = p.get("OutputActivationFunc") or ("linear" if self.mc.is_linear_target() else "sigmoid")
        return MLPSpec(n_in, hidden, acts, n_out, out_act, str(p.get("Loss", "squared")))

    def _train_nn(self, tid, p, ts, y, train_m, valid_m, sw, ova_class):
        mc, ms = self.mc, self.ms
        X, vX = ts.X, ts.vX
        # NN feature subsampling per bag (TrainModelProcessor :880-900 -> shifu.nn.feature.subset)
        self._nn_subset = None
        from ..models.gbdt import _strategy_count
        k = _strategy_count(p.get("FeatureSubsetStrategy", "ALL"), X.shape[1], X.shape[1], 1)
        if 0 < k < X.shape[1]:
            cols = np.sort(np.random.default_rng(7 + tid).choice(X.shape[1], k, replace=False))
            X = np.asarray(X)[:, cols]
            vX = None if vX is None else np.asarray(vX)[:, cols]
            self._nn_subset = cols
        n_in = X.shape[1]
        multi = mc.is_multiclass() and ova_class is None
        n_out = len(mc.tags()) if multi else 1
        spec = self._nn_spec(p, n_in, n_out)
        epochs = int(mc.train.get("numTrainEpochs", 100))
        init = None
        grow = None
        cont = bool(mc.train.get("isContinuous", False))
        mpath = ms.pf.model_path(tid, "nn")
        if cont and os.path.exists(mpath):
            net = nn_format.read_encog(mpath)
            sizes = [n_in] + spec.hidden + [n_out]
            if net.sizes == sizes:
                init = net.flat()["weights"]
                _log.info("continuous training from %s", mpath)
            elif can_grow(net.sizes, sizes):
                grow = net               # NNMaster.fitExistingModelIn: the old net inside the new one
                _log.info("continuous training from %s: existing %s grown into %s", mpath, net.sizes, sizes)
            else:
                _log.warning("!!! Model training parameters like hidden nodes, activation and others are not "
                             "consistent with settings, model training will start from scratch.")
        tr = MLPTrainer(spec, self.dev, str(p.get("Propagation", "R")), float(_num(p.get("LearningRate"), 0.1)),
                        momentum=float(_num(p.get("Momentum"), 0.5)),
                        adam_beta1=float(_num(p.get("AdamBeta1"), 0.9)),
                        adam_beta2=float(_num(p.get("AdamBeta2"), 0.999)),
                        learning_decay=float(_num(p.get("LearningDecay"), 0.0)),
                        reg=float(_num(p.get("RegularizedConstant"), 0.0)), reg_level=p.get("L1orL2", "NONE"),
                        seed=1000 + tid, weight_init=p.get("WeightInitializer", "default"),
                        # FixedLayers / FixedBias act only when training continues from an existing
                        # model (NNMaster.initOrRecoverParams :340-352): whole layers for the same
                        # structure, the copied block for a grown one (grow_weights below)
                        init_flat_encog=init, fixed_layers=p.get("FixedLayers") if init is not None else None,
                        dropout_rate=float(_num(p.get("DropoutRate"), 0.0)),
                        fixed_bias=False)
        if grow is not None:
            nfix = grow_weights(tr, grow.weights, p.get("FixedLayers"),
                                fixed_bias=str(p.get("FixedBias", "true")).lower() == "true")
            _log.info("fitExistingModelIn: %d weights frozen", nfix)
        yy = y
        if multi:
            yy = np.eye(n_out, dtype=np.float32)[np.clip(np.rint(y).astype(int), 0, n_out - 1)]
        yy = yy.reshape(len(y), -1)
        w = np.asarray(ts.w, dtype=np.float32) * sw
        tri = np.nonzero(train_m)[0]
        from ..data.rowstore import Bf16Rows

        def rows_of(A, idx):
            # bf16 NormalizedData goes to HBM as its bf16 bits (rows / columns gathered on the
            # device); anything else as fp32 host rows
            if isinstance(A, Bf16Rows) and tr.gpu:
                return A.device_rows(tr.device, rows=idx)
            return torch.from_numpy(np.asarray(A[idx] if idx is not None else A, dtype=np.float32))
        split_dev = (vX is None and valid_m.any() and isinstance(X, Bf16Rows) and tr.gpu)
        if split_dev:                 # training and validation rows from ONE read of the cache
            Xt, Xv = X.device_rows_multi(tr.device, [tri, np.nonzero(valid_m)[0]])
        else:
            Xt = rows_of(X, tri)
        data = tr.prepare(Xt, yy[tri], w[tri])
        vdata = None
        if vX is not None:
            vy = np.asarray(ts.vy, np.float32)
            if ova_class is not None:
                vy = (np.rint(vy) == ova_class).astype(np.float32)
            if multi:
                vy = np.eye(n_out, dtype=np.float32)[np.clip(np.rint(vy).astype(int), 0, n_out - 1)]
            vdata = tr.prepare(rows_of(vX, None), vy.reshape(len(vy), -1), np.asarray(ts.vw, np.float32))
        elif valid_m.any():
            vi = np.nonzero(valid_m)[0]
            vdata = tr.prepare(Xv if split_dev else rows_of(X, vi), yy[vi], np.asarray(ts.w)[vi])
        n_train = torch.tensor([float(len(tri))], dtype=torch.float64, device=tr.device)
        dist.all_reduce_(n_train)
        n_train = float(n_train.item())
        es = EarlyStop(str(p.get("EnableEarlyStop", "false")).lower() == "true",
                       int(os.environ.get("SHIFU_EARLYSTOP_WINDOW", 20)),
                       float(_num(p.get("ValidationTolerance"), 0.0)),
                       float(_num(mc.train.get("convergenceThreshold"), 0.0)))
        ckpt = os.path.join(ms.pf.checkpoint_dir, f"nn_trainer{tid}.pt")
        start = 0
        best_v, best_w = math.inf, None
        if self.resume and os.path.exists(ckpt):
            st = torch.load(ckpt, weights_only=True)
            if st.get("spec_sizes") == [n_in] + spec.hidden + [n_out]:
                _check_split_scheme(st, f"trainer {tid}")
                tr.load_state_dict(st)
                start = int(st["epoch"])
                best_v = float(st.get("best_v", math.inf))
                best_w = st["best_w"].to(tr.device) if st.get("best_w") is not None else None
                _log.info("resumed trainer %d from checkpoint at epoch %d", tid, start)
        factor = checkpoint_interval(p, max(epochs // 25, 20))
        verr = float("nan")
        # MiniBatchs=k: iteration i trains on slice (i-1) mod k of the rows (SubGradient :326-340)
        mb = max(1, min(1000, int(_num(p.get("MiniBatchs"), 1))))
        with IterationWatchdog(iteration_limit(3600.0), "NN epoch") as wd:
            tr.comm_events = []                    # (start, end) of each gradient all-reduce -> allreduce_ms
            for ep in range(start + 1, epochs + 1):
                wd.tick()
                t_ep = time.perf_counter()
                with trace_range(f"nn.epoch{ep}"):
                    if mb > 1:
                        b = (ep - 1) % mb
                        lo, hi = data.n * b // mb, data.n * (b + 1) // mb
                        terr = tr.step(data, lo, hi)
                        rows_ep = n_train / mb
                    else:
                        terr = tr.step(data, num_train_global=n_train)
                        rows_ep = n_train
                    t_train = time.perf_counter() - t_ep     # step() ends with a host read of the error
                    verr = tr.evaluate(vdata) if vdata is not None else float("nan")
                check_finite("training error", terr, ep)
                if not math.isnan(verr) and verr < best_v:
                    best_v, best_w = verr, tr.params.flat.detach().clone()
                self._log_epoch(tid, ep, terr, verr, extra=self._epoch_extra(tr, rows_ep, t_train))
                if self.info.rank == 0 and ep % factor == 0 and ep < epochs:
                    self._write_nn(tid, spec, tr, tmp_epoch=ep)
                    os.makedirs(ms.pf.checkpoint_dir, exist_ok=True)
                    sd = tr.state_dict()
                    sd.update(epoch=ep, spec_sizes=[n_in] + spec.hidden + [n_out], best_v=best_v, split_scheme=SPLIT_SCHEME,
                              best_w=None if best_w is None else best_w.cpu())
                    sd.pop("spec", None)
                    torch.save(sd, ckpt)
                maybe_fault(ep, self.info.rank)
                if es.update(ep, terr, verr):
                    _log.info("trainer %d early stop at epoch %d", tid, ep)
                    break
        if best_w is not None and vdata is not None:
            tr.params.flat.copy_(best_w)      # NNOutput keeps the weights of the min validation error
            verr = best_v
        if self.info.rank == 0:
            self._write_nn(tid, spec, tr)
            if os.path.exists(ckpt):
                os.remove(ckpt)
        return verr

    def _nn_network(self, spec, tr) -> nn_format.NNNetwork:
        ws = tr.params.views()
        weights = [ws[l][:, : spec.layer_in[l] + 1].detach().double().cpu().numpy() for l in range(len(ws))]
        net = nn_format.NNNetwork([spec.n_in] + spec.hidden + [spec.n_out], spec.acts + [spec.out_act], weights)
        sub = getattr(self, "_nn_subset", None)
        if sub is not None:            # input positions of the bag's feature subset
            net.feature_set = [int(i) for i in sub]
            net.properties = {nn_format.SUBSET_PROP: ",".join(str(int(i)) for i in sub)}
        return net

    def _write_nn(self, tid, spec, tr, tmp_epoch=None):
        ms = self.ms
        net = self._nn_network(spec, tr)
        if tmp_epoch is not None:
            nn_format.write_encog(net, ms.pf.ensure(ms.pf.tmp_model_path(tid, tmp_epoch, "nn")))
            return
        nn_format.write_encog(net, ms.pf.model_path(tid, "nn"))
        cols = ms.input_columns()
        nn_format.write_binary_nn(os.path.join(ms.pf.bmodels_dir, f"model{tid}.nn"), self.mc.norm_type,
                                  nn_column_stats(self.mc, cols), {c.num: i for i, c in enumerate(cols)}, [net])

    # -- LR ---------------------------------------------------------------------------------
    def _train_lr(self, tid, p, ts, y, train_m, valid_m, sw):
        mc, ms = self.mc, self.ms
        X = ts.X
        tr = lrmod.LRTrainer(X.shape[1], self.dev, str(p.get("Propagation", "R")),
                             float(_num(p.get("LearningRate"), 0.1)), float(_num(p.get("RegularizedConstant"), 0.0)),
                             p.get("L1orL2", "NONE"), float(_num(p.get("LearningDecay"), 0.0)), seed=tid)
        cont = bool(mc.train.get("isContinuous", False))
        mpath = ms.pf.model_path(tid, "lr")
        if cont and os.path.exists(mpath):
            w0 = lrmod.read_lr(mpath)
            if len(w0) == X.shape[1] + 1:
                tr.w.copy_(torch.from_numpy(w0.astype(np.float32)))
        w = np.asarray(ts.w, np.float32) * sw
        tri = np.nonzero(train_m)[0]
        data = tr.prepare(np.asarray(X[tri], np.float32), y[tri], w[tri])
        vdata = None
        if ts.vX is not None:
            vdata = tr.prepare(np.asarray(ts.vX, np.float32), np.asarray(ts.vy, np.float32), None)
        elif valid_m.any():
            vi = np.nonzero(valid_m)[0]
            vdata = tr.prepare(np.asarray(X[vi], np.float32), y[vi], None)
        epochs = int(mc.train.get("numTrainEpochs", 100))
        es = EarlyStop(str(p.get("EnableEarlyStop", "false")).lower() == "true", 20,
                       float(_num(p.get("ValidationTolerance"), 0.0)),
                       float(_num(mc.train.get("convergenceThreshold"), 0.0)))
        verr = float("nan")
        for ep in range(1, epochs + 1):
            terr = tr.step(data)
            verr = tr.evaluate(vdata) if vdata is not None else float("nan")
            self._log_epoch(tid, ep, terr, verr)
            if es.update(ep, terr, verr):
                break
        if self.info.rank == 0:
            lrmod.write_lr(mpath, tr.weights())
        return verr

    # -- SVM (legacy LOCAL, SVMTrainer.java:38-185) -----------------------------------------
    def _train_svm(self, tid, p, ts, y, train_m, valid_m, sw):
        """One C-SVC per bag on this process (the reference trains SVM locally only); rank 0 trains
        and writes ``models/model<i>.svm``, the other ranks wait."""
        from ..config import environment
        from ..models import svm as S
        mc, ms = self.mc, self.ms
        verr = float("nan")
        if self.info.rank == 0:
            with dist.local_only():
                X = np.asarray(ts.X, np.float32)
                tri = np.nonzero(train_m & (sw > 0))[0]
                cap = int(environment.get("shifu.svm.maxRows", 65536))
                if len(tri) > cap:
                    _log.warning("SVM: %d training rows > shifu.svm.maxRows=%d, training on a random subset",
                                 len(tri), cap)
                    tri = np.sort(np.random.default_rng(tid).choice(tri, cap, replace=False))
                kern = S.kernel_name(p.get("Kernel", "linear"))
                m = S.train_svm(X[tri], y[tri], kern, float(_num(p.get("Const"), 1.0)),
                                float(_num(p.get("Gamma"), 1.0)), weights=sw[tri], device=self.dev,
                                log=lambda s: _log.info("trainer %d: %s", tid, s))
                if ts.vX is not None:
                    vx, vy = np.asarray(ts.vX, np.float32), np.asarray(ts.vy, np.float64)
                else:
                    vi = np.nonzero(valid_m)[0]
                    vx, vy = X[vi], y[vi].astype(np.float64)
                if len(vy):
                    verr = float(np.mean(m.predict(vx, self.dev) != vy))
                tri_err = float(np.mean(m.predict(X[tri], self.dev) != y[tri])) if len(tri) else float("nan")
                self._log_epoch(tid, 1, tri_err, verr)
                S.write_svm(ms.pf.model_path(tid, "svm"), m, X.shape[1])
                _log.info("Trainer #%d finish training: train error %.6f validation error %.6f (%s kernel)",
                          tid, tri_err, verr, kern)
        dist.barrier()
        return verr

    # -- WDL --------------------------------------------------------------------------------
    def _train_wdl(self, tid, p, ts, y, train_m, valid_m, sw):
        from ..models.wdl import train_wdl_step
        return train_wdl_step(self, tid, p, ts, y, train_m, valid_m, sw)

    # -- trees -------------------------------------------------------------------------------
    def _train_tree(self, tid, p, ts, y, train_m, valid_m, sw):
        from ..models.gbdt import BinnedData, TreeConfig, TreeTrainer
        mc, ms = self.mc, self.ms
        alg = mc.algorithm
        meta = ts.meta
        nb = np.asarray(meta["nbins"], np.int32)
        is_cat = np.asarray(meta["is_cat"], np.uint8)
        codes = ts.codes
        w = np.asarray(ts.w, np.float32)
        tri = np.nonzero(train_m)[0]
        dev = self.dev
        # uint8 codes go to the device one 32-feature group at a time (no host int32 staging)
        codes_np = codes if isinstance(codes, np.ndarray) else np.asarray(codes)
        all_rows = len(tri) == codes_np.shape[0]
        with trace_range("train.upload_bins"):
            if self._host_bins(len(tri), codes_np.shape[1]):
                _log.info("tree bins stay in pinned host memory (%d rows x %d features)", len(tri), codes_np.shape[1])
                d = BinnedData.host_resident(codes_np, y[tri], nb, is_cat, w[tri], device=dev,
                                             rows=None if all_rows else tri)
            else:
                d = BinnedData.from_codes(codes_np, y[tri], nb, is_cat, w[tri], device=dev,
                                          rows=None if all_rows else tri)
            vd = None
            if ts.vcodes is not None:
                vd = BinnedData.from_codes(np.asarray(ts.vcodes), np.asarray(ts.vy, np.float32), nb, is_cat,
                                           np.asarray(ts.vw, np.float32), device=dev)
            elif valid_m.any():
                vi = np.nonzero(valid_m)[0]
                vd = BinnedData.from_codes(codes_np, y[vi], nb, is_cat, w[vi], device=dev, rows=vi)
        tree_num = int(_num(p.get("TreeNum"), 100))
        cfg = TreeConfig(alg, tree_num=tree_num, max_depth=int(_num(p.get("MaxDepth"), 7 if alg == "GBT" else 10)),
                         min_instances_per_node=int(_num(p.get("MinInstancesPerNode"), 5)),
                         min_info_gain=float(_num(p.get("MinInfoGain"), 0.0)),
                         impurity=str(p.get("Impurity", "variance")), loss=str(p.get("Loss", "squared")),
                         learning_rate=float(_num(p.get("LearningRate"), 0.05)),
                         feature_subset_strategy=p.get("FeatureSubsetStrategy", "TWOTHIRDS"),
                         bagging_sample_rate=float(mc.train.get("baggingSampleRate", 1.0)),
                         sample_with_replacement=bool(p.get("GBTSampleWithReplacement", False)) if alg == "GBT"
                         else bool(mc.train.get("baggingWithReplacement", True)),
                         dropout_rate=float(_num(p.get("DropoutRate"), 0.0)), seed=tid,
                         max_leaves=int(_num(p.get("MaxLeaves"), 0)),
                         max_batch_split=int(_num(p.get("MaxBatchSplitSize"), 0)),
                         max_stats_memory_mb=int(_num(p.get("MaxStatsMemoryMB"), 0)),
                         valid_tolerance=float(_num(p.get("ValidationTolerance"), 0.0)),
                         early_stop=str(p.get("EnableEarlyStop", "false")).lower() == "true",
                         n_classes=len(mc.tags()) if (mc.is_multiclass() and not mc.is_one_vs_all()) else 0)
        tt = TreeTrainer(cfg, d, vd)
        es = EarlyStop(cfg.early_stop, int(os.environ.get("SHIFU_EARLYSTOP_WINDOW", 20)), cfg.valid_tolerance)
        stop = [False]

        def cb(i, tree, terr, verr):
            st = tt.last_tree_stats or {}
            lv = st.get("levels") or []
            if lv:          # DTWorker-style phase line (DTWorker.java:581-687, 858-884)
                _log.debug("tree %d: %.1f ms, hist rows %d, hist allreduce %.2f ms, levels %s", i + 1,
                           st.get("ms", 0.0), st.get("hist_rows", 0), st.get("allreduce_ms", 0.0),
                           " ".join(f"L{e['level']}:{e['hist_rows']}r/{e['hist_split_ms']:.1f}"
                                    f"+{e.get('partition_ms', 0.0):.1f}ms" for e in lv))
            self._log_epoch(tid, i + 1, terr, verr,
                            extra={"tree_ms": round(st.get("ms", 0.0), 3), "hist_rows": st.get("hist_rows", 0),
                                   "allreduce_ms": round(st.get("allreduce_ms", 0.0), 3),
                                   "levels": [{k: (round(v, 3) if isinstance(v, float) else v) for k, v in e.items()}
                                              for e in lv]})
            if es.update(i + 1, terr, verr):
                stop[0] = True
        ckpt = os.path.join(ms.pf.checkpoint_dir, f"tree_trainer{tid}.pt")
        if self.resume and os.path.exists(ckpt):
            st = torch.load(ckpt, weights_only=True)
            _check_split_scheme(st, f"trainer {tid}")
            st.pop("split_scheme", None)
            tt.load_state_dict(st)
            _log.info("resumed trainer %d from checkpoint with %d trees", tid, len(tt.trees))
        else:
            existing = self._continuous_trees(tid, cfg)
            if existing == -1:
                return float("nan")
            if existing:
                tt.continue_from(existing)
        interval = checkpoint_interval(p, max(1, tree_num // 10))   # DTOutput: tmp models every treeNum/10
        with IterationWatchdog(iteration_limit(800.0), "tree") as wd:
            while len(tt.trees) < tree_num:
                wd.tick()
                with trace_range(f"gbdt.tree{len(tt.trees) + 1}"):
                    tt.train(1, callback=cb)
                n = len(tt.trees)
                check_finite("training error", tt.train_errors[-1], n)
                if self.info.rank == 0 and n % interval == 0 and n < tree_num:
                    os.makedirs(ms.pf.checkpoint_dir, exist_ok=True)
                    torch.save({**tt.state_dict(), "split_scheme": SPLIT_SCHEME}, ckpt)
                maybe_fault(n, self.info.rank)
                if stop[0]:
                    break
        if self.info.rank == 0:
            with trace_range("train.write_model"):
                self._write_trees(tid, tt)
            if os.path.exists(ckpt):
                os.remove(ckpt)
        return tt.valid_errors[-1] if tt.valid_errors else float("nan")

    def _host_bins(self, n_rows: int, n_feat: int) -> bool:
        """Out-of-core trees: ``shifu.train.tree.hostBins`` = true / false / auto
        (default: when the blocked uint8 bins would take more than 60 % of the GPU's free memory,
        they stay in pinned host memory and the kernels read them over the host link)."""
        from ..config import environment
        if self.dev.type != "cuda":
            return False
        mode = str(environment.get("shifu.train.tree.hostBins", "auto")).lower()
        if mode in ("true", "1", "on"):
            return True
        if mode in ("false", "0", "off"):
            return False
        need = n_rows * (-(-n_feat // 32) * 32)
        from ..utils.device import free_hbm
        free = free_hbm(self.dev)
        return need > 0.6 * free

    def _continuous_trees(self, tid, cfg):
        """``checkContinuousTraining`` (TrainModelProcessor.java:1149-1197) for trees: GBT only, the
        existing model must be GBT with the same loss and fewer than TreeNum trees.  Returns the
        existing trees as heap trees, [] (train from scratch) or -1 (already >= TreeNum trees:
        this trainer is skipped, as the reference skips it)."""
        mc, ms = self.mc, self.ms
        if not bool(mc.train.get("isContinuous", False)):
            return []
        path = ms.pf.model_path(tid, mc.algorithm.lower())
        if not os.path.exists(path):
            _log.info("No existing model, model training will start from scratch.")
            return []
        if not cfg.is_gbt:
            _log.warning("RF doesn't support continuous training")
            return []
        m = tree_format.read_tree_model(path)
        if m.algorithm.upper() != "GBT":
            _log.warning("Only GBT supports continuous training, while not GBT, will start from scratch")
            return []
        if m.loss.lower() != cfg.loss.lower():
            _log.warning("Loss is changed, continuous training is disabled, will start from scratch")
            return []
        recs = [t for bag in m.bags for t in bag]
        if not recs:
            return []
        if len(recs) >= cfg.tree_num:
            _log.warning("Model with index %d with size of trees is over treeNum, such training will not be "
                         "started.", tid)
            return -1
        cols = [c for c in ms.input_columns()]
        trees = [tree_format.record_to_heap_tree(r, cols) for r in recs]
        _log.info("continuous training of trainer %d from %s with %d existing trees", tid, path, len(trees))
        return trees

    def _write_trees(self, tid, tt):
        ms, mc = self.ms, self.mc
        cols = [c for c in ms.input_columns()]
        recs = [tree_format.heap_tree_to_record(t, i, cols, learning_rate=t.weight,
                                                is_classification=False) for i, t in enumerate(tt.trees)]
        m = tree_format.TreeModelFile(
            algorithm=mc.algorithm, loss=tt.cfg.loss, is_classification=mc.is_multiclass(),
            is_one_vs_all=mc.is_one_vs_all(), input_count=len(cols),
            numerical_means={c.num: float(c.mean or 0.0) for c in cols if not c.is_categorical()},
            names={c.num: c.name for c in cols},
            categories={c.num: list(c.bin_category or []) for c in cols if c.is_categorical()},
            column_mapping={c.num: i for i, c in enumerate(cols)}, bags=[recs])
        tree_format.write_tree_model(ms.pf.model_path(tid, mc.algorithm.lower()), m)
        fi = tree_format.feature_importance(m)
        with open(ms.pf.feature_importance + f".{tid}", "w") as f:
            for k, v in fi.items():
                f.write(f"{k}\t{m.names.get(k, k)}\t{v}\n")


def nn_column_stats(mc, cols):
    from ..algos.normalize import woe_mean_std
    out = []
    cutoff = float(mc.normalize.get("stdDevCutOff", 6.0))
    for c in cols:
        try:
            wm, ws = woe_mean_std(c, False)
            wwm, wws = woe_mean_std(c, True)
        except Exception:
            wm = ws = wwm = wws = 0.0
        out.append(nn_format.NNColumnStats(
            c.num, c.name, c.type or "N", cutoff, c.mean or 0.0, c.std_dev or 0.0, float(wm), float(ws), float(wwm),
            float(wws), list(c.bin_boundary or []), list(c.bin_category or []), list(c.bin_pos_rate or []),
            list(c.bin_count_woe or []), list(c.bin_weighted_woe or [])))
    return out


def run_train(root: str = ".", dry: bool = False, device=None) -> int:
    return TrainStep(ModelSet(root), dry=dry, device=device).process()
