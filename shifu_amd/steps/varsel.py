"""``varsel`` step (B6): filter KS/IV/mix/pareto, SE/ST sensitivity (``-r N`` recursive), FI for
trees, voted GA wrapper, auto-filter with history, ``-reset/-list/-autofilter/-recoverauto``.

``VarSelectModelProcessor.run`` (J/core/processor/VarSelectModelProcessor.java:121-281):
* binary targets: ``filterBy`` in KS/IV/MIX/PARETO -> ``VariableSelector.selectByFilter``; FI ->
  tree feature importance; SE/ST -> ``distributedSEWrapper`` (:633-674: train an NN on the
  candidates, then ``VarSelectMapper`` sensitivity + ``VarSelectReducer`` top-by-RMS keeping
  ``filterNum`` or ``inputs*(1-filterOutRatio)``); V (voted) -> ``votedVariablesSelection``
  (:403-438, GA over subsets scored by small NN validation error).
* multi-class: force-selected (if any) else every good candidate.
* then ``autoVarSelCondition`` (:1008-1050) + correlation filter; changes are appended to
  ``varsel/varsel.history`` so ``-recoverauto`` can undo them.
"""
from __future__ import annotations

import os
import time

import numpy as np
import torch

from ..algos import normalize as N
from ..algos import varsel as V
from ..config.column_config import has_candidates
from ..formats.nn_format import NNNetwork
from ..models.nn import MLPSpec, MLPTrainer
from ..utils.log import get_logger
from ..utils.trace import trace_range
from ..parallel import dist
from .base import ModelSet, _writer, shard_model_data

_log = get_logger("steps.varsel")


def _good(ms):
    hc = has_candidates(ms.ccs)
    return [c for c in ms.ccs if c.is_good_candidate(hc, ms.mc.is_binary()) or c.is_force_select()]


def _history_append(ms, changes, reason):
    if not _writer():
        return
    os.makedirs(ms.pf.varsel_dir, exist_ok=True)
    with open(ms.pf.varsel_history, "a") as f:
        for c, old, new in changes:
            f.write(f"{c.num},{c.name},{str(old).lower()},{str(new).lower()},{reason}\n")


def _normalized_rows(ms, cols, device=None):
    """This rank's (X fp32 [n, len(cols)], y, w) from the norm step's NormalizedData when it holds
    exactly the candidate columns (the usual init -> stats -> norm -> varsel order); None otherwise.
    The reference's SE job reads the normalized training data too (VarSelectMapper); reading it
    here avoids a second parse + normalisation of the raw text."""
    from .base import load_dataset_cache
    from .train import _shard
    t0 = time.perf_counter()
    cache = load_dataset_cache(ms.pf.normalized_data)
    if cache is None:
        return None
    meta, arr = cache
    t_open = time.perf_counter() - t0
    if meta.get("input_nums") != [c.num for c in cols] or "X" not in arr or "y" not in arr:
        return None
    info = dist.info()
    from ..data.rowstore import Bf16Rows
    from ..utils.device import default_device
    dev = torch.device(device) if device is not None else default_device()
    if isinstance(arr["X"], Bf16Rows) and dev.type == "cuda":
        # bf16 cache on a GPU: the rank's rows go to HBM as bf16 bits (no host fp32 expansion)
        n = len(arr["X"])
        lo, hi = n * info.rank // info.world_size, n * (info.rank + 1) // info.world_size
        X = arr["X"].device_rows(dev, rows=np.arange(lo, hi) if (lo, hi) != (0, n) else None)
    else:
        X = np.asarray(_shard(arr["X"], info), dtype=np.float32)
    y = np.asarray(_shard(arr["y"], info), dtype=np.float32).reshape(len(X), -1)[:, :1]
    w = np.asarray(_shard(arr["w"], info), dtype=np.float32) if "w" in arr else np.ones(len(X), np.float32)
    _log.info("varsel: sensitivity rows from NormalizedData (%d x %d): open %.2fs, rows %.2fs %s", X.shape[0],
              X.shape[1], t_open, time.perf_counter() - t0 - t_open,
              {k: round(v, 2) for k, v in Bf16Rows.LAST_STATS.items()} if isinstance(arr["X"], Bf16Rows) else "")
    return X, y, w


def _train_quick_nn(ms, cols, epochs, device=None, seed=0, rows=None):
    """Train the NN used for sensitivity analysis on the candidate columns; returns (net, X, md).
    ``rows``: (X, y, w) already normalized (``_normalized_rows``); else the raw data is loaded
    and normalized here."""
    mc = ms.mc
    md = None
    if rows is not None:
        X, y, w = rows
    else:
        md = shard_model_data(ms.load_raw(cols))     # data parallel: each rank its row range
        X, _, _ = N.normalize_table(mc, ms.ccs, md.table, columns=cols)
        y, w = md.y.reshape(-1, 1), md.w.astype(np.float32)
    p = mc.train.get("params") or {}
    hidden = [int(h) for h in (p.get("NumHiddenNodes") or [50])][: int(p.get("NumHiddenLayers", 1) or 1)]
    spec = MLPSpec(X.shape[1], hidden, list(p.get("ActivationFunc") or ["tanh"]), 1, "sigmoid")
    from ..utils.device import default_device
    dev = torch.device(device) if device is not None else default_device()
    tr = MLPTrainer(spec, dev, str(p.get("Propagation", "R")), float(p.get("LearningRate", 0.1)), seed=seed)
    data = tr.prepare(X if torch.is_tensor(X) else torch.from_numpy(np.ascontiguousarray(X, dtype=np.float32)), y, w)
    for _ in range(max(1, epochs)):
        tr.step(data)
    ws = tr.params.views()
    net = NNNetwork([spec.n_in] + spec.hidden + [1], spec.acts + ["sigmoid"],
                    [ws[l][:, : spec.layer_in[l] + 1].detach().double().cpu().numpy() for l in range(len(ws))])
    return net, X, md


def _reusable_se_model(ms, cols):
    """``shifu.varsel.se.reuse=true`` (VarSelectModelProcessor.distributedSEWrapper :633-642): skip
    training and analyse the current ``models/model0.nn`` when it was trained on these candidates
    (same input width); otherwise None (train the sensitivity model)."""
    from ..config import environment
    if not environment.get_bool("shifu.varsel.se.reuse", False):
        return None
    from ..formats.nn_format import read_encog
    path = ms.pf.model_path(0, "nn")
    if not os.path.exists(path):
        _log.warning("shifu.varsel.se.reuse: %s not found, training the SE model", path)
        return None
    net = read_encog(path)
    if net.n_in != len(cols) or net.n_out != 1:
        _log.warning("shifu.varsel.se.reuse: %s has %d inputs for %d candidates, training the SE model",
                     path, net.n_in, len(cols))
        return None
    _log.info("shifu.varsel.se.reuse: sensitivity of the existing %s", path)
    return net


PHASES: dict = {}          # last SE run: load / training / sensitivity seconds (bench.py pipeline)


def _sync(device):
    if torch.cuda.is_available() and (device is None or torch.device(device).type == "cuda"):
        torch.cuda.synchronize()


def select_by_sensitivity(ms, by="SE", device=None, seed=0):
    mc = ms.mc
    cols = _good(ms)
    if not cols:
        return []
    epochs = max(1, int(mc.train.get("numTrainEpochs", 100)) // 2)
    t0 = time.perf_counter()
    net = _reusable_se_model(ms, cols)
    trained = net is None
    with trace_range("varsel.load_rows"):
        rows = _normalized_rows(ms, cols, device)
    t1 = time.perf_counter()
    if net is not None:
        if rows is not None:
            X = rows[0]
        else:
            md = shard_model_data(ms.load_raw(cols))
            X, _, _ = N.normalize_table(mc, ms.ccs, md.table, columns=cols)
    else:
        with trace_range("varsel.se_train"):
            net, X, md = _train_quick_nn(ms, cols, epochs, device, seed, rows=rows)
    _sync(device)
    t2 = time.perf_counter()
    with trace_range("varsel.sensitivity"):
        mean, rms, var = V.sensitivity(net, X, device=device)
    _sync(device)
    t3 = time.perf_counter()
    # phase split of the SE job (the reference's 70 min = 45 min of training + 25 min of sensitivity)
    PHASES.update(load_s=t1 - t0, train_s=t2 - t1, train_epochs=epochs if trained else 0, sensitivity_s=t3 - t2)
    _log.info("varsel SE phases: rows %.2fs, training %.2fs (%d epochs), sensitivity %.2fs",
              t1 - t0, t2 - t1, epochs, t3 - t2)
    filter_num = int(mc.varSelect.get("filterNum", 200) or 0)
    keep = filter_num if filter_num > 0 else int(len(cols) * (1 - float(mc.varSelect.get("filterOutRatio", 0.05))))
    order = np.argsort(-rms, kind="stable")          # VarSelectReducer sorts by RMS for SE and ST
    keep_nums = {cols[i].num for i in order[:keep]}
    for c in ms.ccs:
        c.final_select = (c.num in keep_nums) or c.is_force_select()
    return [(cols[i].num, cols[i].name, float(mean[i]), float(rms[i]), float(var[i])) for i in order]


def select_by_fi(ms, device=None):
    from ..models.gbdt import BinnedData, TreeConfig, TreeTrainer
    from ..formats.tree_format import heap_tree_to_record
    mc = ms.mc
    cols = _good(ms)
    md = shard_model_data(ms.load_raw(cols))     # histograms all-reduced inside TreeTrainer
    C, nb, is_cat = N.tree_bin_codes(ms.ccs, md.table, cols)
    from ..utils.device import default_device
    dev = torch.device(device) if device is not None else default_device()
    d = BinnedData.from_codes(torch.from_numpy(C), md.y, nb, is_cat, md.w.astype(np.float32), device=dev)
    p = mc.train.get("params") or {}
    cfg = TreeConfig(mc.algorithm if mc.algorithm in ("GBT", "RF") else "GBT",
                     tree_num=min(int(float(p.get("TreeNum", 50))), 50), max_depth=int(p.get("MaxDepth", 6)),
                     learning_rate=float(p.get("LearningRate", 0.05)), feature_subset_strategy="ALL")
    tt = TreeTrainer(cfg, d)
    tt.train()
    imp = np.zeros(len(cols))
    for t in tt.trees:
        for nid in np.nonzero(t.exists)[0]:
            f = int(t.feat[nid])
            if f >= 0:
                imp[f] += float(t.gain[nid]) * float(t.wgt_cnt[nid])
    filter_num = int(mc.varSelect.get("filterNum", 200) or 0) or len(cols)
    order = np.argsort(-imp, kind="stable")
    keep = {cols[i].num for i in order[:filter_num] if imp[i] > 0}
    for c in ms.ccs:
        c.final_select = (c.num in keep) or c.is_force_select()
    return [(cols[i].name, float(imp[i])) for i in order]


def voted_selection(ms, device=None, seed: int = 0):
    """``filterBy V``: genetic wrapper (``algos/ga_varsel.py``; WrapperMasterConductor +
    CandidateGenerator + ValidationConductor) with the population trained as one batched GEMM."""
    from ..algos.ga_varsel import voted_selection as ga
    from ..parallel import dist
    mc = ms.mc
    cols = _good(ms)
    md = ms.load_raw(cols)
    X, _, nums = N.normalize_table(mc, ms.ccs, md.table, columns=cols)
    info = dist.info()
    lo, hi = md.n * info.rank // info.world_size, md.n * (info.rank + 1) // info.world_size
    from ..utils.device import default_device
    dev = torch.device(device) if device is not None else default_device()
    params = dict(mc.varSelect.get("params") or {})
    nn_params = dict(mc.train.get("params") or {})
    epochs = int(mc.train.get("numTrainEpochs", 100) or 100)
    best, hist = ga(X[lo:hi], md.y[lo:hi], md.w[lo:hi], cols, params, nn_params, epochs,
                    float(mc.train.get("validSetRate", 0.2) or 0.2), seed, dev,
                    log=lambda it, e: _log.info("voted varsel generation %d best validation error %.6f", it, e))
    chosen = {c.num for c in best}
    for c in ms.ccs:
        c.final_select = c.is_force_select() or c.num in chosen
    return [c.name for c in best]


def run_auto_filter(ms):
    before = {c.num: c.final_select for c in ms.ccs}
    corr, corr_nums = None, None
    thr = float(ms.mc.varSelect.get("correlationThreshold", 1.0) or 1.0)
    if thr < 1.0 and os.path.exists(ms.pf.correlation_csv):
        from .stats import read_correlation
        names, corr = read_correlation(ms.pf.correlation_csv)
        byname = {c.name: c.num for c in ms.ccs}
        corr_nums = [byname.get(nm, -1) for nm in names]
    removed = V.auto_filter(ms.mc, ms.ccs, corr, corr_nums)
    changes = [(c, before[c.num], c.final_select) for c in ms.ccs if before[c.num] != c.final_select]
    if changes:
        _history_append(ms, changes, "auto")
    _log.info("auto filter removed %d variables: %s", len(removed), removed[:20])
    return removed


def recover_auto(ms):
    if not os.path.exists(ms.pf.varsel_history):
        _log.warning("no varsel history")
        return 0
    byid = {c.num: c for c in ms.ccs}
    n = 0
    for line in open(ms.pf.varsel_history):
        parts = line.strip().split(",")
        if len(parts) < 5:
            continue
        c = byid.get(int(parts[0]))
        old, new = parts[2] == "true", parts[3] == "true"
        if c is not None and c.final_select == new:
            c.final_select = old
            n += 1
    dist.barrier()                      # every rank has read the history before rank 0 drops it
    if _writer():
        os.remove(ms.pf.varsel_history)
    return n


def run_varsel(root: str = ".", reset: bool = False, list_only: bool = False, autofilter: bool = False,
               recover: bool = False, recursive: int = 1, device=None) -> int:
    ms = ModelSet(root).setup("VARSELECT")
    mc = ms.mc
    if reset:
        for c in ms.ccs:
            c.final_select = False
    elif list_only:
        for c in ms.ccs:
            if c.final_select and _writer():
                print(c.name)
        return 0
    elif autofilter:
        run_auto_filter(ms)
    elif recover:
        _log.info("recovered %d variables", recover_auto(ms))
    else:
        if mc.is_binary():
            by = str(mc.varSelect.get("filterBy", "KS")).upper()
            if by in ("KS", "IV", "MIX", "PARETO"):
                V.select_by_filter(mc, ms.ccs)
            elif by == "FI":
                if mc.algorithm not in ("GBT", "RF"):
                    raise ValueError("Filter by FI only works with GBT/RF")
                select_by_fi(ms, device)
            elif by in ("SE", "ST"):
                if mc.algorithm not in ("NN", "LR"):
                    raise ValueError("Filter by SE/ST only works with NN/LR")
                os.makedirs(ms.pf.varsel_dir, exist_ok=True)
                for i in range(max(1, recursive)):
                    ms.save_cc()
                    if _writer():
                        import shutil
                        shutil.copyfile(ms.pf.column_config, ms.pf.varsel_cc_backup(i))
                    res = select_by_sensitivity(ms, by, device, seed=i)
                    if _writer():
                        with open(ms.pf.varsel_se(i), "w") as f:
                            for num, name, mean, rms, var in res:
                                f.write(f"{num}\t{name}\t{mean}\t{rms}\t{var}\n")
            elif by in ("V", "VOTED"):
                voted_selection(ms, device)
            else:
                raise ValueError(f"unknown filterBy {by}")
        else:
            forced = [c for c in ms.ccs if c.is_force_select()]
            hc = has_candidates(ms.ccs)
            for c in ms.ccs:
                c.final_select = c.is_force_select() if forced else c.is_good_candidate(hc, False)
        if bool(mc.varSelect.get("autoFilterEnable", True)):
            run_auto_filter(ms)
    ms.save_cc(backup=True)
    _log.info("varsel: %d variables selected", sum(1 for c in ms.ccs if c.final_select))
    return 0
