"""``stats`` step (B4): binning + column statistics, ``-c`` correlation, ``-p`` PSI, ``-rebin``.

``StatsModelProcessor.run`` (J/core/processor/StatsModelProcessor.java:116-251): one pass over the
purified (``stats.sampleRate``) data computes every column's bins and stats
(:func:`shifu_amd.algos.stats.compute_column_stats`); ``-c`` (``runCorrMapReduceJob`` :300,
``computeCorrValue`` :490) writes ``correlation.csv`` over the normalized candidate columns;
``-p`` runs PSI by ``stats.psiColumnName``; ``-rebin`` (``doReBin`` :670,
``ColumnConfigDynamicBinning`` J/core/binning/ColumnConfigDynamicBinning.java:27-180) merges
adjacent bins with the smallest IV loss down to ``-n`` bins (``-ivr`` keeps >= ratio of IV).
"""
from __future__ import annotations

import os

import numpy as np

from ..algos import normalize as N
from ..algos import stats as S
from ..algos.binning import rebin_categorical
from ..utils.log import get_logger
from .base import ModelSet

_log = get_logger("steps.stats")


def run_stats(root: str = ".", correlation: bool = False, psi: bool = False, rebin: bool = False,
              expected_bins: int | None = None, iv_keep_ratio: float = 1.0, bin_avg_score_only: bool = False,
              device=None, min_inst_cnt: float = 0, request_vars: list[str] | None = None) -> int:
    ms = ModelSet(root).setup("STATS")
    mc = ms.mc
    cols = ms.stats_columns()
    from ..parallel import dist
    if rebin and not correlation and dist.info().world_size > 1:
        # rebin (ColumnConfig only, no data pass): rank 0 alone; correlation and PSI are data
        # parallel (row-sharded sums / counts, one all-reduce each)
        if dist.info().rank == 0:
            with dist.local_only():
                return run_stats(root, correlation, psi, rebin, expected_bins, iv_keep_ratio,
                                 bin_avg_score_only, device, min_inst_cnt, request_vars)
        return 0
    if rebin:
        do_rebin(ms, expected_bins or 0, iv_keep_ratio, min_inst_cnt, request_vars)
        ms.save_cc()
        return 0
    if correlation:                     # `stats -c` only computes correlation (stats must exist)
        run_correlation(ms, device)
        return 0
    if not psi:
        from ..parallel import dist
        from ..utils.device import default_device
        with S.deferred_metrics(device if device is not None else default_device()):
            _stats_pass(ms, mc, cols, device)
        ms.save_cc(backup=True)
    if dist.info().world_size > 1:
        dist.barrier()
    if psi or mc.stats.get("psiColumnName"):
        unit = mc.stats.get("psiColumnName")
        if unit:
            from .base import shard_model_data
            cc_unit = [c for c in ms.ccs if c.name == unit]
            md = shard_model_data(ms.load_raw(cols + cc_unit))
            S.compute_psi(mc, ms.ccs, md, unit,
                          unit_stats_path=os.path.join(ms.pf.tmp_dir, "columnconfig.unitstats"))
            ms.save_cc()
        else:
            _log.warning("stats -p: stats.psiColumnName is empty")
    return 0


def _use_streaming(ms: ModelSet) -> bool:
    """``shifu.stats.streaming``: true / false / auto (default).  auto streams when the data set is
    larger than ``shifu.stats.streamThresholdGB`` (default 8) or the run is data parallel (every
    rank then parses only its own byte range instead of the whole data set)."""
    from ..config import environment
    from ..data.purifier import plan_dataset
    from ..data.stream import data_bytes
    from ..parallel import dist
    mode = str(environment.get("shifu.stats.streaming", "auto")).lower()
    if S.parity_algorithm(ms.mc):            # reference sketches consume whole columns in row order
        return False
    if mode in ("true", "1", "yes"):
        return True
    if mode in ("false", "0", "no"):
        return False
    if dist.info().world_size > 1:
        return True
    try:
        nbytes = data_bytes(plan_dataset(ms.mc, ms.mc.dataSet))
    except Exception:
        return False
    return nbytes > float(environment.get("shifu.stats.streamThresholdGB", 8)) * (1 << 30)



def _stats_pass(ms, mc, cols, device) -> None:
    from ..parallel import dist
    if _use_streaming(ms):
        _stats_streamed(ms, cols, device)
    else:
        md = ms.load_raw(cols, sample_rate=float(mc.stats.get("sampleRate", 1.0)),
                         sample_neg_only=bool(mc.stats.get("sampleNegOnly", False)))
        _log.info("stats: %d valid rows (%s)", md.n, md.counters.as_dict())
        if dist.info().world_size > 1:
            # data parallel over an in-memory table (shifu.stats.streaming=false)
            from ..algos.dist_stats import compute_column_stats_dp
            from .base import shard_model_data
            compute_column_stats_dp(mc, ms.ccs, shard_model_data(md), device=device,
                                    columns={c.name for c in cols})
        else:
            S.compute_column_stats(mc, ms.ccs, md, device=device, columns={c.name for c in cols})

def _parse_device(device):
    """The CUDA device (with its index) a streamed step computes on, or None on the CPU."""
    import torch
    from ..utils.device import is_gpu_available
    if device is None:
        if not is_gpu_available():
            return None
        device = "cuda"
    d = torch.device(device)
    if d.type != "cuda":
        return None
    return d if d.index is not None else torch.device("cuda", torch.cuda.current_device())


def _stats_streamed(ms: ModelSet, cols, device=None) -> None:
    """Stats over row chunks of this rank's byte range (algos/stats_stream.py)."""
    import torch
    from ..algos.stats_stream import compute_column_stats_streamed
    from ..config import environment
    from ..data import stream as DS
    from ..data.purifier import plan_dataset
    from ..parallel import dist
    mc = ms.mc
    info = dist.info()
    plan = plan_dataset(mc, mc.dataSet, [c.name for c in cols if not c.is_categorical()],
                        [c.name for c in cols if c.is_categorical()])
    rate = float(mc.stats.get("sampleRate", 1.0))
    neg_only = bool(mc.stats.get("sampleNegOnly", False))

    row0 = DS.rank_row_offset(plan, info.rank, info.world_size) if rate < 1.0 else 0
    multi = info.world_size > 1
    if multi and device is None:
        device = dist.coll_device()
    # the candidate numeric columns are parsed on the GPU and binned where they land (K0 -> K4)
    pdev = _parse_device(device)
    gpu_cols = [c.name for c in cols if not c.is_categorical() and not c.is_target() and not c.is_meta()]
    # 1 GB blocks on the GPU path: per-block fixed costs (parse syncs, per-batch K4/K1 launches)
    # over 4x fewer blocks (3M x 1600: stats 5.19 -> 4.60 s, profiles/r4/pipe_lab_3Mx1600_chunk1G_r4l.txt);
    # 2 GB since r5 (20M x 1600 with every parsed block resident: 11.9-12.8 -> 10.7-11.0 s)
    chunk = int(float(environment.get("shifu.stats.chunkMB", 2048 if pdev is not None else 256)) * (1 << 20))

    def chunks(resume=None, with_keys=False):
        return DS.iter_model_data(mc, plan, chunk, info.rank, info.world_size, rate, neg_only, row0=row0,
                                  resume=resume, with_keys=with_keys, gpu_cols=gpu_cols, dev=pdev)
    n = compute_column_stats_streamed(
        mc, ms.ccs, chunks, device=device, columns={c.name for c in cols},
        reduce=(lambda t, op: dist.all_reduce_(t, op)) if multi else None,
        allgather=dist.all_gather_cat if multi else None,
        gather_objects=dist.all_gather_objects if multi else None)
    _log.info("stats (streamed, %d MB chunks, rank %d/%d): %d valid rows", chunk >> 20, info.rank,
              info.world_size, n)


def run_correlation(ms: ModelSet, device=None, chunk_rows: int = 1 << 18):
    """Pairwise-complete Pearson over numeric raw values (categoricals via their pos-rate encoding),
    written as ``correlation.csv`` (header row + one row per column, ``ColumnConfig`` order).

    Rows stream through ``CorrAccumulator`` in ``chunk_rows`` chunks (only one chunk of fp64 values
    exists at a time); data parallel: row shards, sums reduce-scattered by column blocks, rows
    gathered to the writer.  ``shifu.stats.corr.reuse=true`` with a previous run's matrix for the
    same columns under ``tmp/CorrelationPath`` skips the data pass (StatsModelProcessor :140-146,
    dumpAndCalculateCorrelationResult)."""
    import json
    from ..config import environment
    from ..parallel import dist
    mc = ms.mc
    cols = [c for c in ms.stats_columns() if c.bin_boundary or c.bin_category]
    nums = [c.num for c in cols]
    from .base import _writer, shard_model_data
    cache_dir = ms.pf.correlation_path
    cache_m, cache_c = os.path.join(cache_dir, "corr.npy"), os.path.join(cache_dir, "columns.json")
    C = None
    if environment.get_bool("shifu.stats.corr.reuse", False) and os.path.exists(cache_m) and \
            os.path.exists(cache_c) and json.load(open(cache_c)) == nums:
        _log.info("correlation: reusing %s (shifu.stats.corr.reuse)", cache_m)
        C = np.load(cache_m, allow_pickle=False)
    elif _use_streaming(ms):
        C = _correlation_streamed(ms, cols, device)
        if _writer() and C is not None:
            os.makedirs(cache_dir, exist_ok=True)
            np.save(cache_m, C)
            with open(cache_c, "w") as f:
                json.dump(nums, f)
    else:
        md = shard_model_data(ms.load_raw(cols))
        # center on the stats step's means (the same on every rank; Pearson is shift invariant)
        shift = [0.0 if c.is_categorical() or not isinstance(c.mean, (int, float)) or not np.isfinite(c.mean)
                 else float(c.mean) for c in cols]
        acc = S.CorrAccumulator(len(cols), device, shift=shift)
        for r0 in range(0, max(md.n, 1), chunk_rows):
            r1 = min(md.n, r0 + chunk_rows)
            if r1 <= r0:
                break
            mats = []
            for c in cols:
                col = md.table[c.name]
                if c.is_categorical():
                    mats.append(N.normalize_column(c, col.slice(r0, r1), "OLD_ZSCALE", None)[:, 0])
                else:
                    mats.append(col.numeric()[r0:r1].astype(np.float64))
            acc.update(np.stack(mats, 1) if mats else np.zeros((r1 - r0, 0)))
        C = acc.finalize(0)
        if _writer() and C is not None:
            os.makedirs(cache_dir, exist_ok=True)
            np.save(cache_m, C)
            with open(cache_c, "w") as f:
                json.dump(nums, f)
    if not _writer():
        return C, [c.num for c in cols]
    path = ms.pf.correlation_csv
    # StatsModelProcessor.computeCorrValue layout (:490-590): an index line, a name line, then one
    # row per computed column: "<num>,<name>,<corr with every ColumnConfig column, ', '-joined>"
    # (columns without a correlation - meta, target-less, not computed - read 0.0)
    pos = {c.num: i for i, c in enumerate(cols)}
    with open(path, "w") as f:
        f.write("ColumnIndex," + "".join(f",{c.num}" for c in ms.ccs) + "\n")
        f.write(",ColumnName" + "".join(f",{c.name}" for c in ms.ccs) + "\n")
        for i, c in enumerate(cols):
            vals = [repr(float(C[i, pos[o.num]])) if o.num in pos else "0.0" for o in ms.ccs]
            f.write(f"{c.num},{c.name}," + ", ".join(vals) + "\n")
    _log.info("correlation: %d columns -> %s", len(cols), path)
    return C, [c.num for c in cols]


def _correlation_streamed(ms: ModelSet, cols, device=None):
    """``stats -c`` over this rank's byte range chunk by chunk (the data set never sits in host
    memory whole: 20M x 1600 fp64 would be 256 GB).  On a GPU the numeric columns are parsed on
    the device (K0) and fed to the accumulator as [rows, F] views of the parsed block; categorical
    columns take their pos-rate encoding on the host.  Same rows (purified, all of them) and the
    same accumulator as the in-memory pass; with the exact int8-digit sums (GPU) the matrix is
    identical."""
    import torch
    from ..config import environment
    from ..data import stream as DS
    from ..data.gpu_parse import device_rows
    from ..data.purifier import plan_dataset
    from ..parallel import dist
    mc = ms.mc
    info = dist.info()
    plan = plan_dataset(mc, mc.dataSet, [c.name for c in cols if not c.is_categorical()],
                        [c.name for c in cols if c.is_categorical()])
    pdev = _parse_device(device)
    chunk = int(float(environment.get("shifu.stats.chunkMB", 1024 if pdev is not None else 256)) * (1 << 20))
    shift = [0.0 if c.is_categorical() or not isinstance(c.mean, (int, float)) or not np.isfinite(c.mean)
             else float(c.mean) for c in cols]
    acc = S.CorrAccumulator(len(cols), device, shift=shift)
    num_j = [j for j, c in enumerate(cols) if not c.is_categorical()]
    cat_j = [j for j, c in enumerate(cols) if c.is_categorical()]
    for md in DS.iter_model_data(mc, plan, chunk, info.rank, info.world_size,
                                 gpu_cols=[cols[j].name for j in num_j], dev=pdev):
        n = md.n
        dv = device_rows([md.table.columns.get(cols[j].name) for j in num_j], pdev) if pdev is not None and num_j \
            else None
        if dv is not None:
            X = torch.empty((n, len(cols)), dtype=torch.float64, device=dv.device)
            X[:, num_j] = dv.t()
        else:
            X = np.empty((n, len(cols)), np.float64)
            for j in num_j:
                X[:, j] = md.table[cols[j].name].numeric()
        for j in cat_j:
            v = N.normalize_column(cols[j], md.table[cols[j].name], "OLD_ZSCALE", None)[:, 0]
            X[:, j] = torch.as_tensor(v, device=X.device) if torch.is_tensor(X) else v
        acc.update(X)
    return acc.finalize(0)


def read_correlation(path: str):
    """Parse ``correlation.csv``: returns (names of the computed rows, square matrix over them)."""
    with open(path) as f:
        f.readline()
        names_all = f.readline().rstrip("\n").split(",")[2:]
        keys, names, rows = [], [], []
        for line in f:
            if not line.strip():
                continue
            parts = line.rstrip("\n").split(",")
            keys.append(int(parts[0]))
            names.append(parts[1])
            rows.append([float(v) for v in parts[2:]])
    if not rows:
        return [], np.zeros((0, 0))
    full = np.array(rows)
    # row key -> column position in the all-column value list (ColumnConfig order = columnNum)
    idx = [names_all.index(nm) if nm in names_all else k for k, nm in zip(keys, names)]
    return names, full[:, idx]


def _iv(pos, neg):
    m = S.column_metrics(neg, pos)
    return m[1] if m else 0.0


def rebin_numeric(bounds, cpos, cneg, wpos, wneg, target_bins: int, iv_keep_ratio: float = 1.0):
    """Greedy adjacent merge minimizing IV loss (missing bin last, never merged)."""
    b = list(bounds)
    cp, cn = list(cpos[:-1]), list(cneg[:-1])
    wp, wn = list(wpos[:-1]), list(wneg[:-1])
    miss = (cpos[-1], cneg[-1], wpos[-1], wneg[-1])
    full_iv = _iv(np.array(cp + [miss[0]]), np.array(cn + [miss[1]]))
    while len(b) > max(1, target_bins):
        best, best_iv = None, -np.inf
        for i in range(len(b) - 1):
            p2 = cp[:i] + [cp[i] + cp[i + 1]] + cp[i + 2:] + [miss[0]]
            n2 = cn[:i] + [cn[i] + cn[i + 1]] + cn[i + 2:] + [miss[1]]
            v = _iv(np.array(p2), np.array(n2))
            if v > best_iv:
                best, best_iv = i, v
        if iv_keep_ratio < 1.0 and full_iv > 0 and best_iv < iv_keep_ratio * full_iv:
            break
        i = best
        cp[i:i + 2] = [cp[i] + cp[i + 1]]
        cn[i:i + 2] = [cn[i] + cn[i + 1]]
        wp[i:i + 2] = [wp[i] + wp[i + 1]]
        wn[i:i + 2] = [wn[i] + wn[i + 1]]
        del b[i + 1]
    return b, cp + [miss[0]], cn + [miss[1]], wp + [miss[2]], wn + [miss[3]]


def do_rebin(ms: ModelSet, target_bins: int, iv_keep_ratio: float = 1.0, min_inst_cnt: float = 0,
             request_vars: list[str] | None = None):
    """``stats -rebin`` (StatsModelProcessor.java:165-205, doReBin :670-760): re-bin from the
    binning saved in ``tmp/ColumnConfig.json`` (created on the first rebin, so repeated rebins
    always start from the original stats), for the requested good candidate columns, with the
    IV-keeping dynamic merge of ``algos.dynamic_binning``."""
    import json
    import os
    from ..algos.dynamic_binning import CATEGORICAL_GROUP_VAL_DELIMITER, dynamic_rebin
    from ..config.column_config import save_column_configs
    backup = ms.pf.p("tmp", "ColumnConfig.json")
    if not os.path.exists(backup):
        os.makedirs(os.path.dirname(backup), exist_ok=True)
        save_column_configs(ms.ccs, backup)
    else:
        with open(backup) as f:
            saved = {d["columnName"]: d.get("columnBinning") for d in json.load(f)}
        for c in ms.ccs:
            if saved.get(c.name) is not None:
                c.d["columnBinning"] = saved[c.name]
    binary = ms.mc.is_binary()
    from ..config.column_config import has_candidates
    has_cand = has_candidates(ms.ccs)
    for c in ms.ccs:
        if request_vars and c.name not in request_vars:
            continue
        if not c.is_good_candidate(has_cand, binary) or c.bin_count_pos is None:
            continue
        cp, cn = np.asarray(c.bin_count_pos), np.asarray(c.bin_count_neg)
        wp, wn = np.asarray(c.bin_weighted_pos), np.asarray(c.bin_weighted_neg)
        cat = c.is_categorical()
        keys = (c.bin_category if cat else c.bin_boundary) or []
        if not keys:
            continue
        bins, miss = dynamic_rebin(cat, keys, cp, cn, wp, wn, target_bins or 0, iv_keep_ratio, min_inst_cnt)
        if cat:
            c.bin_category = [CATEGORICAL_GROUP_VAL_DELIMITER.join(b.values) for b in bins]
        else:
            c.bin_boundary = [b.left for b in bins]
        cp2 = [b.pos for b in bins] + [miss.pos]
        cn2 = [b.neg for b in bins] + [miss.neg]
        wp2 = [b.wpos for b in bins] + [miss.wpos]
        wn2 = [b.wneg for b in bins] + [miss.wneg]
        cb = c.binning
        cb["binCountPos"], cb["binCountNeg"] = [int(x) for x in cp2], [int(x) for x in cn2]
        cb["binWeightedPos"], cb["binWeightedNeg"] = [float(x) for x in wp2], [float(x) for x in wn2]
        cb["length"] = len(cp2) - 1
        cp2, cn2 = np.array(cp2, float), np.array(cn2, float)
        cb["binPosRate"] = [float(x) for x in np.where(cp2 + cn2 > 0, cp2 / np.maximum(cp2 + cn2, 1), 0.0)]
        if binary:
            m, mw = S.column_metrics(cn2, cp2), S.column_metrics(np.array(wn2), np.array(wp2))
            if m:
                c.stats["ks"], c.stats["iv"], c.stats["woe"] = m[0], m[1], m[2]
                cb["binCountWoe"] = m[3]
            if mw:
                c.stats["weightedKs"], c.stats["weightedIv"], c.stats["weightedWoe"] = mw[0], mw[1], mw[2]
                cb["binWeightedWoe"] = mw[3]
