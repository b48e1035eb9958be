"""``posttrain`` step (B8, H15): per-bin average model score (``binAvgScore``) and feature importance.

``PostTrainModelProcessor.run`` (J/core/processor/PostTrainModelProcessor.java:86-113) scores the
training data with the ensemble (``PostTrainMapper.map`` J/core/posttrain/PostTrainMapper.java:183-256),
averages the score per (column, bin) and stores it in ``columnBinning.binAvgScore``; tree models
also get gain-based feature importance (``runMRFeatureImportanceJob`` :301).  Reason codes
(``Reasoner`` J/core/Reasoner.java:40-184) rank a row's variables by how far their bin's average
score is below the column's best bin.
"""
from __future__ import annotations

import numpy as np
import torch

from ..algos.normalize import _bin_num
from ..formats import tree_format
from ..parallel import dist
from ..scoring.model_runner import ModelRunner, list_model_files
from ..utils.device import default_device
from ..utils.log import get_logger
from .base import ModelSet, _writer, shard_model_data

_log = get_logger("steps.posttrain")


def _bin_score_sums_host(c, col, score):
    b = _bin_num(c, col)
    nb = c.n_bins()                            # incl. the missing bin (last)
    b = np.where(b < 0, nb - 1, np.minimum(b, nb - 1))
    return np.stack([np.bincount(b, weights=score, minlength=nb), np.bincount(b, minlength=nb).astype(np.float64)])


def _bin_score_sums_gpu(used, table, score, dev, batch: int = 64):
    """K18 on the device: numeric bin indices by ``torch.bucketize`` on the HBM copy of the
    column, categorical through the host LUT, then one ``keyed_hist`` launch per column batch
    (per-bin row counts + fixed-point score sums, ``scoring_kernels.hip``)."""
    from ..algos.binning import bin_index_torch
    from ..ops.stats_ops import keyed_hist
    sc = torch.as_tensor(np.asarray(score, dtype=np.float64)).to(dev)
    out = []
    for i in range(0, len(used), batch):
        cs = used[i: i + batch]
        nbs = [c.n_bins() for c in cs]
        keys = torch.empty(len(cs), sc.numel(), dtype=torch.int32, device=dev)
        for j, c in enumerate(cs):
            col = table[c.name]
            if c.is_categorical():
                b = torch.as_tensor(_bin_num(c, col)).to(dev)
            else:
                bb = torch.as_tensor(np.asarray(c.bin_boundary or [float("-inf")], np.float64)).to(dev)
                if getattr(col, "dev", None) is not None and col._values is None and \
                        col.dev.block.D.device == dev:
                    v = col.dev.tensor()               # GPU-parsed (K0): already in HBM
                else:
                    v = torch.as_tensor(col.numeric().astype(np.float64)).to(dev)
                b = bin_index_torch(v, bb)
            keys[j] = torch.where(b < 0, nbs[j] - 1, torch.clamp(b, max=nbs[j] - 1)).to(torch.int32)
        cnt, ssum = keyed_hist(keys, max(nbs), sc)
        cnt, ssum = cnt.cpu().numpy(), ssum.cpu().numpy()
        out.extend(np.stack([ssum[j, :nb], cnt[j, :nb]]) for j, nb in enumerate(nbs))
    return out


def run_posttrain(root: str = ".", device=None) -> int:
    ms = ModelSet(root).setup("POSTTRAIN", validate=False)
    mc = ms.mc
    runner = ModelRunner(mc, ms.ccs, ms.pf.models_dir, device=device)
    cols = runner.selected
    names = runner.raw_columns()
    byname = {c.name: c for c in ms.ccs}
    # data parallel: every rank scores its row shard; the per-(column, bin) score sums and counts
    # are all-reduced once (the PostTrainMapper -> reducer shuffle), then every rank holds them
    dev = torch.device(device) if device is not None else default_device()
    raw_cols = [byname[n] for n in names if n in byname]
    from .stats import _use_streaming
    if _use_streaming(ms):
        used, parts = _posttrain_streamed(ms, runner, cols, raw_cols, dev)
    else:
        md = shard_model_data(ms.load_raw(raw_cols))
        res = runner.score(md.table, 1000.0)
        score = np.asarray(res["mean"] if "mean" in res else res["class_scores"].max(1))
        used = [c for c in cols if c.name in md.table]
        parts = _bin_score_sums_gpu(used, md.table, score, dev) if dev.type == "cuda" else \
            [_bin_score_sums_host(c, md.table[c.name], score) for c in used]
    if used and dist.info().world_size > 1:
        flat = dist.all_reduce_np(np.concatenate([p.reshape(-1) for p in parts]))
        off = 0
        for i, p in enumerate(parts):
            parts[i] = flat[off:off + p.size].reshape(p.shape)
            off += p.size
    for c, (s, n) in zip(used, parts):
        c.binning["binAvgScore"] = [int(round(v)) for v in np.where(n > 0, s / np.maximum(n, 1), 0.0)]
    ms.save_cc()
    if not _writer():
        return 0
    # feature importance for tree models
    fi_all = {}
    for p in list_model_files(ms.pf.models_dir):
        if p.endswith((".gbt", ".rf")):
            for k, v in tree_format.feature_importance(tree_format.read_tree_model(p)).items():
                fi_all[k] = fi_all.get(k, 0.0) + v
    if fi_all:
        tot = sum(fi_all.values())
        nm = {c.num: c.name for c in ms.ccs}
        with open(ms.pf.feature_importance, "w") as f:
            for k, v in sorted(fi_all.items(), key=lambda kv: -kv[1]):
                f.write(f"{k}\t{nm.get(k, k)}\t{v / tot}\n")
    _log.info("posttrain: binAvgScore for %d columns", len(cols))
    return 0


def _posttrain_streamed(ms, runner, cols, raw_cols, dev):
    """The posttrain pass over this rank's byte range chunk by chunk (out of core, SURVEY §5.7;
    the reference streams rows through PostTrainMapper): each chunk is scored and its per-(column,
    bin) score sums / counts are added up; on a GPU the model's numeric inputs are parsed on the
    device (K0) and binned where they land.  -> (columns, [2, n_bins] arrays)."""
    from ..config import environment
    from ..data import stream as DS
    from ..data.purifier import plan_dataset
    from .stats import _parse_device
    mc = ms.mc
    info = dist.info()
    plan = plan_dataset(mc, mc.dataSet, [c.name for c in raw_cols if not c.is_categorical()],
                        [c.name for c in raw_cols if c.is_categorical()])
    pdev = _parse_device(dev) if dev.type == "cuda" else None
    chunk = int(float(environment.get("shifu.stats.chunkMB", 1024 if pdev is not None else 256)) * (1 << 20))
    present = set(plan.header)
    used = [c for c in cols if c.name in present]
    acc = None
    for md in DS.iter_model_data(mc, plan, chunk, info.rank, info.world_size,
                                 gpu_cols=[c.name for c in raw_cols if not c.is_categorical()], dev=pdev):
        res = runner.score(md.table, 1000.0)
        score = np.asarray(res["mean"] if "mean" in res else res["class_scores"].max(1))
        parts = _bin_score_sums_gpu(used, md.table, score, pdev) if pdev is not None else \
            [_bin_score_sums_host(c, md.table[c.name], score) for c in used]
        acc = parts if acc is None else [a + p for a, p in zip(acc, parts)]
    if acc is None:                            # no rows on this rank: zeros for the all-reduce
        acc = [np.zeros((2, c.n_bins())) for c in used]
    return used, acc


def reason_codes(ccs, table, top_k: int = 3):
    """Per row the ``top_k`` variable names whose bin average score is furthest below the
    column's maximum bin average score (Reasoner semantics)."""
    cols = [c for c in ccs if c.final_select and c.bin_avg_score and c.name in table]
    if not cols:
        return [[] for _ in range(table.n)]
    gaps = []
    for c in cols:
        avg = np.asarray(c.bin_avg_score, dtype=np.float64)
        b = _bin_num(c, table[c.name])
        b = np.where(b < 0, len(avg) - 1, np.minimum(b, len(avg) - 1))
        gaps.append(avg.max() - avg[b])
    G = np.stack(gaps, 1)
    order = np.argsort(-G, axis=1, kind="stable")[:, :top_k]
    return [[cols[j].name for j in row] for row in order]
