"""Scoring runtime (I6): load a model set's models by suffix and score raw rows.

* ``ModelSpecLoaderUtils.loadModel`` (J/util/ModelSpecLoaderUtils.java:389-445): ``model<i>.nn``
  (Encog text or binary v1), ``.lr``, ``.gbt``, ``.rf``, ``.wdl``; sorted by model index.
* ``ModelRunner.compute`` / ``Scorer.scoreNsData`` (J/core/ModelRunner.java:140-260,
  J/core/Scorer.java:219-506): NN/LR/WDL get the ColumnConfig-normalized selected columns, trees
  the raw values; per model one score (or one per class), then mean/max/min/median x scoreScale
  (``EvalScoreUDF`` J/udf/EvalScoreUDF.java:226).
* generic models (``models/*.json`` GenericModelConfig, ``scoring/generic.py``) when the
  algorithm is ``generic`` / ``tensorflow``.
* ``IndependentNNModel`` (binary ``.nn`` with embedded column stats, J/core/dtrain/nn/IndependentNNModel.java:211-232)
  and ``IndependentTreeModel`` (``.gbt``) as dependency-light production scorers.

Scoring is batched: the normalized matrix is built once per table and every NN bag runs as
GEMMs on the device.
"""
from __future__ import annotations

import glob
import os
import re
from collections import OrderedDict

import numpy as np
import torch

from ..algos.normalize import normalize_table
from ..config.column_config import ColumnConfig
from ..formats import nn_format, tree_format
from ..models import lr as lrmod
from ..utils.log import get_logger
from .tree_ensemble import TreeScorer

_log = get_logger("scoring")
SUFFIXES = ("nn", "lr", "gbt", "rf", "wdl")


def list_model_files(models_dir: str, alg: str | None = None):
    files = []
    for ext in SUFFIXES:
        files += glob.glob(os.path.join(models_dir, f"model*.{ext}"))
    if alg:
        want = {"NN": "nn", "LR": "lr", "GBT": "gbt", "RF": "rf", "WDL": "wdl"}.get(alg.upper())
        if want and any(f.endswith("." + want) for f in files):
            files = [f for f in files if f.endswith("." + want)]

    def key(p):
        m = re.search(r"model(\d+)", os.path.basename(p))
        return int(m.group(1)) if m else 1 << 30
    return sorted(files, key=key)


def _dev(device):
    return torch.device(device) if device is not None else (
        torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))


def _nn_forward_bf16(net, Xt, dev, chunk):
    """bf16 forward on the trainer's hand-written MFMA GEMMs (gemm_kernels.hip shifu_gemm_nt,
    EPI_ACT: activation + bias column + zero padding in the epilogue), fp32 accumulation."""
    from ..models.nn import ACT_IDS
    from ..ops import _native as nat
    pad = lambda k: ((k + 127) // 128) * 128
    dims = [net.weights[0].shape[1] - 1] + [W.shape[0] for W in net.weights]
    kp = [pad(d + 1) for d in dims]
    Wb = []
    for l, W in enumerate(net.weights):
        w = torch.zeros(dims[l + 1], kp[l], dtype=torch.bfloat16, device=dev)
        w[:, : dims[l] + 1] = torch.as_tensor(np.asarray(W), dtype=torch.float32)
        Wb.append(w)
    out = []
    for r in range(0, Xt.shape[0], chunk):
        xb = Xt[r: r + chunk].to(dev, torch.float32)
        m = xb.shape[0]
        a = torch.zeros(m, kp[0], dtype=torch.bfloat16, device=dev)
        a[:, : dims[0]] = xb
        a[:, dims[0]] = 1.0
        st = nat.stream_of(a)
        for l in range(len(Wb)):
            act = ACT_IDS[net.acts[l]]
            c = torch.empty(m, kp[l + 1], dtype=torch.bfloat16, device=dev)
            c2 = torch.empty_like(c) if act in (5, 8) else None
            last = l == len(Wb) - 1
            nat.call_hip("shifu_gemm_nt", a, kp[l], Wb[l], kp[l], dims[l + 1], c, kp[l + 1], c2, kp[l + 1], None, 0,
                         None, 0, m, kp[l + 1], kp[l], 0, act, dims[l + 1], 0 if last else 1, 0.0, st)
            a = c
        out.append(a[:, : dims[-1]].double().cpu())
    return torch.cat(out).numpy() if out else np.zeros((0, net.n_out))


@torch.no_grad()
def nn_forward(net: nn_format.NNNetwork, X, device=None, chunk: int = 1 << 18, precision: str | None = None) -> np.ndarray:
    """Batched forward of an input-first network on the device -> [N, n_out] float64.

    fp32 by default (``shifu.eval.nnPrecision=fp32``): scores agree with the reference's float
    scoring (IndependentNNModel) to ~1e-6 -- eval / posttrain / SE base scores are written as text
    and compared across runs.  On a GPU this runs on the framework's own MFMA GEMM over
    split-bf16 operands (``ops/gemm_ops.linear_fp32``, 6 part products = fp32 accuracy, activation
    in the fp32 tile epilogue); ``fp32_torch`` keeps the vendor fp32 GEMM (the oracle, and the CPU
    path).  ``bf16``: the trainer's own MFMA kernels (``_nn_forward_bf16``), ~3 significant
    digits, for throughput-bound scoring."""
    from ..models.nn import ACT_IDS, act_fwd
    dev = _dev(device)
    if precision is None:
        from ..config import environment
        precision = environment.get("shifu.eval.nnPrecision", "fp32")
    Xt = torch.as_tensor(X)
    sub = net.input_subset()
    if sub is not None and Xt.shape[1] != net.n_in:
        Xt = Xt[:, torch.as_tensor(sub, dtype=torch.long)]
    if precision == "bf16" and dev.type == "cuda":
        return _nn_forward_bf16(net, Xt, dev, chunk)
    Ws = [torch.as_tensor(np.asarray(W), dtype=torch.float32, device=dev) for W in net.weights]
    own = precision == "fp32" and dev.type == "cuda"
    if own:
        from ..ops.gemm_ops import SplitWeights, linear_fp32
        sws = [SplitWeights(W[:, :-1], W[:, -1].contiguous(), terms=6) for W in Ws]
    out = []
    for r in range(0, Xt.shape[0], chunk):
        a = Xt[r: r + chunk].to(dev, torch.float32)
        for l, W in enumerate(Ws):
            if own:
                a = linear_fp32(a, None, None, sw=sws[l], act=ACT_IDS[net.acts[l]])
            else:
                a = act_fwd(net.acts[l], a @ W[:, :-1].t() + W[:, -1])
        out.append(a.double().cpu())
    return torch.cat(out).numpy() if out else np.zeros((0, net.n_out))


class LoadedModel:
    def __init__(self, path: str, kind: str, obj, n_out: int = 1):
        self.path, self.kind, self.obj, self.n_out = path, kind, obj, n_out

    @property
    def name(self):
        return os.path.splitext(os.path.basename(self.path))[0]


def load_model(path: str, device=None, gbt_convert: str = "RAW") -> LoadedModel:
    ext = path.rsplit(".", 1)[-1].lower()
    if ext == "nn":
        if nn_format.is_binary_nn(path):
            d = nn_format.read_binary_nn(path)
            return LoadedModel(path, "nn_binary", d, d["networks"][0].n_out)
        net = nn_format.read_encog(path)
        return LoadedModel(path, "nn", net, net.n_out)
    if ext == "lr":
        return LoadedModel(path, "lr", lrmod.read_lr(path))
    if ext in ("gbt", "rf"):
        m = tree_format.read_tree_model(path)
        return LoadedModel(path, "tree", TreeScorer(m, _dev(device), gbt_convert))
    if ext == "wdl":
        from ..models.wdl import read_wdl
        return LoadedModel(path, "wdl", read_wdl(path))
    raise ValueError(f"unknown model file {path}")


class ModelRunner:
    """Scores RawTables with every model of a model set."""

    def __init__(self, mc, ccs, models_dir: str | None = None, model_paths=None, device=None,
                 gbt_convert: str | None = None):
        self.mc, self.ccs = mc, ccs
        self.dev = _dev(device)
        conv = gbt_convert or "RAW"
        from .generic import GENERIC_ALGORITHMS, find_generic_models, load_generic
        generic = str(mc.algorithm or "").lower() in GENERIC_ALGORITHMS
        if model_paths is not None:
            paths = model_paths
        elif generic:
            paths = find_generic_models(models_dir)
        else:
            paths = list_model_files(models_dir, mc.algorithm)
        if not paths:
            raise FileNotFoundError(f"no models under {models_dir}")
        self.models = [LoadedModel(p, "generic", load_generic(p)) if p.endswith(".json")
                       else load_model(p, self.dev, conv) for p in paths]
        from ..config.column_config import model_input_columns
        self.selected = model_input_columns(ccs, mc.is_binary())

    def raw_columns(self):
        cols = {c.name for c in self.selected}
        for m in self.models:
            if m.kind == "tree":
                cols |= set(m.obj.model.names.values())
            if m.kind == "nn_binary":
                cols |= {s.column_name for s in m.obj["column_stats"]}
            if m.kind == "generic":
                cols |= set(m.obj.input_names)
        return cols

    def _normalized_dev(self, table, cache):
        """The normalized rows left in HBM when the K5 pass made them (NN scoring reads them in
        place: no D2H + H2D round trip of [n, width] fp32), else the host rows."""
        if "X" not in cache and "Xd" not in cache:
            plan = self._norm_plan()
            if plan is not None:
                cache["Xd"] = plan.run(table, keep_device=True)["X"]
        return cache["Xd"] if "Xd" in cache else self._normalized(table, cache)

    def _normalized(self, table, cache):
        if "X" not in cache and "Xd" in cache:
            cache["X"] = cache["Xd"].cpu().numpy()
        if "X" not in cache:
            plan = self._norm_plan()
            if plan is not None:
                # the norm step's fused K5 pass (the same kernel that wrote the training rows): one
                # launch per chunk instead of a host numpy pass per column
                cache["X"] = plan.run(table)["X"]
            else:
                X, _, _ = normalize_table(self.mc, self.ccs, table, columns=self.selected)
                cache["X"] = X
        return cache["X"]

    def _norm_plan(self):
        """GPU NormPlan of the selected columns (``shifu.eval.gpuNorm``, default true on a GPU;
        within 1e-6 of the fp64 host oracle, tests/test_stats_kernels_gpu.py); None on the CPU."""
        if getattr(self, "_nplan", False) is False:
            self._nplan = None
            from ..config import environment
            if self.dev.type == "cuda" and environment.get_bool("shifu.eval.gpuNorm", True):
                from ..algos.normalize import NormPlan
                self._nplan = NormPlan(self.mc, self.ccs, self.selected, want_x=True, x_dtype="float32",
                                       device=self.dev)
        return self._nplan

    def score_models(self, table) -> list:
        """-> list of [N, n_out] raw score arrays (one per model)."""
        cache = {}
        outs = []
        for m in self.models:
            if m.kind == "nn":
                outs.append(nn_forward(m.obj, self._normalized_dev(table, cache), self.dev))
            elif m.kind == "nn_binary":
                outs.append(IndependentNNModel(m.obj, self.dev).compute(table))
            elif m.kind == "lr":
                outs.append(lrmod.lr_score(m.obj, self._normalized(table, cache))[:, None])
            elif m.kind == "tree":
                tm = m.obj.model
                if self.mc.is_multiclass() and tm.is_classification and not tm.is_one_vs_all:
                    outs.append(m.obj.class_votes(table, len(self.mc.tags())))
                else:
                    outs.append(m.obj.score(table)[:, None])
            elif m.kind == "wdl":
                outs.append(m.obj.score_table(self.mc, self.ccs, table)[:, None])
            elif m.kind == "generic":
                outs.append(m.obj.compute(self._generic_inputs(m.obj, table, cache)))
        return outs

    def _generic_inputs(self, gm, table, cache):
        """Normalized inputs in the generic model's ``inputnames`` order (default: selected)."""
        names = gm.input_names
        if not names:
            return self._normalized(table, cache)
        key = ("generic", tuple(names))
        if key not in cache:
            by_name = {c.name: c for c in self.ccs}
            missing = [n for n in names if n not in by_name]
            if missing:
                raise KeyError(f"generic model inputs not in ColumnConfig: {missing[:5]}")
            X, _, _ = normalize_table(self.mc, self.ccs, table, columns=[by_name[n] for n in names])
            cache[key] = X
        return cache[key]

    def score(self, table, scale: float | None = None):
        """-> OrderedDict(mean, max, min, median, model0.. [N]) scaled by ``scoreScale``;
        multi-class: per class index the mean over models plus per-model columns."""
        scale = float(scale if scale is not None else 1000.0)
        outs = self.score_models(table)
        res = OrderedDict()
        if self.mc.is_multiclass():
            if self.mc.is_one_vs_all():
                S = np.stack([o[:, 0] for o in outs], 1) * scale          # model i = class i
                res["class_scores"] = S
            else:
                S = np.stack(outs, 0) * scale                             # [M, N, C]
                res["class_scores"] = S.mean(0)
                for i, o in enumerate(outs):
                    res[f"model{i}"] = o * scale
            res["pred_class"] = res["class_scores"].argmax(1)
            return res
        S = np.stack([o[:, 0] for o in outs], 1) * scale
        res["mean"] = S.mean(1)
        res["max"] = S.max(1)
        res["min"] = S.min(1)
        res["median"] = np.median(S, 1)
        for i in range(S.shape[1]):
            res[f"model{i}"] = S[:, i]
        return res


class IndependentNNModel:
    """Binary ``.nn`` scorer with its own normalization (no ColumnConfig needed)."""

    def __init__(self, d: dict, device=None):
        self.d = d
        self.dev = _dev(device)
        self.norm = d["norm_type"]
        self.ccs = []
        for s in sorted(d["column_stats"], key=lambda s: d["column_mapping"].get(s.column_num, s.column_num)):
            cc = ColumnConfig()
            cc.num, cc.name, cc.type = s.column_num, s.column_name, s.column_type
            cc.final_select = True
            st, cb = cc.stats, cc.binning
            st["mean"], st["stdDev"] = s.mean, s.stddev
            cb["binBoundary"] = list(s.bin_boundaries) if s.bin_boundaries else None
            cb["binCategory"] = list(s.bin_categories) if s.bin_categories else None
            cb["binPosRate"] = list(s.bin_pos_rates)
            cb["binCountWoe"] = list(s.bin_count_woes)
            cb["binWeightedWoe"] = list(s.bin_weight_woes)
            cc.d["_woeMeanStd"] = (s.woe_mean, s.woe_stddev, s.woe_wgt_mean, s.woe_wgt_stddev)
            cc.d["_cutoff"] = s.cutoff
            self.ccs.append(cc)

    def compute(self, table) -> np.ndarray:
        from ..config.model_config import ModelConfig
        mc = ModelConfig({"normalize": {"normType": self.norm,
                                        "stdDevCutOff": self.ccs[0].d["_cutoff"] if self.ccs else 6.0}})
        X, _, _ = normalize_table(mc, self.ccs, table, columns=self.ccs, norm_type=self.norm)
        outs = [nn_forward(net, X, self.dev) for net in self.d["networks"]]
        return np.mean(outs, 0)


class IndependentTreeModel(TreeScorer):
    """``IndependentTreeModel.loadFromStream(...).compute`` equivalent for one ``.gbt``/``.rf``."""

    @staticmethod
    def load(path: str, device=None, convert: str = "RAW"):
        return IndependentTreeModel(tree_format.read_tree_model(path), _dev(device), convert)
