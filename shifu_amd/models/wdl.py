"""Wide & Deep (H11, I4).

Semantics of ``WideAndDeep`` (J/core/dtrain/wdl/WideAndDeep.java:112-232): the wide part is a
sparse per-field LR over categorical bin indices (one weight per category + missing) plus a
dense LR over the numeric inputs plus a bias; the deep part concatenates the numeric inputs with
per-field embeddings (``NumEmbedColumnIds`` x ``NumEmbedOuputs``) and runs dense + activation
layers down to one logit; ``p = sigmoid(wide + deep)``; the gradient is the sigmoid-MSE one
``(p - y) p (1 - p) s`` with L2 (``WDLL2Reg``).  Full-batch epochs with the gradient all-reduced
over ranks like the NN trainer (``WDLMaster.doCompute`` :164-184 sums worker gradients).

On the GPU the wide sums and the deep input gathers are one HIP pass (``wdl_kernels.hip``), and
the deep tower's GEMMs run on the MLP's hand-written bf16 MFMA kernels (``_DeepMFMA``).  File format ``.wdl``: the reference's
``BinaryWDLSerializer`` / ``IndependentWDLModel`` layout (``formats/wdl_format.py``).
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch

from ..formats.javaio import JavaIn, JavaOut
from ..parallel import dist
from ..utils.log import get_logger
from .nn import act_fwd

_log = get_logger("models.wdl")


# GPU wide sums + deep input gathers in one pass (ops/csrc/wdl_kernels.hip); SHIFU_WDL_HIP=0: torch ops
WDL_HIP = os.environ.get("SHIFU_WDL_HIP", "1") != "0"


class _WdlGather(torch.autograd.Function):
    """(dense, cats, wide tables, embedding tables) -> (wide sum per row, [dense | embeddings]) with
    the HIP gather kernels; backward scatters into the concatenated tables."""

    @staticmethod
    def forward(ctx, dense, cats, wt, et, woff, eoff, efield, D, want_wide, want_deep):
        from ..ops import _native as nat
        n, nd = dense.shape
        Fc, E = cats.shape[1], int(efield.numel())
        wide = torch.empty(n, device=dense.device) if want_wide else None
        A = torch.empty(n, nd + E * D, device=dense.device) if want_deep else None
        nat.call_hip("shifu_wdl_gather", 0, dense, nd, cats, Fc, wt, woff, et, eoff, efield, E, D, wide, A,
                     nd + E * D, None, None, wt.numel(), et.numel(), n, nat.stream_of(dense))
        ctx.save_for_backward(cats, woff, eoff, efield)
        ctx.meta = (n, nd, Fc, E, D, wt.numel(), et.numel(), bool(want_wide), bool(want_deep))
        return (wide if wide is not None else dense.new_zeros(n)), (A if A is not None else dense.new_zeros(n, 0))

    @staticmethod
    def backward(ctx, g_wide, g_A):
        from ..ops import _native as nat
        cats, woff, eoff, efield = ctx.saved_tensors
        n, nd, Fc, E, D, nw, ne, want_wide, want_deep = ctx.meta
        dev = cats.device
        # an output that was not produced (the 1-element / 0-column placeholder) gets an
        # autograd-materialised zero gradient: never scatter it into the placeholder tables
        gw = g_wide.contiguous() if (want_wide and g_wide is not None) else None
        gA = g_A.contiguous() if (want_deep and g_A is not None and g_A.shape[1] == nd + E * D) else None
        dwt = torch.zeros(nw, device=dev) if gw is not None else None
        det = torch.zeros(ne, device=dev) if gA is not None else None
        nat.call_hip("shifu_wdl_gather", 1, None, nd, cats, Fc, None, woff, None, eoff, efield, E, D, gw, gA,
                     nd + E * D, dwt, det, nw, ne, n, nat.stream_of(cats))
        ddense = gA[:, :nd] if gA is not None else None
        return ddense, None, dwt, det, None, None, None, None, None, None


# deep layers on the hand-written bf16 MFMA GEMMs (gemm_kernels.hip); SHIFU_WDL_DEEP=torch: fp32 torch
WDL_DEEP_HIP = os.environ.get("SHIFU_WDL_DEEP", "hip") != "torch"
_P = 128                                  # row widths padded to 128 (gemm_nt K % 64, wgrad_tn K % 128)


def _pad(k: int) -> int:
    return ((k + _P - 1) // _P) * _P


def _deriv_from_out(act: str, a: torch.Tensor) -> torch.Tensor:
    """f'(z) from the activation output a = f(z) (common.h act_deriv_out)."""
    if act == "sigmoid":
        return a * (1 - a)
    if act == "tanh":
        return 1 - a * a
    if act == "linear":
        return torch.ones_like(a)
    if act == "relu":
        return (a > 0).to(a.dtype)
    if act == "leakyrelu":
        return torch.where(a <= 0, torch.full_like(a, 0.01), torch.ones_like(a))
    if act == "ptanh":
        return torch.where(a > 0, 1 - a * a, 0.25 * (1 - 16 * a * a))
    if act == "log":
        return torch.exp(-a.abs())
    raise ValueError(act)


def deep_forward(A, final, acts, Ws):
    """Deep tower (dense + activation layers, then the linear output neuron) with every GEMM on
    the MLP's own kernels: forward ``shifu_gemm_nt`` EPI_ACT (activation, bias column and zero
    padding written by the epilogue as the next layer's bf16 rows -- no per-layer cat).  Returns
    (out [n] fp32, state for ``deep_backward``).  bf16 activations, fp32 accumulation (the NN
    trainer's precision); WideAndDeep.java:163-232 semantics (no flat spot)."""
    from ..ops import _native as nat
    from .nn import ACT_IDS
    dev, n = A.device, A.shape[0]
    st = nat.stream_of(A)
    dims = [A.shape[1]] + [W.shape[0] for W in Ws]
    kp = [_pad(d + 1) for d in dims]
    X = torch.zeros(n, kp[0], dtype=torch.bfloat16, device=dev)
    X[:, : dims[0]] = A
    X[:, dims[0]] = 1.0
    xs, ders, wbs = [X], [], []
    for l, (W, act) in enumerate(zip(Ws, acts)):
        wb = torch.zeros(dims[l + 1], kp[l], dtype=torch.bfloat16, device=dev)
        wb[:, : dims[l] + 1] = W
        C = torch.empty(n, kp[l + 1], dtype=torch.bfloat16, device=dev)
        aid = ACT_IDS[act]
        C2 = None if aid in (0, 1, 2, 3, 4, 6, 7) else torch.empty_like(C)
        nat.call_hip("shifu_gemm_nt", xs[-1], kp[l], wb, kp[l], dims[l + 1], C, kp[l + 1], C2, kp[l + 1], None, 0,
                     None, 0, n, kp[l + 1], kp[l], 0, aid, dims[l + 1], 1, 0.0, st)
        xs.append(C)
        ders.append(C2)
        wbs.append(wb)
    # output neuron over [h_L | 1] (the bias column of xs[-1]): one wave per row (wdl_kernels.hip)
    out = torch.empty(n, dtype=torch.float32, device=dev)
    nat.call_hip("shifu_rowdot_bf16", xs[-1], kp[-1], n, dims[-1] + 1, final[0].float().contiguous(), out, st)
    return out, (list(acts), dims, kp, ders, wbs, final, xs, list(Ws))


def deep_backward(state, g):
    """(dA [n, in] fp32, d final [1, h_L + 1], [dW_l]) of ``sum_i g_i out_i``: ``shifu_gemm_nt``
    EPI_DACT (dgrad x f'(a) fused) and ``shifu_wgrad_tn`` (fp32 weight gradients)."""
    from ..ops import _native as nat
    from .nn import ACT_IDS
    acts, dims, kp, ders, wbs, final, xs, Ws = state
    L = len(Ws)
    n, dev = xs[-1].shape[0], xs[-1].device
    st = nat.stream_of(xs[-1])
    g = g.contiguous().float()
    # output-weight gradient sum_i g_i [h_L | 1]_i: per-256-row partials + a fixed-order sum
    g_final = torch.empty(1, dims[-1] + 1, dtype=torch.float32, device=dev)
    part = torch.empty(max(1, -(-n // 256)) * (dims[-1] + 1), dtype=torch.float32, device=dev)
    nat.call_hip("shifu_coldot_bf16", g, xs[-1], kp[-1], n, dims[-1] + 1, part, g_final, st)
    # output delta -> last hidden layer delta (elementwise; the output neuron is linear)
    aL = xs[-1][:, : dims[-1]].float()
    dl = ders[-1][:, : dims[-1]].float() if ders[-1] is not None else _deriv_from_out(acts[-1], aL)
    D = torch.zeros(n, kp[-1], dtype=torch.bfloat16, device=dev)
    D[:, : dims[-1]] = (g[:, None] * final[0, : dims[-1]][None, :]) * dl
    gWs = [None] * L
    for l in range(L - 1, -1, -1):
        G = torch.zeros(dims[l + 1], kp[l], dtype=torch.float32, device=dev)
        nat.call_hip("shifu_wgrad_tn", D, kp[l + 1], xs[l], kp[l], G, kp[l], n, dims[l + 1], kp[l],
                     max(1, min(n // 256, 256)), st)
        gWs[l] = G[:, : dims[l] + 1]
        # delta of the layer below (or the input gradient): D W_l through W_l^T as B rows
        wt = torch.zeros(kp[l], kp[l + 1], dtype=torch.bfloat16, device=dev)
        wt[: dims[l] + 1, : dims[l + 1]] = Ws[l].t()
        Dn = torch.empty(n, kp[l], dtype=torch.bfloat16, device=dev)
        if l > 0:
            aid = ACT_IDS[acts[l - 1]]
            nat.call_hip("shifu_gemm_nt", D, kp[l + 1], wt, kp[l + 1], kp[l], Dn, kp[l], None, 0,
                         xs[l], kp[l], ders[l - 1], kp[l], n, kp[l], kp[l + 1], 1, aid, dims[l], 0, 0.0, st)
        else:
            nat.call_hip("shifu_gemm_nt", D, kp[1], wt, kp[1], kp[0], Dn, kp[0], None, 0, None, 0, None, 0,
                         n, kp[0], kp[1], 2, 2, dims[0], 0, 0.0, st)
        D = Dn
    return D[:, : dims[0]].float(), g_final, gWs


class _DeepMFMA(torch.autograd.Function):
    """autograd wrapper of ``deep_forward`` / ``deep_backward`` (scoring and the kernel tests)."""

    @staticmethod
    def forward(ctx, A, final, acts, *Ws):
        out, state = deep_forward(A, final, acts, Ws)
        ctx.state = state
        return out

    @staticmethod
    def backward(ctx, g):
        dA, g_final, gWs = deep_backward(ctx.state, g)
        ctx.state = None
        return (dA, g_final, None, *gWs)


class WideDeepNet(torch.nn.Module):
    def __init__(self, n_dense: int, cat_sizes: list, embed_fields: list, embed_dim: int, hidden: list,
                 acts: list, wide: bool = True, deep: bool = True):
        super().__init__()
        self.n_dense, self.cat_sizes = n_dense, list(cat_sizes)
        self.embed_fields, self.embed_dim = list(embed_fields), int(embed_dim)
        self.hidden, self.acts = list(hidden), list(acts)
        self.wide_on, self.deep_on = wide, deep
        self.wide_tables = torch.nn.ParameterList([torch.nn.Parameter(torch.zeros(s + 1)) for s in cat_sizes])
        self.wide_dense = torch.nn.Parameter(torch.zeros(n_dense))
        self.bias = torch.nn.Parameter(torch.zeros(1))
        g = torch.Generator().manual_seed(7)
        self.embeds = torch.nn.ParameterList([
            torch.nn.Parameter(torch.randn(cat_sizes[f] + 1, embed_dim, generator=g) * 0.05) for f in embed_fields])
        dims = [n_dense + embed_dim * len(embed_fields)] + self.hidden
        self.layers = torch.nn.ParameterList()
        for i in range(len(self.hidden)):
            lim = (6.0 / (dims[i] + dims[i + 1])) ** 0.5
            self.layers.append(torch.nn.Parameter((torch.rand(dims[i + 1], dims[i] + 1, generator=g) * 2 - 1) * lim))
        self.final = torch.nn.Parameter((torch.rand(1, dims[-1] + 1, generator=g) * 2 - 1) * 0.1)

    def _hip_forward(self, dense, cats):
        dev = dense.device
        if getattr(self, "_offs", None) is None or self._offs[0].device != dev:
            ws = [s + 1 for s in self.cat_sizes]
            woff = torch.tensor(np.concatenate([[0], np.cumsum(ws)[:-1]]) if ws else [0], dtype=torch.int32)
            es = [(self.cat_sizes[f] + 1) for f in self.embed_fields]
            eoff = torch.tensor(np.concatenate([[0], np.cumsum(es)[:-1]]) if es else [0], dtype=torch.int32)
            self._offs = (woff.to(dev), eoff.to(dev), torch.tensor(self.embed_fields or [0], dtype=torch.int32).to(dev))
        woff, eoff, efield = self._offs
        if not self.embed_fields:
            efield = efield[:0]
        wt = torch.cat(list(self.wide_tables)) if self.wide_on and len(self.wide_tables) else dense.new_zeros(1)
        et = torch.cat([e.reshape(-1) for e in self.embeds]) if self.deep_on and len(self.embeds) else \
            dense.new_zeros(1)
        if not self.deep_on:
            efield = efield[:0]
        wide, A = _WdlGather.apply(dense.float().contiguous(), cats.long().contiguous(), wt, et, woff, eoff, efield,
                                   self.embed_dim, self.wide_on and len(self.wide_tables) > 0, self.deep_on)
        logit = torch.zeros(dense.shape[0], device=dev)
        if self.wide_on:
            logit = logit + dense @ self.wide_dense + self.bias + wide
        if self.deep_on:
            if WDL_DEEP_HIP and len(self.layers):
                logit = logit + _DeepMFMA.apply(A, self.final, tuple(self.acts), *self.layers)
            else:
                a = A
                for W, act in zip(self.layers, self.acts):
                    a = act_fwd(act, a @ W[:, :-1].t() + W[:, -1])
                logit = logit + (a @ self.final[:, :-1].t() + self.final[:, -1])[:, 0]
        return logit

    def forward(self, dense: torch.Tensor, cats: torch.Tensor) -> torch.Tensor:
        if dense.is_cuda and WDL_HIP and dense.shape[0]:
            return self._hip_forward(dense, cats)
        n = dense.shape[0]
        logit = torch.zeros(n, device=dense.device)
        if self.wide_on:
            logit = logit + dense @ self.wide_dense + self.bias
            for f, t in enumerate(self.wide_tables):
                logit = logit + t[cats[:, f]]
        if self.deep_on:
            parts = [dense] + [e[cats[:, f]] for e, f in zip(self.embeds, self.embed_fields)]
            a = torch.cat(parts, 1) if len(parts) > 1 else dense
            for W, act in zip(self.layers, self.acts):
                a = act_fwd(act, a @ W[:, :-1].t() + W[:, -1])
            logit = logit + (a @ self.final[:, :-1].t() + self.final[:, -1])[:, 0]
        return logit

    def arch(self):
        return dict(n_dense=self.n_dense, cat_sizes=self.cat_sizes, embed_fields=self.embed_fields,
                    embed_dim=self.embed_dim, hidden=self.hidden, acts=self.acts, wide=self.wide_on, deep=self.deep_on)


def wdl_inputs(ccs, table, cols, norm_cutoff: float):
    """(dense z-scored numerics [N, Dn] float32, categorical indices [N, Dc] int64, cat sizes)."""
    from ..algos.normalize import _cat_index, normalize_column
    num = [c for c in cols if not c.is_categorical()]
    cat = [c for c in cols if c.is_categorical()]
    n = table.n
    dense = np.stack([normalize_column(c, table[c.name], "ZSCALE", norm_cutoff)[:, 0] for c in num], 1) \
        if num else np.zeros((n, 0))
    sizes = [len(c.bin_category or []) for c in cat]
    idx = np.stack([np.where((i := _cat_index(c, table[c.name])) < 0, s, i) for c, s in zip(cat, sizes)], 1) \
        if cat else np.zeros((n, 0), np.int64)
    return dense.astype(np.float32), idx.astype(np.int64), sizes, num, cat


class WDLModel:
    def __init__(self, net: WideDeepNet, norm_type: str, col_stats: list, columns: list, cutoff: float):
        self.net, self.norm_type, self.col_stats, self.columns, self.cutoff = net, norm_type, col_stats, columns, cutoff

    def score_table(self, mc, ccs, table) -> np.ndarray:
        byname = {c.name: c for c in ccs}
        cols = [byname[n] for n in self.columns if n in byname]
        dense, idx, _, _, _ = wdl_inputs(ccs, table, cols, self.cutoff)
        dev = next(self.net.parameters()).device
        with torch.no_grad():
            return torch.sigmoid(self.net(torch.from_numpy(dense).to(dev), torch.from_numpy(idx).to(dev))).cpu() \
                .double().numpy()


def write_wdl(path: str, model: WDLModel):
    """Reference ``.wdl`` layout (``formats/wdl_format.py``, BinaryWDLSerializer :57-108)."""
    from ..formats.wdl_format import WDLSpec, write_wdl_file
    net = model.net
    nums = {cs.column_name: cs.column_num for cs in model.col_stats}
    types = {cs.column_name: cs.column_type for cs in model.col_stats}
    num_names = [n for n in model.columns if types.get(n, "N") != "C"]
    cat_names = [n for n in model.columns if types.get(n, "N") == "C"]
    ids = lambda names: [int(nums.get(n, k)) for k, n in enumerate(names)]   # noqa: E731
    dense_ids, wide_ids = ids(num_names), ids(cat_names)
    f32 = lambda t: t.detach().float().cpu().numpy()   # noqa: E731
    spec = WDLSpec(
        n_dense=net.n_dense, dense_ids=dense_ids, embed_ids=[wide_ids[f] for f in net.embed_fields],
        embed_outputs=[net.embed_dim] * len(net.embed_fields), wide_ids=wide_ids,
        cate_sizes={cid: s + 1 for cid, s in zip(wide_ids, net.cat_sizes)}, hidden=list(net.hidden),
        acts=list(net.acts), l2reg=float(getattr(model, "l2reg", 0.0)),
        hidden_W=[f32(W[:, :-1]).T.copy() for W in net.layers], hidden_b=[f32(W[:, -1]) for W in net.layers],
        final_W=f32(net.final[:, :-1]).T.copy(), final_b=f32(net.final[:, -1]),
        embed_W=[f32(e) for e in net.embeds], wide_W=[f32(t) for t in net.wide_tables],
        wide_dense=f32(net.wide_dense), bias=float(net.bias.detach()[0]), wide_on=net.wide_on, deep_on=net.deep_on)
    write_wdl_file(path, model.norm_type, model.col_stats, spec)


def read_wdl(path: str) -> WDLModel:
    from ..formats.wdl_format import read_wdl_file
    _, norm, stats, sp = read_wdl_file(path)
    byid = {cs.column_num: cs for cs in stats}
    cat_sizes = [int(sp.cate_sizes.get(c, len(w) if w is not None else 1)) - 1
                 for c, w in zip(sp.wide_ids, sp.wide_W or [None] * len(sp.wide_ids))]
    embed_fields = [sp.wide_ids.index(c) for c in sp.embed_ids]
    embed_dim = sp.embed_outputs[0] if sp.embed_outputs else (sp.embed_W[0].shape[1] if sp.embed_W else 8)
    net = WideDeepNet(sp.n_dense, cat_sizes, embed_fields, embed_dim, list(sp.hidden), list(sp.acts),
                      sp.wide_on, sp.deep_on)
    t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float32))   # noqa: E731
    with torch.no_grad():
        if sp.wide_on:
            for q, w in zip(net.wide_tables, sp.wide_W):
                q.copy_(t(w))
            net.wide_dense.copy_(t(sp.wide_dense))
            net.bias.fill_(float(sp.bias or 0.0))
        if sp.deep_on:
            for q, w in zip(net.embeds, sp.embed_W):
                q.copy_(t(w))
            for q, W, b in zip(net.layers, sp.hidden_W, sp.hidden_b):
                q.copy_(torch.cat([t(W).t(), t(b)[:, None]], 1))
            net.final.copy_(torch.cat([t(sp.final_W).t(), t(sp.final_b)[:, None]], 1))
    names = [byid[c].column_name for c in sp.dense_ids + sp.wide_ids if c in byid]
    cutoff = stats[0].cutoff if stats else 6.0
    return WDLModel(net, norm, stats, names, cutoff)


# ------------------------------------------------------------------------------------------------
# Training: WDLMaster + WDLWorker semantics (J/core/dtrain/wdl/WDLMaster.java:159-186,
# WDLWorker.java:679-718, WideAndDeep.java:163-232, the layers' backward, GradientDescent.java:44-63)
# ------------------------------------------------------------------------------------------------
class WDLRows:
    """This rank's training rows as (dense fp32 [m, nd], category indices int64 [m, Fc]) chunks.

    ``X`` is an [n, F] float array (the ZSCALE_INDEX NormalizedData memmap shard, or inputs built
    from raw columns) whose columns ``num_pos`` are the dense inputs and ``cat_pos`` the category
    indices (missing / unknown = the category count).  On the GPU the rows are uploaded once and
    stay resident when they fit in half of the free HBM; otherwise every epoch streams them from
    the host in chunks (a reader thread fills pinned buffers while the previous chunk computes).
    On the CPU the chunks are read from the memmap as they are used (bounded host memory)."""

    def __init__(self, X, num_pos, cat_pos, device, chunk_rows: int = 1 << 20):
        self.X, self.num_pos, self.cat_pos = X, list(num_pos), list(cat_pos)
        self.n = int(np.shape(X)[0])
        self.dev = torch.device(device)
        self.chunk_rows = int(chunk_rows)
        self.nd, self.fc = len(self.num_pos), len(self.cat_pos)
        self._resident = None
        if self.dev.type == "cuda":
            from ..utils.device import free_hbm
            need = self.n * (self.nd * 4 + self.fc * 8)
            force = os.environ.get("SHIFU_WDL_STREAM") == "1"
            if not force and need < 0.5 * free_hbm(self.dev):
                self._resident = [self._host_chunk(a, min(self.n, a + self.chunk_rows))
                                  for a in range(0, self.n, self.chunk_rows)]
                self._resident = [(d.to(self.dev), c.to(self.dev)) for d, c in self._resident]

    def _host_chunk(self, a, b):
        blk = np.asarray(self.X[a:b], dtype=np.float32)
        dense = torch.from_numpy(np.ascontiguousarray(blk[:, self.num_pos]) if self.nd else np.zeros((b - a, 0), np.float32))
        cats = torch.from_numpy(np.rint(blk[:, self.cat_pos]).astype(np.int64) if self.fc else np.zeros((b - a, 0), np.int64))
        return dense, cats

    def chunks(self):
        """-> (row0, row1, dense, cats) over the shard, on the device."""
        if self._resident is not None:
            for i, (d, c) in enumerate(self._resident):
                a = i * self.chunk_rows
                yield a, a + d.shape[0], d, c
            return
        bounds = [(a, min(self.n, a + self.chunk_rows)) for a in range(0, self.n, self.chunk_rows)]
        if self.dev.type != "cuda":
            for a, b in bounds:
                d, c = self._host_chunk(a, b)
                yield a, b, d, c
            return
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(1) as ex:            # reader thread: next chunk into pinned memory
            nxt = ex.submit(lambda ab: [t.pin_memory() for t in self._host_chunk(*ab)], bounds[0]) if bounds else None
            for i, (a, b) in enumerate(bounds):
                d, c = nxt.result()
                if i + 1 < len(bounds):
                    nxt = ex.submit(lambda ab: [t.pin_memory() for t in self._host_chunk(*ab)], bounds[i + 1])
                yield a, b, d.to(self.dev, non_blocking=True), c.to(self.dev, non_blocking=True)


class WDLTrainer:
    """Full-batch, data-parallel Wide & Deep training with the reference's master / worker math.

    Per epoch every rank runs ``WideAndDeep.forward`` / ``backward`` over its training rows:
    ``p = sigmoid(wide + deep)``, the logit gradient ``(p - y) p (1 - p) s`` (s: significance,
    WideAndDeep.java:203-207), every layer's weight gradients SUMMED over the rows, plus the layers'
    per-row L2 term (``l2reg * w`` added once per row to the dense layers' and the wide dense
    layer's weights, and per row to the wide-field weight the row touches; none on biases or
    embeddings: DenseLayer.java:188-198, WideDenseLayer.java:96-104, WideFieldLayer.java:97-109,
    EmbedFieldLayer.java:107-117).  The gradients of all ranks are summed by one all-reduce
    (WDLMaster.aggregateWorkerGradients) and the master's ``GradientDescent(LearningRate)``
    (``w -= lr * sum_grad``, GradientDescent.java:44-63, hard-wired in WDLMaster.java:175) runs
    on the replicated weights -- on the GPU in ``optimizer_kernel`` (rule B, momentum 0, on the
    ascent direction).  ``Optimizer: ADAM / ADAGRAD`` are extensions (the mean gradient through
    those rules).  The errors are ``sum s (p - y)^2 / row count`` for the training and the
    validation rows with the epoch's weights (WDLWorker.java:689-706).

    One documented deviation: the reference ASSIGNS the bias gradients per row (DenseLayer.java:197
    ``bGrads[j] = backInputs[j]``, BiasLayer.java:54), so only a worker's last row reaches the
    master; here bias gradients are summed over the rows like every other gradient (the assignment
    makes the result depend on the row order and the worker count).

    GPU: the wide sums / deep input gathers and their scatters are ``wdl_kernels.hip``, the dense
    wide part and its gradient the row / column dot kernels, the deep tower ``deep_forward`` /
    ``deep_backward`` (bf16 MFMA GEMMs, fp32 sums); no autograd, no torch.optim."""

    def __init__(self, net: WideDeepNet, device, lr: float, l2: float = 0.0, optimizer: str = "GD"):
        from .nn import Optimizer
        self.dev = torch.device(device)
        self.gpu = self.dev.type == "cuda"
        self.net = net.to(self.dev)
        # explicit order (Module.parameters() lists a module's own parameters before its lists')
        ps = list(net.wide_tables) + [net.wide_dense, net.bias] + list(net.embeds) + list(net.layers) + [net.final]
        self.params = ps
        sizes = [p.numel() for p in ps]
        self.flat = torch.empty(sum(sizes), dtype=torch.float32, device=self.dev)
        self.offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        for p, a, b in zip(ps, self.offs[:-1], self.offs[1:]):
            self.flat[a:b].copy_(p.data.reshape(-1))
            p.data = self.flat[a:b].view_as(p.data)
        self.grad = torch.zeros_like(self.flat)
        self.gviews = [self.grad[a:b].view_as(p) for p, a, b in zip(ps, self.offs[:-1], self.offs[1:])]
        fc, E, L = len(net.wide_tables), len(net.embeds), len(net.layers)
        self.i_wide, self.i_wd, self.i_bias = 0, fc, fc + 1
        self.i_emb, self.i_layers, self.i_final = fc + 2, fc + 2 + E, fc + 2 + E + L
        # rows whose weights take the per-row L2 term: wide dense, dense layers and final layer
        # weights (not their bias columns)
        l2row = torch.zeros_like(self.flat)
        mv = [l2row[a:b].view_as(p) for p, a, b in zip(ps, self.offs[:-1], self.offs[1:])]
        mv[self.i_wd].fill_(1.0)
        for i in list(range(self.i_layers, self.i_layers + L)) + [self.i_final]:
            mv[i][:, :-1] = 1.0
        self.l2row = l2row
        self.l2 = float(l2)
        self.lr = float(lr)
        self.opt_name = (optimizer or "GD").upper()
        rule = {"ADAM": "ADAM", "ADAGRAD": "ADAGRAD"}.get(self.opt_name, "B")
        self.opt = Optimizer(self.flat.numel(), self.dev, rule, learning_rate=self.lr, momentum=0.0)
        self.wide_cnt = None                     # per wide-table entry: training rows of this rank
        self.n_train = 0.0

    # ---- forward / backward of one chunk ------------------------------------------------------
    def _tables(self):
        net = self.net
        fc, E = len(net.wide_tables), len(net.embeds)
        wt = self.flat[self.offs[self.i_wide]: self.offs[self.i_wide + fc]] if fc else self.flat.new_zeros(1)
        et = self.flat[self.offs[self.i_emb]: self.offs[self.i_emb + E]] if E else self.flat.new_zeros(1)
        return wt, et

    def _forward_backward(self, dense, cats, y, s_tr):
        """logit of every row; accumulates the (ascent-direction) gradients of sum_i s_i * loss_i
        into self.grad.  Returns p."""
        net = self.net
        if self.gpu and WDL_HIP:
            return self._fb_hip(dense, cats, y, s_tr)
        n = dense.shape[0]
        gv = self.gviews
        logit = torch.zeros(n, device=self.dev)
        if net.wide_on:
            logit = logit + (dense @ net.wide_dense if net.n_dense else 0.0) + net.bias
            for f, t in enumerate(net.wide_tables):
                logit = logit + t[cats[:, f]]
        acts_out, zs = [], []
        if net.deep_on:
            parts = [dense] + [e[cats[:, f]] for e, f in zip(net.embeds, net.embed_fields)]
            a = torch.cat(parts, 1) if len(parts) > 1 else dense
            acts_out = [a]
            for W, act in zip(net.layers, net.acts):
                z = a @ W[:, :-1].t() + W[:, -1]
                a = act_fwd(act, z)
                zs.append(z)
                acts_out.append(a)
            logit = logit + (a @ net.final[0, :-1] + net.final[0, -1])
        p = torch.sigmoid(logit)
        g = (y - p) * p * (1 - p) * s_tr                      # ascent on the logit
        if net.wide_on:
            if net.n_dense:
                gv[self.i_wd].add_(g @ dense)
            gv[self.i_bias].add_(g.sum())
            for f in range(len(net.wide_tables)):
                gv[self.i_wide + f].index_add_(0, cats[:, f], g)
        if net.deep_on:
            from .nn import act_deriv
            aL = acts_out[-1]
            gv[self.i_final][0, :-1].add_(g @ aL)
            gv[self.i_final][0, -1].add_(g.sum())
            d = g[:, None] * net.final[0, :-1][None, :]
            for l in range(len(net.layers) - 1, -1, -1):
                a_in = acts_out[l]
                d = d * act_deriv(net.acts[l], zs[l], acts_out[l + 1])
                gv[self.i_layers + l][:, :-1].add_(d.t() @ a_in)
                gv[self.i_layers + l][:, -1].add_(d.sum(0))
                d = d @ net.layers[l][:, :-1]
            off = net.n_dense
            for k, f in enumerate(net.embed_fields):
                D = net.embed_dim
                gv[self.i_emb + k].index_add_(0, cats[:, f], d[:, off + k * D: off + (k + 1) * D])
        return p

    def _fb_hip(self, dense, cats, y, s_tr):
        from ..ops import _native as nat
        net = self.net
        n = dense.shape[0]
        st = nat.stream_of(dense)
        woff, eoff, efield = self._offsets()
        fc, E, D = len(net.wide_tables), len(net.embed_fields), net.embed_dim
        wt, et = self._tables()
        want_wide = net.wide_on and fc > 0
        wide = torch.zeros(n, device=self.dev)
        A = torch.empty(n, net.n_dense + E * D, device=self.dev) if net.deep_on else None
        ef = efield if (net.deep_on and E) else efield[:0]
        nat.call_hip("shifu_wdl_gather", 0, dense, net.n_dense, cats, fc, wt, woff, et, eoff, ef,
                     len(ef), D, wide if want_wide else None, A, net.n_dense + E * D, None, None, wt.numel(),
                     et.numel(), n, st)
        logit = wide
        if net.wide_on:
            if net.n_dense:
                lin = torch.empty(n, device=self.dev)
                nat.call_hip("shifu_rowdot_f32_act", dense, net.n_dense, n, net.n_dense, net.wide_dense, 0.0, -1, -1,
                             lin, st)
                logit = logit + lin
            logit = logit + net.bias
        state = None
        if net.deep_on:
            out, state = deep_forward(A, net.final, tuple(net.acts), tuple(net.layers))
            logit = logit + out
        p = torch.sigmoid(logit)
        g = ((y - p) * p * (1 - p) * s_tr).contiguous()
        gv = self.gviews
        if net.wide_on:
            if net.n_dense:
                tmp = torch.empty(net.n_dense, device=self.dev)
                part = torch.empty(max(1, -(-n // 256)) * net.n_dense, device=self.dev)
                nat.call_hip("shifu_coldot_f32", g, dense, net.n_dense, n, net.n_dense, part, tmp, st)
                gv[self.i_wd].add_(tmp)
            gv[self.i_bias].add_(g.sum())
        dwt = self.grad[self.offs[self.i_wide]: self.offs[self.i_wide + fc]] if want_wide else None
        dA = None
        if net.deep_on:
            dA, g_final, gWs = deep_backward(state, g)
            gv[self.i_final].add_(g_final)
            for l, G in enumerate(gWs):
                gv[self.i_layers + l].add_(G)
        det = self.grad[self.offs[self.i_emb]: self.offs[self.i_emb + len(net.embeds)]] if (dA is not None and E) else None
        if dwt is not None or det is not None:
            nat.call_hip("shifu_wdl_gather", 1, None, net.n_dense, cats, fc, None, woff, None, eoff, ef, len(ef), D,
                         g if dwt is not None else None, dA.contiguous() if det is not None else None,
                         net.n_dense + E * D, dwt, det, wt.numel(), et.numel(), n, st)
        return p

    def _offsets(self):
        net = self.net
        if getattr(self, "_offs", None) is None:
            ws = [s + 1 for s in net.cat_sizes]
            woff = torch.tensor(np.concatenate([[0], np.cumsum(ws)[:-1]]) if ws else [0], dtype=torch.int32)
            es = [(net.cat_sizes[f] + 1) for f in net.embed_fields]
            eoff = torch.tensor(np.concatenate([[0], np.cumsum(es)[:-1]]) if es else [0], dtype=torch.int32)
            ef = torch.tensor(net.embed_fields or [0], dtype=torch.int32)
            if not net.embed_fields:
                ef = ef[:0]
            self._offs = (woff.to(self.dev), eoff.to(self.dev), ef.to(self.dev))
        return self._offs

    # ---- one epoch ------------------------------------------------------------------------------
    def epoch(self, rows: WDLRows, y: np.ndarray, s_tr: np.ndarray, s_va: np.ndarray, n_tr: float, n_va: float):
        """One full-batch iteration.  y / s_tr / s_va: per-row labels, training significance (0 off
        the training set), validation weight (0 off the validation set).  Returns (train error,
        validation error) of the weights the epoch started from."""
        if self.wide_cnt is None:
            self._count_wide(rows, s_tr)
        self.grad.zero_()
        err = torch.zeros(2, dtype=torch.float64, device=self.dev)
        yt, st_, sv = (torch.from_numpy(np.asarray(a, np.float32)) for a in (y, s_tr, s_va))
        with torch.no_grad():
            for a, b, dense, cats in rows.chunks():
                yy = yt[a:b].to(self.dev, non_blocking=True)
                tr = st_[a:b].to(self.dev, non_blocking=True)
                va = sv[a:b].to(self.dev, non_blocking=True)
                p = self._forward_backward(dense, cats, yy, tr)
                e2 = (p - yy) ** 2
                err[0] += (e2 * tr).sum().double()
                err[1] += (e2 * va).sum().double()
            if self.l2 > 0:                       # per-row L2 of the layers (ascent: minus)
                self.grad.add_(-self.l2 * (self.n_train * self.l2row + self.wide_cnt) * self.flat)
            dist.all_reduce_(self.grad)
            dist.all_reduce_(err)
            tot = torch.tensor([n_tr, n_va], dtype=torch.float64, device=self.dev)
            dist.all_reduce_(tot)
            n_all = float(tot[0])
            g = self.grad if self.opt_name not in ("ADAM", "ADAGRAD") else self.grad / max(n_all, 1.0)
            self.opt.step(self.flat, g, n_all)
        terr = float(err[0]) / max(n_all, 1.0)
        verr = float(err[1]) / float(tot[1]) if float(tot[1]) > 0 else float("nan")
        return terr, verr

    def _count_wide(self, rows: WDLRows, s_tr: np.ndarray):
        """Training rows per wide-table entry on this rank (the wide fields' per-row L2 term)."""
        net = self.net
        cnt = torch.zeros_like(self.flat)
        on = torch.from_numpy((np.asarray(s_tr) != 0).astype(np.float32))
        self.n_train = float(on.sum())
        if net.wide_on and len(net.wide_tables):
            cv = [cnt[a:b] for a, b in zip(self.offs[:-1], self.offs[1:])]
            with torch.no_grad():
                for a, b, _, cats in rows.chunks():
                    w = on[a:b].to(self.dev)
                    for f in range(len(net.wide_tables)):
                        cv[self.i_wide + f].index_add_(0, cats[:, f], w)
        self.wide_cnt = cnt


def wdl_rows_from_cache(ms, ts):
    """(X, num_pos, cat_pos) of a ZSCALE_INDEX-family NormalizedData shard (``ts.X``), or None."""
    from ..config.enums import is_index_norm
    if ts.X is None or not is_index_norm(ms.mc.norm_type):
        return None
    nums = list(ts.meta.get("input_nums") or [])
    cols = ms.input_columns()
    pos = {n: i for i, n in enumerate(nums)}
    if len(nums) != np.shape(ts.X)[1] or any(c.num not in pos for c in cols):
        return None
    num_pos = [pos[c.num] for c in cols if not c.is_categorical()]
    cat_pos = [pos[c.num] for c in cols if c.is_categorical()]
    return ts.X, num_pos, cat_pos


def train_wdl_step(step, tid, p, ts, y, train_m, valid_m, sw):
    """Train one WDL bag inside ``TrainStep``.  Rows: this rank's shard of the ZSCALE_INDEX
    NormalizedData (z-scored numerics, category indices) with the step's counter-based split;
    other norm types: the inputs are rebuilt from this rank's shard of the raw columns."""
    from ..steps.base import shard_model_data
    from ..steps.train import TrainSet, split_masks
    ms, mc = step.ms, step.mc
    cols = ms.input_columns()
    num = [c for c in cols if not c.is_categorical()]
    cat = [c for c in cols if c.is_categorical()]
    cutoff = float(mc.normalize.get("stdDevCutOff", 6.0))
    src = wdl_rows_from_cache(ms, ts)
    if src is not None:
        X, num_pos, cat_pos = src
        w = np.asarray(ts.w, np.float32)
        yy = np.asarray(y, np.float32)
        tr_m, va_m, sw_ = train_m, valid_m, sw
    else:
        info = dist.info()
        full = ms.load_raw(cols)
        md = shard_model_data(full)
        dense, idx, _, _, _ = wdl_inputs(ms.ccs, md.table, cols, cutoff)
        X = np.concatenate([dense, idx.astype(np.float32)], 1)
        num_pos, cat_pos = list(range(dense.shape[1])), list(range(dense.shape[1], X.shape[1]))
        w, yy = md.w.astype(np.float32), md.y.astype(np.float32)
        fake = TrainSet(y=yy, w=w, row0=full.n * info.rank // info.world_size)
        n_kfold = int(mc.train.get("numKFold", -1) or -1)
        seed = max(0, int(mc.train.get("baggingSampleSeed", -1)))
        tr_m, va_m, sw_ = split_masks(mc, fake, tid, n_kfold, seed)
    sizes = [len(c.bin_category or []) for c in cat]
    embed_ids = p.get("NumEmbedColumnIds")
    cat_nums = [c.num for c in cat]
    embed_fields = [cat_nums.index(c) for c in embed_ids if c in cat_nums] if embed_ids else list(range(len(cat)))
    hidden = [int(h) for h in (p.get("NumHiddenNodes") or [50])][: int(p.get("NumHiddenLayers", 1) or 1)]
    acts = list(p.get("ActivationFunc") or ["relu"])
    while len(acts) < len(hidden):
        acts.append(acts[-1])
    net = WideDeepNet(len(num), sizes, embed_fields, int(p.get("NumEmbedOuputs", p.get("EmbedOutputs", 8)) or 8),
                      hidden, acts[: len(hidden)])
    for prm in net.parameters():
        dist.broadcast_(prm.data, 0)
    l2 = float(p.get("WDLL2Reg", 0.0) or 0.0)
    trainer = WDLTrainer(net, step.dev, float(p.get("LearningRate", 0.1)), l2, str(p.get("Optimizer", "GD")))
    rows = WDLRows(X, num_pos, cat_pos, step.dev)
    _log.info("WDL trainer %d: %d rows on rank %d from %s (%s on the device), %s lr %g, L2 %g", tid, rows.n,
              dist.info().rank, "the NormalizedData cache" if src is not None else "the raw columns",
              "resident" if rows._resident is not None else ("streamed" if rows.dev.type == "cuda" else "host"),
              trainer.opt_name, trainer.lr, l2)
    s_tr = (w * np.asarray(sw_, np.float32) * np.asarray(tr_m, np.float32)).astype(np.float32)
    s_va = (w * np.asarray(va_m, np.float32)).astype(np.float32)
    n_tr, n_va = float(np.count_nonzero(np.asarray(tr_m) & (np.asarray(sw_) > 0))), float(np.count_nonzero(va_m))
    epochs = int(mc.train.get("numTrainEpochs", 100))
    verr = float("nan")
    for ep in range(1, epochs + 1):
        terr, verr = trainer.epoch(rows, yy, s_tr, s_va, n_tr, n_va)
        step._log_epoch(tid, ep, terr, verr)
    if step.info.rank == 0:
        from ..steps.train import nn_column_stats
        m = WDLModel(net.cpu(), mc.norm_type, nn_column_stats(mc, cols), [c.name for c in cols], cutoff)
        m.l2reg = l2
        write_wdl(ms.pf.model_path(tid, "wdl"), m)
    return verr
