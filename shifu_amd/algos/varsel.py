"""Variable selection (H13).

* filter: KS / IV / mix / pareto ranking up to ``filterNum`` (or ``filterOutRatio``),
  ForceSelect always in, ForceRemove/meta/target/bad candidates out
  (``VariableSelector.selectByFilter`` J/core/VariableSelector.java:110-286).
* auto filter: missing rate >= threshold, IV/KS below minimum, and for each highly correlated
  pair drop the column with the lower ``postCorrelationMetric``
  (``VarSelectModelProcessor.autoVarSelCondition`` :1008-1050, ``varSelectByCorrelation`` :1052).
* sensitivity SE/ST (``VarSelectMapper.map`` J/core/varselect/VarSelectMapper.java:277-333 with
  ``CacheFlatNetwork`` first-layer caching): for every row and input i the score with input i
  zeroed is ``net(S - w_i x_i)``; accumulate sum|d| and sum d^2 -> mean / RMS / variance and keep
  the top by RMS (SE) or by mean (ST).  On the GPU the perturbed first layer for a feature chunk
  is one batched tensor op over the cached S (the dominant cost for 10k features).
* voted: genetic wrapper (``CandidateGenerator`` inherit / hybrid / mutate) scored by small NNs.
"""
from __future__ import annotations

import os

import math

import numpy as np
import torch

from ..utils.log import get_logger

_log = get_logger("algos.varsel")


def _candidates(mc, ccs):
    from ..config.column_config import has_candidates
    hc = has_candidates(ccs)
    cand_names = set(mc.candidate_names())
    out, forced = [], []
    for c in ccs:
        if c.is_meta() or c.is_target() or c.is_force_remove() or c.is_weight():
            continue
        if c.is_force_select():
            if c.mean is not None and c.std_dev is not None:
                forced.append(c)
            continue
        if not c.is_good_candidate(hc, mc.is_binary()):
            continue
        if cand_names and c.name not in cand_names:
            continue
        out.append(c)
    return out, forced


def pareto_sort(tuples, epsilons=None):
    """``VariableSelector.sortByPareto`` (J/core/VariableSelector.java:296-404): an epsilon-box
    archive over (ks, iv) tuples ``(num, ks, iv)`` in the reference's orientation (smaller box
    coordinates dominate; same box -> the one nearer the box corner stays); ``epsilons`` from
    ``varSelect.epsilons`` (default [0.01, 0.05]).  Returns the archive in insertion order."""
    eps = list(epsilons) if epsilons else [0.01, 0.05]
    arch = []                                  # [(box, tuple)]
    for t in tuples:
        vals = (t[1], t[2])
        ebox = [math.floor((vals[0] if i == 0 else vals[1]) / e) for i, e in enumerate(eps)]
        idx, keep = 0, True
        while idx < len(arch):
            abox, at = arch[idx]
            adom = sdom = nondom = False
            for i in range(len(eps)):
                if abox[i] < ebox[i]:
                    adom = True
                    if sdom:
                        nondom = True
                        break
                elif abox[i] > ebox[i]:
                    sdom = True
                    if adom:
                        nondom = True
                        break
            if nondom:
                idx += 1
                continue
            if adom:
                keep = False
                break
            if sdom:
                del arch[idx]
                continue
            corner = [b * e for b, e in zip(ebox, eps)]
            sd = sum(((vals[0] if j == 0 else vals[1]) - corner[j]) ** 2 for j in range(len(eps)))
            ad = sum(((at[1] if j == 0 else at[2]) - corner[j]) ** 2 for j in range(len(eps)))
            if ad < sd:
                keep = False
                break
            del arch[idx]
        if keep:
            arch.append((ebox, t))
    return [t for _, t in arch]


def select_by_filter(mc, ccs):
    vs = mc.varSelect
    cands, forced = _candidates(mc, ccs)
    selected = [c.num for c in forced]
    if not vs.get("filterEnable", True):
        for c in ccs:
            c.final_select = c.num in selected
        return ccs
    key = str(vs.get("filterBy", "KS")).lower()
    filter_num = int(vs.get("filterNum", 200))
    ratio = vs.get("filterOutRatio")
    if filter_num <= 0 and ratio is not None:   # setFilterNumberByFilterOutRatio
        filter_num = int(len(cands) * (1 - float(ratio)))
    ks_list = sorted(cands, key=lambda c: -(c.ks or 0.0))
    iv_list = sorted(cands, key=lambda c: -(c.iv or 0.0))
    par = pareto_sort([(c.num, c.ks or 0.0, c.iv or 0.0) for c in cands], mc.varSelect.get("epsilons"))
    expected = min(len(selected) + len(ks_list), filter_num)
    for c in ccs:
        c.final_select = False
    pk = pi = pp = 0
    sel = list(selected)
    guard = 0
    while len(sel) < expected and guard < 10 * (len(cands) + 1):
        guard += 1
        if key == "iv":
            sel.append(iv_list[pi].num); pi += 1
        elif key == "mix":
            if pk < len(ks_list):
                c = ks_list[pk]; pk += 1
                if c.num not in sel:
                    sel.append(c.num)
            if len(sel) >= expected:
                break
            if pi < len(iv_list):
                c = iv_list[pi]; pi += 1
                if c.num not in sel:
                    sel.append(c.num)
        elif key == "pareto":
            if pp < len(par):
                sel.append(par[pp][0]); pp += 1
            else:
                c = ks_list[pk]; pk += 1
                if c.num not in sel:
                    sel.append(c.num)
        else:   # ks (default)
            sel.append(ks_list[pk].num); pk += 1
    bynum = {c.num: c for c in ccs}
    for n in sel:
        if n in bynum:
            bynum[n].final_select = True
    return ccs


def auto_filter(mc, ccs, corr: np.ndarray | None = None, corr_nums=None):
    """Returns the list of auto-filtered column names (and sets finalSelect False)."""
    vs = mc.varSelect
    if not vs.get("autoFilterEnable", True):
        return []
    miss_thr = float(vs.get("missingRateThreshold", 0.98))
    min_iv = float(vs.get("minIvThreshold", 0.0))
    min_ks = float(vs.get("minKsThreshold", 0.0))
    corr_thr = float(vs.get("correlationThreshold", 1.0))
    metric = str(vs.get("postCorrelationMetric", "IV")).upper()
    filtered = []
    for c in ccs:
        if not c.final_select or c.is_force_select():
            continue
        mp = c.missing_pct
        if mp is not None and mp >= miss_thr:
            c.final_select = False
            filtered.append(c.name)
            continue
        if mc.is_binary():
            if (c.iv or 0.0) < min_iv or (c.ks or 0.0) < min_ks:
                c.final_select = False
                filtered.append(c.name)
    if corr is not None and corr_thr < 1.0:
        idx = {n: i for i, n in enumerate(corr_nums)}
        sel = [c for c in ccs if c.final_select and c.num in idx]
        val = (lambda c: c.iv or 0.0) if metric == "IV" else (lambda c: c.ks or 0.0)
        sel.sort(key=lambda c: -val(c))
        kept = []
        for c in sel:
            if any(abs(corr[idx[c.num], idx[k.num]]) > corr_thr for k in kept):
                if not c.is_force_select():
                    c.final_select = False
                    filtered.append(c.name)
                    continue
            kept.append(c)
    return filtered


@torch.no_grad()
def first_layer_fp32(xb: torch.Tensor, W1: torch.Tensor, b1: torch.Tensor, fl_cache: dict | None = None):
    """S = X W1^T + b1 in fp32.  GPU: ONE own-MFMA GEMM (gemm_kernels.hip, EPI_F32 tile) over
    split-bf16 operands concatenated along K (``ops/gemm_ops.linear_fp32``, the 6 part products
    hi*hi, hi*mid, mid*hi, hi*lo, lo*hi, mid*mid, exact in the fp32 accumulator): fp32-accurate, as
    eval scoring, so near-tied SE scores rank as the reference's float computation does (3 terms,
    ~2^-17 relative, could reorder them).  ``fl_cache`` keeps the split weights and the operand buffer across
    row chunks."""
    if xb.device.type != "cuda":
        return xb @ W1.t() + b1
    from ..ops.gemm_ops import SplitWeights, linear_fp32
    fl_cache = {} if fl_cache is None else fl_cache
    if fl_cache.get("sw") is None:
        fl_cache["sw"] = SplitWeights(W1, b1, terms=6)
    sw = fl_cache["sw"]
    # the split operand is 6 x K bf16 per row (~120 KB at 10k inputs): at most ~4 GB of it at once
    step = max(4096, (4 << 30) // (sw.kp * 2))
    if xb.shape[0] <= step:
        return linear_fp32(xb, W1, b1, sw=sw)
    out = torch.empty(xb.shape[0], sw.N, dtype=torch.float32, device=xb.device)
    for r0 in range(0, xb.shape[0], step):
        out[r0: r0 + step] = linear_fp32(xb[r0: r0 + step], W1, b1, sw=sw)
    return out


def sensitivity(network, X, y=None, w=None, device=None, feat_chunk: int = 64, row_chunk: int = 1 << 16,
                deep_rows: int = 2048):
    """SE sensitivity over inputs of a trained MLP (NNNetwork, input-first weights).

    ``VarSelectMapper.map`` (J/core/varselect/VarSelectMapper.java:277-333) with
    ``CacheFlatNetwork`` (J/core/dtrain/nn/CacheFlatNetwork.java:117-180): the first-layer
    pre-activation S = X W1^T + b is computed once per row, an input's removal is the rank-1
    correction S - x_f W1[:, f], and only the layers above are re-evaluated.  Returns
    (mean |d|, rms, variance) per input, accumulated over rows.

    ``X``: device tensor, host array, or :class:`models.nn.HostRows` (rows streamed to HBM on a
    copy stream that overlaps the SE kernels).  GPU paths:
    * 1 hidden layer (K14, ``sensitivity_kernel``): correction + activation + output neuron
      fused, register-blocked (the v_exp/v_rcp issue rate bounds it -- see profiles/);
    * deeper nets (K14b): ``se_perturb_kernel`` writes the perturbed first hidden layer of every
      (row, input) pair as bf16 MLP rows, the remaining layers run as the framework's own bf16
      MFMA GEMMs (``shifu_gemm_nt``, fp32 accumulation) over R x feat_chunk pair rows at a time;
    * both: the cached first layer S is one own-MFMA GEMM over split-bf16 operands with an fp32
      tile epilogue (``first_layer``), fp32-accurate to ~2^-17.
    CPU: the fp32 torch oracle of the same decomposition."""
    from ..models.nn import ACT_IDS, HostRows, act_fwd
    dev = torch.device(device) if device is not None else \
        (torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
    Ws = [torch.as_tensor(W, dtype=torch.float32, device=dev) for W in network.weights]
    acts = network.acts
    n_rows, F = (len(X), X.shape[1]) if not isinstance(X, HostRows) else X.shape
    s_abs = torch.zeros(F, dtype=torch.float64, device=dev)
    s_sq = torch.zeros(F, dtype=torch.float64, device=dev)
    n = 0
    W1 = Ws[0][:, :-1]          # [H1, F]
    b1 = Ws[0][:, -1]

    def row_chunks(rc):
        """device fp32 [m, F] row blocks (HostRows: pinned staging + H2D on a copy stream)."""
        if isinstance(X, HostRows):
            k0 = ((F + 1 + 127) // 128) * 128
            sub = max(4096, min(rc, (8 << 30) // (4 * F)))     # fp32 blocks of <= ~8 GB
            for _, _, xd in X.chunks(0, n_rows, rc, k0, dev):
                for s0 in range(0, xd.shape[0], sub):
                    yield xd[s0: s0 + sub, :F].float()
            return
        for r0 in range(0, n_rows, rc):
            xb = X[r0: r0 + rc]
            yield (xb if torch.is_tensor(xb) else torch.as_tensor(np.asarray(xb), dtype=torch.float32)).to(
                dev, dtype=torch.float32).contiguous()

    fl_cache = {}

    def first_layer(xb):
        return first_layer_fp32(xb, W1, b1, fl_cache)


    def tail(z1):
        a = act_fwd(acts[0], z1)
        for l in range(1, len(Ws)):
            a = act_fwd(acts[l], a @ Ws[l][:, :-1].t() + Ws[l][:, -1])
        return a[..., 0]

    if dev.type == "cuda" and len(Ws) == 2 and Ws[1].shape[0] == 1 and W1.shape[0] <= 1024:
        # K14: S cached per row, rank-1 correction + activation + output neuron fused
        from ..ops import stats_ops
        from ..ops import _native as nat
        acc = torch.zeros(F, 2, dtype=torch.float64, device=dev)
        W1t = W1.t().contiguous()
        W2 = Ws[1][0, :-1].float().contiguous()
        b2 = float(Ws[1][0, -1])
        for xb in row_chunks(row_chunk * 16):
            S = first_layer(xb).contiguous()
            base = torch.empty(S.shape[0], dtype=torch.float32, device=dev)
            nat.call_hip("shifu_rowdot_f32_act", S, S.stride(0), S.shape[0], S.shape[1], W2, b2, ACT_IDS[acts[0]],
                         ACT_IDS[acts[1]], base, nat.stream_of(S))
            stats_ops.sensitivity_1h(S, xb, W1t, W2, b2, base, ACT_IDS[acts[0]], ACT_IDS[acts[1]], acc)
            n += xb.shape[0]
        s_abs, s_sq = acc[:, 0], acc[:, 1]
    elif dev.type == "cuda" and Ws[-1].shape[0] == 1:
        # K14b: perturbed first layer as bf16 rows -> MFMA GEMM tail
        from ..ops import stats_ops
        from ..ops import _native as nat
        H1 = W1.shape[0]
        pad64 = lambda k: ((k + 63) // 64) * 64
        hpad = pad64(H1 + 1)
        W1t = W1.t().contiguous()
        Wb = [W.to(torch.bfloat16) for W in Ws]
        # own MFMA GEMMs (gemm_kernels.hip shifu_gemm_nt, EPI_ACT): each layer's activation, bias
        # column and zero padding are written by the GEMM epilogue as the next layer's bf16 rows;
        # W_l padded to [out_l, pad64(in_l + 1)] with the bias weight at column in_l (the Encog
        # flat layout).  SHIFU_SE_TAIL=torch: the previous torch bf16 matmul + cat tail.
        hip_tail = os.environ.get("SHIFU_SE_TAIL", "hip") != "torch"
        Wp, kin = [None], [hpad]
        for l in range(1, len(Ws)):
            o, i1 = Ws[l].shape
            w = torch.zeros(o, pad64(i1), dtype=torch.bfloat16, device=dev)
            w[:, :i1] = Wb[l]
            Wp.append(w)
            kin.append(pad64(o + 1) if l < len(Ws) - 1 else 64)
        bufs = {}

        def tail_bf16(A):                         # A [M, hpad] bf16 rows with bias column
            if hip_tail:
                M = A.shape[0]
                st = nat.stream_of(A)
                for l in range(1, len(Ws)):
                    if l == len(Ws) - 1:          # output neuron: fp32 dot over the bf16 rows (a
                        k = Ws[l].shape[1]        # bf16-rounded output would put a noise floor on d)
                        z = torch.empty(M, dtype=torch.float32, device=dev)
                        nat.call_hip("shifu_rowdot_bf16", A, A.stride(0), M, k, Ws[l][0].float().contiguous(), z, st)
                        return act_fwd(acts[l], z)
                    last = False
                    N, act = kin[l], ACT_IDS[acts[l]]
                    key = (l, M)
                    if key not in bufs:
                        bufs[key] = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
                    C = bufs[key]
                    C2 = None
                    if act in (5, 8):             # swish / sin: derivative not derivable from output
                        C2 = bufs.setdefault(("d", l, M), torch.empty(M, N, dtype=torch.bfloat16, device=dev))
                    nat.call_hip("shifu_gemm_nt", A, kin[l - 1], Wp[l], kin[l - 1], Ws[l].shape[0], C, N, C2, N,
                                 None, 0, None, 0, M, N, kin[l - 1], 0, act, Ws[l].shape[0], 0 if last else 1, 0.0,
                                 st)
                    A = C
                return A[:, 0].float()
            k = H1 + 1
            for l in range(1, len(Ws)):
                z = (A[:, :k] @ Wb[l].t()).float()
                a = act_fwd(acts[l], z)
                if l == len(Ws) - 1:
                    return a[:, 0]
                k = a.shape[1] + 1
                A = torch.cat([a, torch.ones(a.shape[0], 1, device=a.device)], 1).to(torch.bfloat16)
            return A[:, 0].float()
        act1 = ACT_IDS[acts[0]]
        for xb in row_chunks(deep_rows):
            R = xb.shape[0]
            S = first_layer(xb).contiguous()
            # unperturbed rows through the same kernel (x_f = 0 correction): base and perturbed
            # activations share rounding, so an input with x_f = 0 gives d = 0 exactly
            base = tail_bf16(stats_ops.se_perturb(S, torch.zeros(R, 1, device=dev), W1t[:1], 0, 1, act1, hpad))
            buf = torch.empty(R * feat_chunk, hpad, dtype=torch.bfloat16, device=dev)
            for f0 in range(0, F, feat_chunk):
                fc = min(feat_chunk, F - f0)
                P = stats_ops.se_perturb(S, xb, W1t, f0, fc, act1, hpad, buf[: R * fc])
                d = (base[:, None] - tail_bf16(P).view(R, fc)).double()
                s_abs[f0:f0 + fc] += d.abs().sum(0)
                s_sq[f0:f0 + fc] += (d * d).sum(0)
            n += R
    else:
        for xb in row_chunks(row_chunk):
            S = xb @ W1.t() + b1                     # cached first layer [R, H1]
            base = tail(S)                           # [R]
            for f0 in range(0, F, feat_chunk):
                f1 = min(F, f0 + feat_chunk)
                Z = S[:, None, :] - xb[:, f0:f1, None] * W1.t()[None, f0:f1, :]   # [R, fc, H1]
                d = (base[:, None] - tail(Z)).double()
                s_abs[f0:f1] += d.abs().sum(0)
                s_sq[f0:f1] += (d * d).sum(0)
            n += xb.shape[0]
    from ..parallel import dist
    if dist.info().world_size > 1:        # row-sharded SE: one all-reduce of the per-input sums
        t = torch.cat([s_abs, s_sq, torch.tensor([float(n)], dtype=torch.float64, device=s_abs.device)])
        dist.all_reduce_(t)
        s_abs, s_sq, n = t[:F], t[F:2 * F], int(t[-1].item())
    mean = (s_abs / max(n, 1)).cpu().numpy()
    rms = torch.sqrt(s_sq / max(n, 1)).cpu().numpy()
    var = (s_sq / max(n, 1)).cpu().numpy() - mean ** 2
    return mean, rms, var


def select_by_sensitivity(ccs, input_cols, mean, rms, keep: int, by: str = "SE"):
    """Keep the top ``keep`` inputs by RMS (SE) or mean (ST); force-selected always kept."""
    order = np.argsort(-(rms if by.upper() == "SE" else mean), kind="stable")
    keep_nums = {input_cols[i].num for i in order[:keep]}
    for c in ccs:
        if c.final_select and not c.is_force_select():
            c.final_select = c.num in keep_nums
    return [(input_cols[i].name, float(mean[i]), float(rms[i])) for i in order]
