"""SVM (legacy LOCAL algorithm, ``SVMTrainer`` J/core/alg/SVMTrainer.java:38-185).

The reference hands the training set to Encog's libsvm port: a C-SVC with the kernel named by
``params.Kernel`` (``linear`` / ``poly`` / ``sigmoid`` / ``rbf``, aliases at :51-61), cost
``params.Const`` and ``params.Gamma`` (defaults ``ModelTrainConf.createParamsByAlg`` :547-550:
linear, gamma 1.0, C 1.0), one SMO run to eps 1e-3 on the (bagged) training rows, validation
error = fraction of misclassified validation rows, model written as ``models/model<i>.svm``
(``EncogDirectoryPersistence``).  libsvm kernel definitions (degree 3, coef0 0):

    linear  u'v          poly  (gamma u'v + coef0)^degree
    rbf     exp(-gamma |u - v|^2)    sigmoid  tanh(gamma u'v + coef0)

MI355X design: the dual is solved by SMO with libsvm's second-order working-set selection
(WSS3, Fan/Chen/Lin 2005) over a kernel matrix that is computed ONCE as a GEMM on the device
(hipBLASLt through torch: the Gram matrix is a plain library GEMM) and kept resident in HBM
(fp32; ``shifu.svm.maxRows`` rows = 65536 -> 16 GB), so every SMO iteration is two column
reads + one fused gradient update + two arg-reductions on the GPU instead of libsvm's
per-iteration kernel-row recomputation and LRU cache.  Rows beyond ``maxRows`` are subsampled
(LOCAL-mode scale, like the reference's in-memory Encog data set).

Artifact: an Encog-EG-style text file with the libsvm model inside (``[SVM]`` sections with
the parameters and the libsvm ``svm_save_model`` text).  The reference ships no ``.svm``
fixture, so byte-level parity with Encog's writer is unpinned; ``read_svm`` reads this
framework's files back for scoring.
"""
from __future__ import annotations

import math
import os
import time

import numpy as np
import torch

KERNELS = {"leaner kernel": "linear", "linear": "linear", "poly kernel": "poly", "poly": "poly",
           "sigmoid kernel": "sigmoid", "sigmoid": "sigmoid", "radialbasisfunction": "rbf", "rbf": "rbf"}
LIBSVM_KERNEL_IDS = {"linear": 0, "poly": 1, "rbf": 2, "sigmoid": 3}
TAU = 1e-12
SMO_BATCH = 2048          # SMO iterations per GPU launch (svm_kernels.hip)


def kernel_name(k) -> str:
    name = KERNELS.get(str(k or "linear").strip().lower())
    if name is None:
        raise ValueError(f"unsupported SVM kernel {k!r} (linear, poly, sigmoid, rbf)")
    return name


def gram(A: torch.Tensor, B: torch.Tensor, kernel: str, gamma: float, degree: int = 3,
         coef0: float = 0.0, sw=None) -> torch.Tensor:
    """K[i, j] = k(A_i, B_j) (fp32, one GEMM + an elementwise map).  On the GPU the product is
    the own MFMA GEMM over split-bf16 operands at fp32 accuracy (ops/gemm_ops.py, 6 terms);
    ``sw``: B's split operand, built once by the caller for many row blocks of A."""
    if A.is_cuda:
        from ..ops.gemm_ops import SplitWeights, linear_fp32
        A = A.float().contiguous()
        sw = sw or SplitWeights(B.float(), None, 6)
        G = linear_fp32(A, B, sw=sw)
    else:
        G = A @ B.t()
    if kernel == "linear":
        return G
    if kernel == "poly":
        return (gamma * G + coef0) ** degree
    if kernel == "sigmoid":
        return torch.tanh(gamma * G + coef0)
    na = (A * A).sum(1, keepdim=True)
    nb = (B * B).sum(1, keepdim=True).t()
    return torch.exp(-gamma * (na + nb - 2.0 * G).clamp_min(0.0))


class SVMModel:
    def __init__(self, kernel, gamma, C, sv, coef, rho, labels, degree=3, coef0=0.0, eps=1e-3):
        self.kernel, self.gamma, self.C = kernel, float(gamma), float(C)
        self.sv = np.asarray(sv, np.float64)            # [nSV, F]
        self.coef = np.asarray(coef, np.float64)        # [nSV] y_i * alpha_i
        self.rho, self.labels = float(rho), list(labels)   # labels[0] <-> decision > 0
        self.degree, self.coef0, self.eps = int(degree), float(coef0), float(eps)

    @property
    def n_in(self) -> int:
        return int(self.sv.shape[1]) if self.sv.ndim == 2 else 0

    def decision(self, X, device=None) -> np.ndarray:
        dev = torch.device(device or "cpu")
        if len(self.coef) == 0:
            return np.full(len(X), -self.rho)
        Xt = torch.as_tensor(np.asarray(X, np.float32), device=dev)
        S = torch.as_tensor(self.sv.astype(np.float32), device=dev)
        out = []
        for r0 in range(0, len(Xt), 1 << 16):
            K = gram(Xt[r0:r0 + (1 << 16)], S, self.kernel, self.gamma, self.degree, self.coef0)
            out.append((K.double() @ torch.as_tensor(self.coef, device=dev)).cpu().numpy() - self.rho)
        return np.concatenate(out) if out else np.zeros(0)

    def predict(self, X, device=None) -> np.ndarray:
        """Class label per row (libsvm ``svm_predict``: labels[0] when the decision value > 0)."""
        d = self.decision(X, device)
        return np.where(d > 0, self.labels[0], self.labels[-1]).astype(np.float64)


def train_svm(X, y, kernel="linear", C=1.0, gamma=1.0, degree=3, coef0=0.0, eps=1e-3, weights=None,
              device=None, max_iter=None, log=None) -> SVMModel:
    """C-SVC dual by SMO/WSS3 on a device-resident kernel matrix.  ``y`` holds the class values
    (any two, e.g. 0/1); ``weights`` (bagging counts) scale each row's C (libsvm's per-instance
    weighting), 0 drops the row."""
    dev = torch.device(device or "cpu")
    X = np.asarray(X, np.float32)
    y = np.asarray(y, np.float64).reshape(-1)
    keep = np.ones(len(y), bool) if weights is None else np.asarray(weights) > 0
    X, y = X[keep], y[keep]
    cw = np.ones(len(y)) if weights is None else np.asarray(weights, np.float64)[keep]
    labels = []
    for v in y:                             # libsvm: labels in first-appearance order
        if v not in labels:
            labels.append(float(v))
    if len(labels) < 2:                     # one class: constant decision (libsvm: rho = -/+1)
        return SVMModel(kernel, gamma, C, np.zeros((0, X.shape[1])), np.zeros(0), -1.0, labels * 2,
                        degree, coef0, eps)
    if len(labels) > 2:
        raise ValueError("SVM: binary classification only (the reference trains SupportVectorClassification "
                         "on 0/1 ideals)")
    s = np.where(y == labels[0], 1.0, -1.0)
    n = len(s)
    Xd = torch.as_tensor(X, device=dev)
    K = torch.empty(n, n, dtype=torch.float32, device=dev)
    sw = None
    if dev.type == "cuda":
        from ..ops.gemm_ops import SplitWeights
        sw = SplitWeights(Xd.float(), None, 6)
    for r0 in range(0, n, 8192):
        K[r0:r0 + 8192] = gram(Xd[r0:r0 + 8192], Xd, kernel, gamma, degree, coef0, sw=sw)
    Y = torch.as_tensor(s, dtype=torch.float64, device=dev)
    Cv = torch.as_tensor(C * cw, dtype=torch.float64, device=dev)
    alpha = torch.zeros(n, dtype=torch.float64, device=dev)
    G = torch.full((n,), -1.0, dtype=torch.float64, device=dev)        # gradient of 0.5 a'Qa - e'a
    Kd = torch.diagonal(K).double().contiguous()
    inf = torch.tensor(float("inf"), dtype=torch.float64, device=dev)
    max_iter = max_iter or max(10_000_000, 100 * n)
    t0 = time.time()
    it = 0
    if dev.type == "cuda" and os.environ.get("SHIFU_SVM_HOST_LOOP") != "1":
        # ops/csrc/svm_kernels.hip: SMO_BATCH iterations per launch inside one workgroup, one host
        # synchronisation per batch (the convergence flag) instead of ~8 per iteration
        from ..ops import _native as nat
        state = torch.zeros(2, dtype=torch.int64, device=dev)
        gap = torch.zeros(1, dtype=torch.float64, device=dev)
        st = nat.stream_of(K)
        next_log = 20000
        while it < max_iter:
            k = int(min(SMO_BATCH, max_iter - it))
            nat.call_hip("shifu_svm_smo", K, n, Y, Cv, Kd, alpha, G, n, k, float(eps), TAU, state, gap, st)
            done, conv = (int(v) for v in state.cpu())
            it = done
            if conv:
                break
            if log is not None and it >= next_log:
                log(f"SVM SMO iteration {it}: gap {float(gap.item()):.3g} ({time.time() - t0:.1f}s)")
                next_log += 20000
    while it < max_iter and (dev.type != "cuda" or os.environ.get("SHIFU_SVM_HOST_LOOP") == "1"):
        # WSS3: i = argmax_{I_up} -y G ; j = argmin over I_low of the second-order gain
        up = ((Y > 0) & (alpha < Cv)) | ((Y < 0) & (alpha > 0))
        low = ((Y > 0) & (alpha > 0)) | ((Y < 0) & (alpha < Cv))
        mG = -Y * G
        gi = torch.where(up, mG, -inf)
        i = int(torch.argmax(gi))
        Gmax = float(gi[i])
        gl = torch.where(low, mG, inf)
        Gmin = float(gl.min())
        if Gmax - Gmin < eps:
            break
        Ki = K[i].double()
        b = Gmax - mG                                         # > 0 on the candidates
        a = (Kd[i] + Kd - 2.0 * Ki).clamp_min(TAU)           # |phi_i - phi_t|^2
        obj = torch.where(low & (b > 0), -(b * b) / a, inf)
        j = int(torch.argmin(obj))
        Kj = K[j].double()
        yi, yj = float(Y[i]), float(Y[j])
        ai, aj, Ci, Cj = float(alpha[i]), float(alpha[j]), float(Cv[i]), float(Cv[j])
        Gi, Gj = float(G[i]), float(G[j])
        Kii, Kjj, Kij = float(Kd[i]), float(Kd[j]), float(Ki[j])
        quad = max(Kii + Kjj - 2 * Kij, TAU)                 # Q_ii + Q_jj -/+ 2 Q_ij, either sign pair
        if yi != yj:
            delta = (-Gi - Gj) / quad
            diff = ai - aj
            ai += delta
            aj += delta
            if diff > 0 and aj < 0:
                aj, ai = 0.0, diff
            elif diff <= 0 and ai < 0:
                ai, aj = 0.0, -diff
            if diff > Ci - Cj and ai > Ci:
                ai, aj = Ci, Ci - diff
            elif diff <= Ci - Cj and aj > Cj:
                aj, ai = Cj, Cj + diff
        else:
            delta = (Gi - Gj) / quad
            sm = ai + aj
            ai -= delta
            aj += delta
            if sm > Ci and ai > Ci:
                ai, aj = Ci, sm - Ci
            elif sm <= Ci and aj < 0:
                aj, ai = 0.0, sm
            if sm > Cj and aj > Cj:
                aj, ai = Cj, sm - Cj
            elif sm <= Cj and ai < 0:
                ai, aj = 0.0, sm
        dai, daj = ai - float(alpha[i]), aj - float(alpha[j])
        # Q_ij = y_i y_j K_ij: G += Q[:, i] dai + Q[:, j] daj
        G += Y * (yi * dai * Ki + yj * daj * Kj)
        alpha[i], alpha[j] = ai, aj
        it += 1
        if log is not None and it % 20000 == 0:
            log(f"SVM SMO iteration {it}: gap {Gmax - Gmin:.3g} ({time.time() - t0:.1f}s)")
    # rho: mean of y G over free SVs (else the midpoint of the feasible interval)
    yG = (Y * G)
    free = (alpha > 0) & (alpha < Cv)
    if bool(free.any()):
        rho = float(yG[free].mean())
    else:
        ub_m = ((Y < 0) & (alpha >= Cv)) | ((Y > 0) & (alpha <= 0))
        lb_m = ((Y > 0) & (alpha >= Cv)) | ((Y < 0) & (alpha <= 0))
        ub = float(yG[ub_m].min()) if bool(ub_m.any()) else math.inf
        lb = float(yG[lb_m].max()) if bool(lb_m.any()) else -math.inf
        rho = (ub + lb) / 2 if math.isfinite(ub) and math.isfinite(lb) else (ub if math.isfinite(ub) else lb)
    sv = (alpha > 0).cpu().numpy()
    coef = (Y * alpha).cpu().numpy()[sv]
    if log is not None:
        log(f"SVM SMO: {it} iterations, {int(sv.sum())} support vectors, rho {rho:.6g} ({time.time() - t0:.1f}s)")
    return SVMModel(kernel, gamma, C, X[sv].astype(np.float64), coef, rho, labels, degree, coef0, eps)


# ---- artifact ---------------------------------------------------------------------------------
def _libsvm_text(m: SVMModel) -> str:
    lines = ["svm_type c_svc", f"kernel_type {['linear', 'polynomial', 'rbf', 'sigmoid'][LIBSVM_KERNEL_IDS[m.kernel]]}"]
    if m.kernel == "poly":
        lines.append(f"degree {m.degree}")
    if m.kernel in ("poly", "rbf", "sigmoid"):
        lines.append(f"gamma {m.gamma!r}")
    if m.kernel in ("poly", "sigmoid"):
        lines.append(f"coef0 {m.coef0!r}")
    npos = int((m.coef > 0).sum())
    lines += ["nr_class 2", f"total_sv {len(m.coef)}", f"rho {m.rho!r}",
              "label " + " ".join(str(int(l)) if float(l).is_integer() else repr(l) for l in m.labels[:2]),
              f"nr_sv {npos} {len(m.coef) - npos}", "SV"]
    order = np.argsort(m.coef <= 0, kind="stable")          # libsvm groups the SVs by class
    for k in order:
        feats = " ".join(f"{f + 1}:{float(v)!r}" for f, v in enumerate(m.sv[k]) if v != 0.0)
        lines.append(f"{float(m.coef[k])!r} {feats}".rstrip())
    return "\n".join(lines) + "\n"


def write_svm(path: str, m: SVMModel, input_count: int) -> None:
    body = [f"encog,SVM,java,3.0.0,1,{int(time.time() * 1000)}", "[SVM:PARAMS]", "[SVM:SVM-PARAM]",
            f"inputCount={input_count}", f"C={m.C!r}", "cacheSize=100.0", f"coef0={m.coef0!r}",
            f"degree={m.degree}", f"eps={m.eps!r}", f"gamma={m.gamma!r}",
            f"kernelType={LIBSVM_KERNEL_IDS[m.kernel]}", "nrWeight=0", "nu=0.5", "p=0.1", "probability=0",
            "shrinking=1", "svmType=0", "[SVM:SVM-MODEL]", _libsvm_text(m).rstrip("\n")]
    with open(path, "w") as f:
        f.write("\n".join(body) + "\n")


def read_svm(path: str) -> SVMModel:
    sec, params, model = None, {}, []
    for line in open(path):
        line = line.rstrip("\n")
        if line.startswith("[SVM:"):
            sec = line
            continue
        if sec == "[SVM:SVM-PARAM]" and "=" in line:
            k, v = line.split("=", 1)
            params[k] = v
        elif sec == "[SVM:SVM-MODEL]":
            model.append(line)
    hdr, svs, in_sv = {}, [], False
    for line in model:
        if in_sv:
            if line.strip():
                svs.append(line.split())
            continue
        if line == "SV":
            in_sv = True
            continue
        k, _, v = line.partition(" ")
        hdr[k] = v
    kernel = {"linear": "linear", "polynomial": "poly", "rbf": "rbf", "sigmoid": "sigmoid"}[hdr["kernel_type"]]
    F = int(params.get("inputCount", 0))
    sv = np.zeros((len(svs), F))
    coef = np.zeros(len(svs))
    for r, toks in enumerate(svs):
        coef[r] = float(toks[0])
        for t in toks[1:]:
            f, v = t.split(":")
            sv[r, int(f) - 1] = float(v)
    labels = [float(x) for x in hdr["label"].split()]
    return SVMModel(kernel, float(hdr.get("gamma", params.get("gamma", 1.0))), float(params.get("C", 1.0)), sv,
                    coef, float(hdr["rho"]), labels, int(hdr.get("degree", params.get("degree", 3))),
                    float(hdr.get("coef0", params.get("coef0", 0.0))), float(params.get("eps", 1e-3)))
