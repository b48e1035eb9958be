"""Logistic regression engine (H9).

Semantics of ``LogisticRegressionWorker.doCompute`` (J/core/dtrain/lr/LogisticRegressionWorker.java:302-352)
and ``LogisticRegressionMaster`` (:227-299): p = sigmoid(w.x + b) (bias = last weight), ascent
gradient ``g_i += (y-p) x_i (p(1-p) + 0.1) s`` (the derivative-with-flat-spot variant), training
error = mean (y-p)^2 (unweighted), then the shared ``Weight`` update rules (RPROP by default).

MI355X mapping: the rows stay resident in HBM (bf16 when large); one epoch is ONE memory-bound
pass of the fused HIP kernel ``lr_grad_kernel`` (K9: dot, sigmoid, gradient accumulation in
registers, block partials) over the shard; then the [F+1(+2)] gradient buffer (with error/count
tail) is all-reduced over RCCL and every rank applies the identical optimizer step (no parameter
server).  The torch two-GEMV path is the CPU oracle.
"""
from __future__ import annotations

import numpy as np
import torch

from ..parallel import dist
from ..utils.log import get_logger
from .nn import Optimizer

_log = get_logger("models.lr")

FLAT_SPOT = 0.1


class LRTrainer:
    def __init__(self, n_in: int, device=None, propagation="R", learning_rate=0.1, reg=0.0, reg_level="NONE",
                 learning_decay=0.0, momentum=0.5, adam_beta1=0.9, adam_beta2=0.999, seed=0, init=None,
                 input_dtype: str | None = None):
        from ..config import environment
        from ..utils.device import default_device
        self.device = torch.device(device) if device is not None else default_device()
        # resident input rows: fp32 (the reference LR is double throughout, LogisticRegressionWorker
        # :302-352); "auto" keeps fp32 unless the fp32 rows would not fit in HBM, then stores bf16
        # rows (fp32 sums) and says so; "bf16" forces that mode (shifu.lr.inputDtype)
        self.input_dtype_request = str(input_dtype or environment.get("shifu.lr.inputDtype", "auto") or "auto").lower()
        if self.input_dtype_request not in ("auto", "fp32", "float32", "bf16", "bfloat16"):
            raise ValueError(f"shifu.lr.inputDtype must be auto, fp32 or bf16, not {self.input_dtype_request}")
        self.input_dtype = "fp32"
        self.n_in = n_in
        g = torch.Generator().manual_seed(seed)
        w = (torch.rand(n_in + 1, generator=g, dtype=torch.float32) - 0.5) if init is None else \
            torch.as_tensor(np.asarray(init, dtype=np.float32))
        self.w = w.to(self.device).contiguous()
        dist.broadcast_(self.w, 0)
        self.gbuf = torch.zeros(n_in + 1, dtype=torch.float32, device=self.device)
        self.opt = Optimizer(n_in + 1, self.device, propagation, learning_rate, momentum, adam_beta1, adam_beta2,
                             learning_decay, reg, reg_level, None)
        self.last_error = float("nan")

    def prepare(self, x, y, s=None):
        x = torch.as_tensor(x)
        n = x.shape[0]
        dt = self._row_dtype(n, x.shape[1])
        if self.device.type == "cuda":      # pad rows to a 16-byte multiple for the vector loads of K9
            fp = (x.shape[1] + 7) // 8 * 8
            xp = torch.zeros(n, fp, dtype=dt, device=self.device)
            xp[:, : x.shape[1]] = x.to(self.device, dt)
            xd = xp[:, : x.shape[1]]
        else:
            xd = x.to(self.device, dt).contiguous()
        yd = torch.as_tensor(y, dtype=torch.float32).reshape(n).to(self.device)
        sd = torch.ones(n, device=self.device) if s is None else \
            torch.as_tensor(s, dtype=torch.float32).reshape(n).to(self.device)
        return xd, yd, sd

    def _row_dtype(self, n: int, f: int) -> torch.dtype:
        req = self.input_dtype_request
        if self.device.type != "cuda" or req in ("fp32", "float32"):
            self.input_dtype = "fp32"
            return torch.float32
        if req in ("bf16", "bfloat16"):
            self.input_dtype = "bf16"
        else:
            from ..utils.device import free_hbm
            fp32_bytes = n * ((f + 7) // 8 * 8) * 4
            self.input_dtype = "bf16" if fp32_bytes > 0.8 * free_hbm(self.device) else "fp32"
        if self.input_dtype == "bf16":
            _log.warning("LR: %d x %d input rows kept as bf16 in HBM (fp32 rows: %.1f GB); dot products and "
                         "gradient sums stay fp32 (shifu.lr.inputDtype=%s)", n, f, n * f * 4 / 1e9, req)
            return torch.bfloat16
        return torch.float32

    def _score(self, x):
        if x.is_cuda:                          # own row-dot kernel (wdl_kernels.hip)
            from ..ops import stats_ops
            return torch.sigmoid(stats_ops.rowdot(x, self.w[:-1]) + self.w[-1])
        z = (x @ self.w[:-1].to(x.dtype)).float() + self.w[-1]
        return torch.sigmoid(z)

    def step(self, data, chunk: int = 1 << 22) -> float:
        x, y, s = data
        g = self.gbuf
        g.zero_()
        # [error sum, row count] in fp64 (an fp32 count rounds past 2^24 rows)
        tail = torch.zeros(2, dtype=torch.float64, device=self.device)
        if self.device.type == "cuda":
            from ..ops import stats_ops           # fused HIP pass (K9): dot + sigmoid + gradient
            r = stats_ops.lr_grad(x, self.w, y, s)
            if r is not None:
                g[: self.n_in + 1] = r[0]
                tail[0] = r[1].double()
                chunk = 0
        for r0 in (range(0, x.shape[0], chunk) if chunk else ()):
            xb, yb, sb = x[r0: r0 + chunk], y[r0: r0 + chunk], s[r0: r0 + chunk]
            p = self._score(xb)
            e = yb - p
            d = e * (p * (1 - p) + FLAT_SPOT) * sb
            if xb.is_cuda:                     # above K9's feature limit: own column-dot kernel
                from ..ops import stats_ops
                g[: self.n_in] += stats_ops.coldot(d, xb)
            else:
                g[: self.n_in] += (d.to(xb.dtype) @ xb).float()
            g[self.n_in] += d.sum()
            tail[0] += (e.double() * e.double()).sum()
        tail[1] = float(x.shape[0])
        dist.all_reduce_(g[: self.n_in + 1])
        dist.all_reduce_(tail)
        n = float(tail[1].item())
        self.opt.step(self.w, g[: self.n_in + 1], n)
        self.last_error = float(tail[0].item()) / max(n, 1.0)
        return self.last_error

    @torch.no_grad()
    def evaluate(self, data) -> float:
        x, y, s = data
        e = (self._score(x) - y)
        t = torch.tensor([float((e * e).sum()), float(x.shape[0])], dtype=torch.float64, device=self.device)
        dist.all_reduce_(t)
        return float(t[0] / max(t[1], 1.0))

    @torch.no_grad()
    def predict(self, x) -> torch.Tensor:
        return self._score(torch.as_tensor(x).to(self.device, torch.float32))

    def weights(self) -> np.ndarray:
        return self.w.detach().cpu().double().numpy()


def write_lr(path: str, weights) -> None:
    """``.lr`` text: ``[w0, w1, ..., bias]`` (``LR.toString`` / ``LR.loadFromString`` J/core/LR.java:43-105)."""
    with open(path, "w") as f:
        f.write("[" + ", ".join(repr(float(v)) for v in weights) + "]")


def read_lr(path: str) -> np.ndarray:
    txt = open(path).read().replace("[", "").replace("]", "")
    return np.array([float(t) for t in txt.split(",") if t.strip()], dtype=np.float64)


def lr_score(weights: np.ndarray, x: np.ndarray) -> np.ndarray:
    z = np.asarray(x, dtype=np.float64) @ weights[:-1] + weights[-1]
    return 1.0 / (1.0 + np.exp(-z))
