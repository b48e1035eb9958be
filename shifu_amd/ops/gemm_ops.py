"""fp32-accurate dense layers on the bf16 MFMA GEMM (``gemm_kernels.hip``, EPI_F32 tile).

``linear_fp32(x, W, b, act)`` = act(x @ W^T + b) for fp32 operands as ONE own-MFMA GEMM over
split-bf16 operands concatenated along K.  A value v is split into bf16 parts v = hi + mid + lo
(+ rest): hi = bf16(v), mid = bf16(v - hi), lo = bf16(v - hi - mid).  Products of bf16 parts are
exact in the fp32 accumulator, so summing the part pairs whose order is <= the kept order gives:

* ``terms=3``: hi*hi + hi*mid + mid*hi                   -- ~2^-17 relative (SE first layer)
* ``terms=6``: + hi*lo + lo*hi + mid*mid                  -- ~2^-24 relative: fp32 accuracy

(the same digit-split idea as K15's exact int8 correlation).  The bias rides along as extra
columns of ones in x against the bias parts in W.  The left operand is built by one HIP pass
(``shifu_split_bf16_rows``: read x once, write its parts per term); the GEMM's fp32 tile epilogue
applies the activation in its accurate libm form and writes C directly.  This is the default
``fp32`` NN scoring path (``scoring/model_runner.py``; the reference scores in float,
IndependentNNModel.java).  CPU tensors take the plain torch product (the oracle).
"""
from __future__ import annotations

import torch

from . import _native as nat

_PAIRS = {3: ((0, 0), (0, 1), (1, 0)),
          6: ((0, 0), (0, 1), (1, 0), (0, 2), (2, 0), (1, 1))}
ACT_LINEAR = 2


def split_bf16(v: torch.Tensor, parts: int):
    """[hi, mid, lo][:parts] bf16 tensors with v ~= sum(parts) (fp32 residual arithmetic)."""
    out, r = [], v.float()
    for _ in range(parts):
        p = r.to(torch.bfloat16)
        out.append(p)
        r = r - p.float()
    return out


def _pad(k: int, m: int) -> int:
    return (k + m - 1) // m * m


class SplitWeights:
    """The split-bf16 K-concatenated weight operand of one layer (built once, reused per chunk)."""

    def __init__(self, W: torch.Tensor, b: torch.Tensor | None, terms: int = 6):
        assert terms in _PAIRS
        self.terms = terms
        self.pairs = _PAIRS[terms]
        self.N, self.K = W.shape
        nparts = 1 + max(max(p) for p in self.pairs)
        wp = split_bf16(W, nparts)
        bp = split_bf16(b, nparts) if b is not None else None
        T = len(self.pairs)
        self.kb = T * self.K                                   # bias columns start here
        self.kp = _pad(self.kb + (T if b is not None else 0), 64)
        self.nh = _pad(self.N, 8)
        B = torch.zeros(self.N, self.kp, dtype=torch.bfloat16, device=W.device)
        for t, (_, wi) in enumerate(self.pairs):
            B[:, t * self.K:(t + 1) * self.K] = wp[wi]
            if bp is not None:
                B[:, self.kb + t] = bp[wi]
        self.B = B
        self.has_bias = b is not None
        self.nparts = nparts
        self.xsel = sum(xi << (2 * t) for t, (xi, _) in enumerate(self.pairs))
        self._A = None

    def operand(self, x: torch.Tensor) -> torch.Tensor:
        """[M, kp] bf16 left operand for the rows of x (buffer reused across chunks)."""
        M = x.shape[0]
        if self._A is None or self._A.shape[0] < M:
            self._A = torch.zeros(M, self.kp, dtype=torch.bfloat16, device=x.device)
            if self.has_bias:
                # the bias column of each term pair carries 1.0 against that pair's bias part
                for t, (xi, _) in enumerate(self.pairs):
                    self._A[:, self.kb + t] = 1.0 if xi == 0 else 0.0
        A = self._A[:M]
        if x.device.type == "cuda" and M:
            x = x.float()
            if x.stride(1) != 1:
                x = x.contiguous()
            nat.call_hip("shifu_split_bf16_rows", x, x.stride(0), M, self.K, A, self.kp, len(self.pairs),
                         self.xsel, nat.stream_of(x))
            return A
        xp = split_bf16(x, self.nparts)
        for t, (xi, _) in enumerate(self.pairs):
            A[:, t * self.K:(t + 1) * self.K] = xp[xi]
        return A


def linear_fp32(x: torch.Tensor, W: torch.Tensor, b: torch.Tensor | None = None, terms: int = 6,
                sw: SplitWeights | None = None, act: int = ACT_LINEAR) -> torch.Tensor:
    """act(x [M, K] @ W[N, K]^T + b), fp32 in / out (see module doc); ``act`` a models.nn.ACT_IDS
    id.  Returns an [M, N] view of an [M, roundup(N, 8)] buffer."""
    if x.device.type != "cuda":
        y = x.float() @ W.float().t()
        y = y + b.float() if b is not None else y
        if act != ACT_LINEAR:
            from ..models.nn import ACT_IDS, act_fwd
            y = act_fwd({v: k for k, v in ACT_IDS.items()}[act], y)
        return y
    sw = sw or SplitWeights(W, b, terms)
    A = sw.operand(x)
    M = x.shape[0]
    C = torch.empty(M, sw.nh, dtype=torch.float32, device=x.device)
    if M:
        nat.call_hip("shifu_gemm_nt", A, sw.kp, sw.B, sw.kp, sw.N, C, sw.nh, None, 0, None, 0, None, 0,
                     M, sw.nh, sw.kp, 3, act, sw.N, 0, 0.0, nat.stream_of(A))
    return C[:, :sw.N]
