"""Encog-compatible MLP trainer (Shifu ``NN`` algorithm) on MI355X.

Semantics follow the reference:
  * network generation  ``DTrainUtils.generateNetwork``  (J/core/dtrain/DTrainUtils.java:303-386):
    hidden activations from ``ActivationFunc``; output layer sigmoid for classification,
    linear/relu/leakyrelu/swish for a linear target; every layer receives a bias neuron.
  * gradient            ``SubGradient.process/processLevel`` (J/core/dtrain/nn/SubGradient.java:224-311):
    delta = (ideal-actual)·(f'(out)+flatSpot)·significance, gradients are *ascent* directions
    summed (not averaged) over all rows; flat spot 0.1 only for sigmoid layers
    (J/core/dtrain/nn/AbstractNNWorker.java:605-609).
  * update              ``Weight.calculateWeights`` (J/core/dtrain/Weight.java:194-343) - every rule adds.
  * error               squared error averaged over records x outputs
    (J/core/dtrain/nn/ParallelGradient.java:206-211).
  * iteration 1 of the reference only syncs weights (J/core/dtrain/nn/AbstractNNWorker.java:525-527);
    here initial weights are broadcast from rank 0 once at construction instead.

MI355X design (not a translation): the whole local shard stays resident in HBM as bf16
rows padded to a multiple of 128 columns with the bias neuron as a real column, each epoch
streams it in row chunks through the hand-written MFMA kernels in ``ops/csrc/mlp_kernels.hip``
(fused forward+activation, fused output/loss/delta row kernel, dgrad with fused derivative,
TN wgrad via ``ds_read_b64_tr_b16``), sums the gradient in one fp32 buffer, all-reduces it once
over RCCL with the error scalars in its tail, and applies the optimizer in one fused kernel on
every rank (replicated optimizer, no parameter server).
"""
from __future__ import annotations

import math
import time
import os
from dataclasses import dataclass, field

import numpy as np
import torch

from ..parallel import dist
from ..utils.trace import trace_range
from ..utils.log import get_logger

_log = get_logger("models.nn")

ACT_IDS = {"sigmoid": 0, "tanh": 1, "linear": 2, "relu": 3, "leakyrelu": 4, "swish": 5,
           "ptanh": 6, "log": 7, "sin": 8,
           "leakyrelu_tf": 9}          # tf.nn.leaky_relu, alpha 0.2 (TENSORFLOW algorithm)
ACT_DERIV_FROM_OUTPUT = {0, 1, 2, 3, 4, 6, 7, 9}
LOSS_IDS = {"squared": 0, "log": 1, "absolute": 2}
RULE_IDS = {"B": 0, "Q": 1, "M": 2, "R": 3, "ADAM": 4, "ADAGRAD": 5, "RMSPROP": 6,
            "MOMENTUM": 7, "NESTEROV": 8}
PAD = 128


def round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def norm_act(name: str) -> str:
    n = (name or "sigmoid").strip().lower()
    return n if n in ACT_IDS else "sigmoid"   # DTrainUtils: unknown -> sigmoid


# ------------------------------------------------------------------------------------------
# activation math (torch, fp32) - the CPU oracle of common.h
# ------------------------------------------------------------------------------------------
def act_fwd(act: str, z: torch.Tensor) -> torch.Tensor:
    if act == "sigmoid":
        return torch.sigmoid(z)
    if act == "tanh":
        return torch.tanh(z)
    if act == "linear":
        return z
    if act == "relu":
        return torch.where(z <= 0, torch.zeros_like(z), z)
    if act == "leakyrelu":
        return torch.where(z <= 0, 0.01 * z, z)
    if act == "leakyrelu_tf":
        return torch.where(z <= 0, 0.2 * z, z)
    if act == "swish":
        return z * torch.sigmoid(z)
    if act == "ptanh":
        t = torch.tanh(z)
        return torch.where(z > 0, t, 0.25 * t)
    if act == "log":
        return torch.where(z >= 0, torch.log1p(z.clamp(min=0)), -torch.log1p((-z).clamp(min=0)))
    if act == "sin":
        return torch.sin(z)
    raise ValueError(act)


def act_deriv(act: str, z: torch.Tensor, a: torch.Tensor) -> torch.Tensor:
    if act == "sigmoid":
        return a * (1 - a)
    if act == "tanh":
        return 1 - a * a
    if act == "linear":
        return torch.ones_like(a)
    if act == "relu":
        return (z > 0).to(a.dtype)
    if act == "leakyrelu":
        return torch.where(z <= 0, torch.full_like(a, 0.01), torch.ones_like(a))
    if act == "leakyrelu_tf":
        return torch.where(z <= 0, torch.full_like(a, 0.2), torch.ones_like(a))
    if act == "swish":
        s = torch.sigmoid(z)
        return s + z * s * (1 - s)
    if act == "ptanh":
        return torch.where(z > 0, 1 - a * a, 0.25 * (1 - 16 * a * a))
    if act == "log":
        return torch.where(z >= 0, 1 / (1 + z.clamp(min=0)), 1 / (1 - z.clamp(max=0)))
    if act == "sin":
        return torch.cos(z)
    raise ValueError(act)


def flat_spot(act: str) -> float:
    return 0.1 if act == "sigmoid" else 0.0


@dataclass
class MLPSpec:
    n_in: int
    hidden: list = field(default_factory=lambda: [50])
    acts: list = field(default_factory=lambda: ["tanh"])
    n_out: int = 1
    out_act: str = "sigmoid"          # "sigmoid" (classification) or linear/relu/leakyrelu/swish
    loss: str = "squared"
    flat: bool = True                 # Encog's sigmoid flat spot (+0.1 on f'); False for TENSORFLOW
    tf_objective: bool = False        # error sums = the TF objective sum(w * loss) (same deltas)

    def __post_init__(self):
        self.hidden = [int(h) for h in self.hidden]
        acts = [norm_act(a) for a in (self.acts or [])]
        while len(acts) < len(self.hidden):
            acts.append(acts[-1] if acts else "sigmoid")
        self.acts = acts[: len(self.hidden)]
        self.out_act = norm_act(self.out_act)
        self.loss = (self.loss or "squared").lower()
        if self.loss not in LOSS_IDS:
            self.loss = "squared"

    @property
    def loss_id(self) -> int:       # kernel loss code: 0-2 Encog error, 3-5 TF objective
        return LOSS_IDS[self.loss] + (3 if self.tf_objective else 0)

    @property
    def layer_in(self):             # logical input width of each weight layer
        return [self.n_in] + self.hidden

    @property
    def layer_out(self):
        return self.hidden + [self.n_out]

    @property
    def layer_kpad(self):           # padded input width incl. bias column
        return [round_up(i + 1, PAD) for i in self.layer_in]

    def flat_spot(self, act: str) -> float:
        return flat_spot(act) if self.flat else 0.0

    def n_weights_encog(self) -> int:
        return sum(o * (i + 1) for i, o in zip(self.layer_in, self.layer_out))


class MLPParams:
    """Flat fp32 parameter buffer with per-layer [out, in_pad] views (bias = column ``in``)."""

    def __init__(self, spec: MLPSpec, device, dtype=torch.float32):
        self.spec = spec
        self.shapes = [(o, k) for o, k in zip(spec.layer_out, spec.layer_kpad)]
        self.offsets = []
        off = 0
        for o, k in self.shapes:
            self.offsets.append(off)
            off += o * k
        self.numel = off
        self.flat = torch.zeros(off, dtype=dtype, device=device)

    def views(self, flat=None):
        flat = self.flat if flat is None else flat
        return [flat[off: off + o * k].view(o, k) for off, (o, k) in zip(self.offsets, self.shapes)]

    def valid_mask(self) -> torch.Tensor:
        """1 for real weights (incl. bias column), 0 for padding."""
        m = torch.zeros(self.numel, dtype=torch.bool)
        for off, (o, k), i in zip(self.offsets, self.shapes, self.spec.layer_in):
            m[off: off + o * k].view(o, k)[:, : i + 1] = True
        return m

    # ---- Encog flat layout (J/core/dtrain/dataset/FloatFlatNetwork.java:148-178) -----------
    # layers output-first; block for (to=layer l+1 neurons, from=layer l incl. bias) is
    # row-major [to][from+1], bias weight last.
    def to_encog_flat(self) -> np.ndarray:
        ws = self.views()
        out = []
        for l in reversed(range(len(ws))):
            i = self.spec.layer_in[l]
            out.append(ws[l][:, : i + 1].detach().double().cpu().numpy().reshape(-1))
        return np.concatenate(out)

    def from_encog_flat(self, flat: np.ndarray) -> None:
        flat = np.asarray(flat, dtype=np.float64)
        assert flat.size == self.spec.n_weights_encog(), (flat.size, self.spec.n_weights_encog())
        ws = self.views()
        pos = 0
        with torch.no_grad():
            self.flat.zero_()
            for l in reversed(range(len(ws))):
                i, o = self.spec.layer_in[l], self.spec.layer_out[l]
                blk = torch.from_numpy(flat[pos: pos + o * (i + 1)].reshape(o, i + 1)).to(self.flat)
                ws[l][:, : i + 1].copy_(blk)
                pos += o * (i + 1)

    def init_random(self, seed: int = 0, method: str = "default") -> None:
        """Weight initialisers of ``DTrainUtils.generateNetwork`` (default / gaussian / xavier /
        he / lecun).  "default" is a Nguyen-Widrow scaled uniform like Encog's reset()."""
        g = torch.Generator().manual_seed(seed)
        method = (method or "default").lower()
        ws = self.views()
        with torch.no_grad():
            for l, w in enumerate(ws):
                i, o = self.spec.layer_in[l], self.spec.layer_out[l]
                if method == "gaussian":
                    blk = torch.randn(o, i + 1, generator=g)
                elif method == "xavier":
                    blk = torch.randn(o, i + 1, generator=g) * math.sqrt(2.0 / (i + o))
                elif method == "he":
                    blk = torch.randn(o, i + 1, generator=g) * math.sqrt(2.0 / i)
                elif method == "lecun":
                    blk = torch.randn(o, i + 1, generator=g) * math.sqrt(1.0 / i)
                else:
                    blk = torch.rand(o, i + 1, generator=g) * 2 - 1
                    beta = 0.7 * (o ** (1.0 / max(1, i)))
                    nrm = blk[:, :i].norm(dim=1, keepdim=True).clamp(min=1e-12)
                    blk[:, :i] = beta * blk[:, :i] / nrm
                    blk[:, i] = (torch.rand(o, generator=g) * 2 - 1) * beta
                w.zero_()
                w[:, : i + 1].copy_(blk.to(w))


class HostRows:
    """Host-resident rows (numpy array / memmap / host tensor, fp32 or bf16) streamed to HBM.

    ``chunks()`` yields device bf16 padded chunks [rows, K0] (bias column = 1): rows are copied into
    a pinned staging buffer on the host, sent H2D on a dedicated copy stream into one of two
    device buffers, cast/padded on the compute stream, and the copy of chunk i+1 overlaps the
    GEMMs of chunk i (events order the buffer reuse)."""

    def __init__(self, x, n_in: int):
        self.x = x
        self.n_in = n_in
        self.shape = (int(np.shape(x)[0]), n_in)
        self._bufs = None

    def __len__(self):
        return self.shape[0]

    def _bf16_source(self) -> bool:
        x = self.x
        probe = x.buf if hasattr(x, "buf") else x
        return torch.is_tensor(probe) and probe.dtype == torch.bfloat16

    def _alloc(self, rows, k0, device):
        if self._bufs is not None and self._bufs["rows"] >= rows and self._bufs["k0"] == k0:
            return self._bufs
        f = self.n_in
        dt = torch.bfloat16 if self._bf16_source() else torch.float32   # bf16 rows travel as bf16
        b = {"rows": rows, "k0": k0, "stream": torch.cuda.Stream(device),
             "pin": [torch.empty(rows, f, dtype=dt).pin_memory() for _ in range(2)],
             "raw": [torch.empty(rows, f, dtype=dt, device=device) for _ in range(2)],
             "dev": [torch.zeros(rows, k0, dtype=torch.bfloat16, device=device) for _ in range(2)],
             "copied": [torch.cuda.Event() for _ in range(2)], "used": [torch.cuda.Event() for _ in range(2)]}
        for d in b["dev"]:
            d[:, f] = 1                       # bias column; padding stays 0
        self._bufs = b
        return b

    def chunks(self, lo, hi, chunk_rows, k0, device):
        from ..ops import _native as nat
        b = self._alloc(min(chunk_rows, hi - lo), k0, device)
        cs, main = b["stream"], torch.cuda.current_stream(device)
        starts = list(range(lo, hi, chunk_rows))
        for i, r0 in enumerate(starts):
            r1 = min(hi, r0 + chunk_rows)
            m, k = r1 - r0, i % 2
            b["copied"][k].synchronize() if i >= 2 else None      # pinned buffer k free again
            src = self.x[r0:r1]
            pin = b["pin"][k][:m]
            pin.copy_(torch.as_tensor(np.asarray(src, dtype=np.float32)) if not torch.is_tensor(src)
                      else src.to(pin.dtype))
            with torch.cuda.stream(cs):
                if i >= 2:
                    cs.wait_event(b["used"][k])                   # GEMMs of chunk i-2 done with buffer k
                b["raw"][k][:m].copy_(b["pin"][k][:m], non_blocking=True)
                b["copied"][k].record(cs)
            main.wait_event(b["copied"][k])
            dev = b["dev"][k][:m]
            if b["raw"][k].dtype == torch.bfloat16:
                dev[:, : self.n_in].copy_(b["raw"][k][:m])
            else:
                nat.call_hip("shifu_cast_bf16", b["raw"][k], self.n_in, dev, k0, m, self.n_in, nat.stream_of(dev))
            yield r0, r1, dev
            b["used"][k].record(main)


@dataclass
class TrainData:
    """Resident (device) training shard: padded bf16/fp32 rows + targets + significance."""
    x: torch.Tensor            # [N, K0] rows incl. bias column
    y: torch.Tensor            # [N, n_out] fp32
    s: torch.Tensor | None     # [N] fp32 significance
    n: int


class Optimizer:
    """Replicated optimizer state + fused update (HIP kernel on GPU, torch on CPU)."""

    def __init__(self, numel: int, device, propagation="R", learning_rate=0.1, momentum=0.5,
                 adam_beta1=0.9, adam_beta2=0.999, learning_decay=0.0, reg=0.0, reg_level="NONE",
                 fixed_mask=None):
        prop = (propagation or "R").upper()
        if prop not in RULE_IDS:
            _log.warning("unknown propagation %s, using R", prop)
            prop = "R"
        self.prop = prop
        self.rule = RULE_IDS[prop]
        self.lr = float(learning_rate)
        self.momentum = float(momentum)
        self.beta1, self.beta2 = float(adam_beta1), float(adam_beta2)
        self.learning_decay = float(learning_decay)
        self.reg = float(reg)
        self.reg_level = {"NONE": 0, "L1": 1, "L2": 2}.get(str(reg_level).upper(), 0)
        self.device = device
        z = lambda: torch.zeros(numel, dtype=torch.float32, device=device)  # noqa: E731
        self.s0, self.s1 = z(), z()
        self.s2 = torch.full((numel,), 0.1, dtype=torch.float32, device=device)  # RPROP update values
        self.fixed = None if fixed_mask is None else fixed_mask.to(device=device, dtype=torch.uint8)
        self.iteration = 0
        self.num_train = 1.0

    def state_dict(self):
        return {"s0": self.s0.cpu(), "s1": self.s1.cpu(), "s2": self.s2.cpu(),
                "iteration": self.iteration, "lr": self.lr}

    def load_state_dict(self, d):
        self.s0.copy_(d["s0"]); self.s1.copy_(d["s1"]); self.s2.copy_(d["s2"])
        self.iteration = int(d["iteration"]); self.lr = float(d["lr"])

    def step(self, w: torch.Tensor, g: torch.Tensor, num_train: float):
        self.iteration += 1
        if self.iteration > 1:
            self.lr = self.lr * (1.0 - self.learning_decay)   # NNMaster.java:269
        self.num_train = max(1.0, float(num_train))
        qeps = 0.35 / self.num_train
        qshrink = self.lr / (1.0 + self.lr)
        if w.device.type == "cuda":
            from ..ops import _native as nat
            nat.call_hip("shifu_optimizer_step", w.data_ptr(), g.data_ptr(), self.s0.data_ptr(),
                         self.s1.data_ptr(), self.s2.data_ptr(),
                         None if self.fixed is None else self.fixed.data_ptr(), w.numel(), self.rule,
                         self.reg_level, self.lr, self.momentum, self.beta1, self.beta2,
                         self.learning_decay, self.reg, self.num_train, qeps, qshrink, 1e-4,
                         self.iteration, nat.stream_of(w))
            return
        self._step_torch(w, g, qeps, qshrink)

    def _step_torch(self, w, g, qeps, qshrink):
        """CPU oracle of optimizer_kernel (fp32)."""
        keep = None if self.fixed is None else self.fixed.bool()
        w0 = w.clone()
        s0, s1, s2, lr = self.s0, self.s1, self.s2, self.lr

        def sgn(v):
            return torch.where(v.abs() < 1e-7, torch.zeros_like(v), torch.sign(v))
        rule = self.prop
        delta = None
        if rule == "B":
            delta = g * lr + s0 * self.momentum
            s0.copy_(delta)
        elif rule == "M":
            delta = torch.where(g.abs() < 1e-17, torch.zeros_like(g), torch.sign(g) * lr)
        elif rule == "Q":
            d, s, p = s0.clone(), -g + 1e-4 * w, -s1
            ns = torch.zeros_like(g)
            neg, pos, zero = d < 0, d > 0, d == 0
            ns = ns + torch.where(neg & (s > 0), -qeps * s, torch.zeros_like(s))
            quad = d * s / torch.where((p - s) == 0, torch.ones_like(s), p - s)
            ns = ns + torch.where(neg, torch.where(s >= qshrink * p, lr * d, quad), torch.zeros_like(s))
            ns = ns + torch.where(pos & (s < 0), -qeps * s, torch.zeros_like(s))
            ns = ns + torch.where(pos, torch.where(s <= qshrink * p, lr * d, quad), torch.zeros_like(s))
            ns = ns + torch.where(zero, -qeps * s, torch.zeros_like(s))
            s0.copy_(ns)
            s1.copy_(g)
            delta = ns
        elif rule == "R":
            ch = sgn(g * s1)
            up = torch.clamp(s2 * 1.2, max=50.0)
            dn = torch.clamp(s2 * 0.5, min=1e-6)
            delta = torch.where(ch > 0, sgn(g) * up, torch.where(ch < 0, -s0, sgn(g) * s2))
            new_s2 = torch.where(ch > 0, up, torch.where(ch < 0, dn, s2))
            new_s1 = torch.where(ch < 0, torch.zeros_like(g), g)
            s2.copy_(new_s2)
            s1.copy_(new_s1)
            s0.copy_(delta)
        elif rule == "ADAM":
            s0.mul_(self.beta1).add_((1 - self.beta1) * g)
            s1.mul_(self.beta2).add_((1 - self.beta2) * g * g)
            mc = s0 / (1 - self.beta1 ** self.iteration)
            vc = s1 / (1 - self.beta2 ** self.iteration)
            w.add_(lr * mc / (vc.sqrt() + 1e-8))
        elif rule == "ADAGRAD":
            s0.add_(g * g)
            w.add_(lr * g / (s0.sqrt() + 1e-8))
        elif rule == "RMSPROP":
            s0.add_(g * g)
            s0.mul_(self.learning_decay).add_((1 - self.learning_decay) * g * g)
            w.add_(lr * g / (s0.sqrt() + 1e-8))
        elif rule == "MOMENTUM":
            d = lr * g + self.momentum * s0
            s0.copy_(d)
            w.add_(d)
        elif rule == "NESTEROV":
            prev = s0.clone()
            s0.copy_(self.momentum * prev + g * lr)
            w.add_(self.momentum * prev - (1 + self.momentum) * s0)
        if delta is not None:
            if self.reg_level == 1 and self.reg != 0:
                sh = self.reg / self.num_train
                w.copy_(torch.sign(delta) * torch.clamp(delta.abs() - sh, min=0))
            elif self.reg_level == 2:
                w.add_(delta - self.reg * w / self.num_train)
            else:
                w.add_(delta)
        if keep is not None:
            w.copy_(torch.where(keep, w0, w))


def can_grow(old_sizes, new_sizes) -> bool:
    """``NNStructureComparator.compare(new, old) == 1`` (J/core/dtrain/nn/NNStructureComparator.java:
    25-37) on input-first layer sizes: the new network has at least as many layers, and aligned from
    the input end every non-output layer of the old network fits (>=) into the new one; the new
    output is at least as wide."""
    if len(new_sizes) < len(old_sizes) or new_sizes[-1] < old_sizes[-1]:
        return False
    return all(new_sizes[k] >= old_sizes[k] for k in range(len(old_sizes) - 1))


def grow_weights(trainer: "MLPTrainer", old_weights, fixed_layers=None, fixed_bias: bool = True) -> int:
    """``NNMaster.fitExistingModelIn`` (J/core/dtrain/nn/NNMaster.java:605-645): copy a smaller
    existing network into the trainer's freshly initialised larger one, layers aligned from the
    input end; each old weight matrix [out, in + 1] fills the top-left block of the new one and its
    bias column moves to the new bias column.  Weights copied into a ``FixedLayers`` layer (1-based
    from the input side; its bias too unless ``FixedBias`` is false) stay frozen.  Returns the
    number of frozen weights."""
    p = trainer.params
    views = p.views()
    mask = torch.zeros(p.numel, dtype=torch.bool)
    fixed = set(int(x) for x in (fixed_layers or []))
    with torch.no_grad():
        for l, W in enumerate(old_weights):
            W = torch.as_tensor(np.asarray(W), dtype=torch.float32)
            o, i = W.shape[0], W.shape[1] - 1
            k_new = trainer.spec.layer_in[l]
            views[l][:o, :i] = W[:, :i].to(views[l].device)
            views[l][:o, k_new] = W[:, i].to(views[l].device)
            if l + 1 in fixed:
                kp = p.shapes[l][1]
                rows = torch.arange(o).unsqueeze(1) * kp + p.offsets[l]
                mask[(rows + torch.arange(i).unsqueeze(0)).reshape(-1)] = True
                if fixed_bias:
                    mask[(torch.arange(o) * kp + p.offsets[l] + k_new)] = True
    dist.broadcast_(p.flat, 0)
    if mask.any():
        prev = trainer.opt.fixed
        m = mask.to(trainer.device)
        trainer.opt.fixed = (m if prev is None else (prev.bool() | m)).to(torch.uint8)
    return int(mask.sum())


class MLPTrainer:
    """Data-parallel full-batch (or mini-batch) MLP trainer."""

    def __init__(self, spec: MLPSpec, device=None, propagation="R", learning_rate=0.1,
                 momentum=0.5, adam_beta1=0.9, adam_beta2=0.999, learning_decay=0.0,
                 reg=0.0, reg_level="NONE", seed=0, weight_init="default",
                 chunk_rows=1 << 20, init_flat_encog=None, fixed_layers=None, wgrad_splits=None,
                 dropout_rate=0.0, fixed_bias=False):
        from ..utils.device import default_device
        self.spec = spec
        self.device = torch.device(device) if device is not None else default_device()
        self.gpu = self.device.type == "cuda"
        if self.gpu:
            from ..ops import _native
            _native.require_gpu_native()
        # the register-resident output row kernel takes last hidden width <= 511 and n_out <= 8;
        # any other shape runs the any-shape output kernel + TN wgrad (mlp_kernels.hip)
        self.wide_out = (spec.layer_kpad[-1] > 512 or spec.n_out > 8 or
                         os.environ.get("SHIFU_WIDE_OUTPUT") == "1")   # (forced: A/B tests)
        self.params = MLPParams(spec, self.device)
        if init_flat_encog is not None:
            self.params.from_encog_flat(init_flat_encog)
        else:
            self.params.init_random(seed, weight_init)
        dist.broadcast_(self.params.flat, 0)
        self.valid = self.params.valid_mask().to(self.device)
        # +2 tail slots: an fp32 copy of [error_sum, weight_sum] (reduced in fp64 as self.err_acc)
        self.gbuf = torch.zeros(self.params.numel + 2, dtype=torch.float32, device=self.device)
        self.grad = self.gbuf[: self.params.numel]
        # > 8 MB of gradients under data parallelism: RCCL all-reduce of finished layers' buckets
        # overlaps the last chunk's remaining backward (back-to-front, parallel/dist.py)
        self._reducer = None
        self._final_chunk = False
        gbytes = self.params.numel * 4
        if dist.info().world_size > 1 and (gbytes > (8 << 20) or os.environ.get("SHIFU_GRAD_OVERLAP") == "1"):
            mb = float(os.environ.get("SHIFU_GRAD_BUCKET_MB", "16"))
            self._reducer = dist.BucketedAllReducer(self.grad, int(mb * (1 << 20)))
        fixed = None
        if fixed_bias:                  # FixedBias: bias weights of every layer stay frozen
            fixed = torch.zeros(self.params.numel, dtype=torch.bool)
            for li, (o, k) in enumerate(self.params.shapes):
                off = self.params.offsets[li]
                fixed[off: off + o * k].view(o, k)[:, spec.layer_in[li]] = True
        if fixed_layers:
            fixed = torch.zeros(self.params.numel, dtype=torch.bool)
            for l in fixed_layers:      # FixedLayers: 1-based hidden layer ids (fine tuning)
                li = int(l) - 1
                if 0 <= li < len(self.params.shapes):
                    o, k = self.params.shapes[li]
                    if fixed is None:
                        fixed = torch.zeros(self.params.numel, dtype=torch.bool)
                    fixed[self.params.offsets[li]: self.params.offsets[li] + o * k] = True
        self.opt = Optimizer(self.params.numel, self.device, propagation, learning_rate, momentum,
                             adam_beta1, adam_beta2, learning_decay, reg, reg_level, fixed)
        self.chunk_rows = int(chunk_rows)
        self.wgrad_splits = wgrad_splits
        # ring-pipelined TN wgrad (LDS-DMA ring 4 k-steps deep, fixed-order split reduction:
        # bitwise reproducible); SHIFU_WGRAD_RING=0 restores the 128x128 split-K atomics kernel
        self.wgrad_ring = os.environ.get("SHIFU_WGRAD_RING", "1") != "0"
        self.fused_head = self._head_eligible()
        self.strip_head = self.fused_head and self._strip_head_eligible()
        self.err_acc = torch.zeros(2, dtype=torch.float64, device=self.device)
        # dropout (NNMaster.dropoutNodes :531-556, FloatFlatNetwork.computeLayer :205-215): each
        # iteration drops hidden nodes with DropoutRate and inputs with 0.4*DropoutRate and scales
        # kept outputs by 1/(1-rate).  Realised as a per-column scale of the NEXT layer's weights
        # (identical forward/backward), the same mask on every rank (shared seed, no broadcast).
        self.dropout_rate = float(dropout_rate or 0.0)
        self._drop_gen = torch.Generator().manual_seed(seed * 7919 + 11)
        self._wflat = self.params.flat
        self._scale = None
        self._ws = {}                  # chunk lane -> activations / deltas / ring slab workspace
        self._lane2 = None             # (side stream, gradient buffer) of the second chunk lane
        self.last_error = float("nan")
        self.comm_events = None        # list -> (start, end) HIP events around each gradient all-reduce

    # --------------------------------------------------------------------------------------
    def prepare(self, x, y, s=None, stream: bool | None = None) -> TrainData:
        """Host/device float rows -> resident padded rows (bias column = 1).

        ``stream=True`` (or rows that would not fit in ~80 % of free HBM) keeps the rows on the host
        (numpy memmap / host tensor) and streams them through HBM chunk by chunk with the H2D copies
        on a side stream overlapping compute (out-of-core rows for 1B x 10k)."""
        if self.gpu:
            nbytes = int(np.prod(np.shape(x))) * 2
            if stream is None:
                from ..utils.device import free_hbm
                free = free_hbm(self.device)
                stream = nbytes > 0.8 * free
            if stream:
                n = int(np.shape(x)[0])
                yd = torch.as_tensor(np.asarray(y, dtype=np.float32)).reshape(n, -1).to(self.device).contiguous()
                sd = None if s is None else torch.as_tensor(np.asarray(s, dtype=np.float32)).reshape(n).to(self.device)
                return TrainData(HostRows(x, self.spec.n_in), yd, sd, n)
        x = torch.as_tensor(x)
        n, f = x.shape
        assert f == self.spec.n_in, (f, self.spec.n_in)
        k0 = self.spec.layer_kpad[0]
        dt = torch.bfloat16 if self.gpu else torch.float32
        xp = torch.zeros(n, k0, dtype=dt, device=self.device)
        xp[:, :f] = x.to(self.device, dt)
        xp[:, f] = 1
        y = torch.as_tensor(y, dtype=torch.float32).reshape(n, -1).to(self.device)
        assert y.shape[1] == self.spec.n_out
        sd = None if s is None else torch.as_tensor(s, dtype=torch.float32).reshape(n).to(self.device)
        return TrainData(xp, y.contiguous(), sd, n)

    def _workspace(self, rows: int, lane: int = 0):
        cur = self._ws.get(lane)
        if cur is not None and cur["rows"] >= rows:
            return cur
        kp = self.spec.layer_kpad
        L = len(self.spec.hidden)
        ws = {"rows": rows, "acts": [], "deltas": [], "derivs": []}
        for l in range(1, L + 1):
            ws["acts"].append(torch.empty(rows, kp[l], dtype=torch.bfloat16, device=self.device))
            ws["deltas"].append(torch.empty(rows, kp[l], dtype=torch.bfloat16, device=self.device))
            need_d = ACT_IDS[self.spec.acts[l - 1]] not in ACT_DERIV_FROM_OUTPUT
            ws["derivs"].append(torch.empty(rows, kp[l], dtype=torch.bfloat16, device=self.device)
                                if need_d else None)
        # fp32 split partials of the ring wgrad (ops/csrc/gemm_ring.hip): one buffer for every layer
        ws["slab"] = None
        if self.gpu and self.wgrad_ring:
            from ..ops import _native as nat
            need = max(nat.hip().shifu_wgrad_ring_ws(rows, self.spec.hidden[l], kp[l]) for l in range(L))
            if need > 0:
                ws["slab"] = torch.empty(need // 4, dtype=torch.float32, device=self.device)
        # head output-wgrad partials per 256-row tile + fixed-order reduction scratch (deterministic
        # replacement of the per-tile atomics, ops/csrc/gemm_kernels.hip colsum_fixed)
        ws["gw_slab"] = ws["gw_part"] = ws["err_slab"] = None
        if self.gpu and self.fused_head:
            tiles = max(-(-rows // 256), 8 * 256 if self.strip_head else 0)   # strip head: grid x 8 waves
            ws["gw_slab"] = torch.empty(tiles * kp[L], dtype=torch.float32, device=self.device)
            ws["err_slab"] = torch.empty(tiles * 2, dtype=torch.float64, device=self.device)
            ws["gw_part"] = torch.empty(-(-tiles // 128) * kp[L], dtype=torch.float32, device=self.device)
        # bf16 output deltas of the any-shape output path (operand of the output-layer wgrad)
        ws["ldl"] = round_up(self.spec.n_out, 8)
        ws["outd"] = (torch.empty(rows, ws["ldl"], dtype=torch.bfloat16, device=self.device)
                      if self.gpu and self.wide_out else None)
        self._ws[lane] = ws
        return ws

    def _weights_bf16(self, train: bool = True):
        """bf16 copies of the hidden-layer weights (+ transposed copies for dgrad)."""
        ws = self.params.views(self._wflat)
        kp = self.spec.layer_kpad
        L = len(self.spec.hidden)
        wb, wt = [], []
        from ..ops import _native as nat
        st = nat.stream_of(self.params.flat)
        for l in range(L):
            w = ws[l]
            o, k = w.shape
            b = torch.empty(o, k, dtype=torch.bfloat16, device=self.device)
            nat.call_hip("shifu_cast_bf16", w.data_ptr(), k, b.data_ptr(), k, o, k, st)
            wb.append(b)
            if l >= 1:   # transposed copy for dgrad: [K_l, K_{l+1}] (columns >= o zero)
                t = torch.empty(k, kp[l + 1], dtype=torch.bfloat16, device=self.device)
                nat.call_hip("shifu_transpose_cast", w.data_ptr(), k, t.data_ptr(), o, k, kp[l + 1], st)
                wt.append(t)
            else:
                wt.append(None)
        return wb, wt

    # --------------------------------------------------------------------------------------
    def accumulate_gradients(self, data: TrainData, row_lo: int = 0, row_hi: int | None = None):
        """Sum gradients/errors of rows [row_lo, row_hi) into self.grad / self.err_acc."""
        row_hi = data.n if row_hi is None else row_hi
        if self.gpu and isinstance(data.x, HostRows):
            wb, wt = self._weights_bf16()
            for r0, r1, xd in data.x.chunks(row_lo, row_hi, self.chunk_rows, self.spec.layer_kpad[0], self.device):
                self._final_chunk = r1 >= row_hi
                self._chunk_hip(data, r0, r1, wb, wt, x_dev=xd)
            return
        if self.gpu:
            wb, wt = self._weights_bf16()
            chunks = [(r0, min(row_hi, r0 + self.chunk_rows)) for r0 in range(row_lo, row_hi, self.chunk_rows)]
            if self._two_lanes(len(chunks)):
                self._accumulate_two_lanes(data, chunks, wb, wt)
                return
            for r0, r1 in chunks:
                self._final_chunk = r1 >= row_hi
                self._chunk_hip(data, r0, r1, wb, wt)
        else:
            for r0 in range(row_lo, row_hi, self.chunk_rows):
                r1 = min(row_hi, r0 + self.chunk_rows)
                self._final_chunk = r1 >= row_hi
                self._chunk_torch(data, r0, r1)

    def _two_lanes(self, nchunks: int) -> bool:
        """Chunks alternate between two HIP streams (SHIFU_CHUNK_LANES, default 2) when there are
        at least two device-resident chunks and no per-layer all-reduce overlap is armed: chunk
        c+1's forward GEMM (8-phase, one 128-KiB block per CU) then shares the chip with chunk c's
        memory-bound dgrad / store-bound epilogues instead of waiting for them."""
        return nchunks >= 2 and self._reducer is None and int(os.environ.get("SHIFU_CHUNK_LANES", "2")) >= 2

    def _accumulate_two_lanes(self, data: TrainData, chunks, wb, wt):
        """Even chunks on the current stream into self.grad, odd chunks on a side stream into a
        second gradient buffer (own workspace, own ring slab), summed in a fixed order at the end:
        deterministic run to run.  The error sums are double atomics (order-free up to rounding)."""
        main = torch.cuda.current_stream(self.device)
        if self._lane2 is None:
            self._lane2 = (torch.cuda.Stream(self.device), torch.zeros_like(self.grad))
        side, g2 = self._lane2
        side.wait_stream(main)                     # bf16 weights, zeroed grads, the rows
        with torch.cuda.stream(side):
            g2.zero_()
        g1 = self.grad
        # stagger (opt-in; measured 299 vs 308M rows/s free-running): chunk i's forward starts once
        # chunk i-1's forward is done, so each lane's forward (fwd GEMMs + head) overlaps the other
        # lane's backward (wgrad/dgrad)
        stagger = os.environ.get("SHIFU_CHUNK_STAGGER", "0") == "1"
        fwd_done = None
        for i, (r0, r1) in enumerate(chunks):
            self._final_chunk = False
            st = main if i % 2 == 0 else side
            if stagger and fwd_done is not None:
                st.wait_event(fwd_done)
            ev = torch.cuda.Event() if stagger else None
            with torch.cuda.stream(st):
                self.grad = g1 if i % 2 == 0 else g2
                try:
                    self._chunk_hip(data, r0, r1, wb, wt, lane=i % 2, fwd_event=ev)
                finally:
                    self.grad = g1
            fwd_done = ev
        main.wait_stream(side)
        self.grad.add_(g2)

    def _grad_ready(self, layer: int) -> None:
        """Layer ``layer``'s gradient is final (last chunk's wgrad enqueued): launch the buckets that
        lie entirely at or after its offset (the process-group stream waits for the compute
        stream, so the all-reduce starts when the wgrad kernel has finished)."""
        if self._reducer is not None and self._final_chunk:
            self._reducer.launch_from(self.params.offsets[layer])

    def _head_eligible(self) -> bool:
        """Fused network head (gemm_kernels.hip: gemm_head_8ph_kernel): last hidden forward GEMM +
        output layer + loss + deltas + output wgrad in one 8-phase GEMM epilogue, so the last
        hidden activations never leave the chip.  n_out == 1, last hidden padded width <= 256,
        an activation whose derivative follows from its output (not ptanh).  On by default on
        the GPU (SHIFU_FUSED_HEAD=0 disables); large chunks only (the 8-phase tile is 256 rows)."""
        sp = self.spec
        L = len(sp.hidden)
        if self.device.type != "cuda" or L == 0 or os.environ.get("SHIFU_FUSED_HEAD", "1") == "0":
            return False
        a = ACT_IDS[sp.acts[L - 1]]
        return bool(sp.n_out == 1 and sp.layer_kpad[L] <= 256 and a in ACT_DERIV_FROM_OUTPUT and
                    sp.acts[L - 1] != "ptanh" and sp.hidden[L - 1] <= 255)

    def _strip_head_eligible(self) -> bool:
        """Fused head + the layer-below dgrad in one persistent kernel (gemm_strip_head.hip): the
        head layer's deltas stay in registers as the dgrad's MFMA operand.  Needs >= 2 hidden
        layers, the head layer padded to 256 (128 < width + 1 <= 256), the layer below padded to
        512, and the same activation on both layers (one instantiation per activation).
        SHIFU_STRIP_HEAD=0 keeps the separate head + dgrad kernels."""
        sp = self.spec
        L = len(sp.hidden)
        if L < 2 or os.environ.get("SHIFU_STRIP_HEAD", "1") == "0":
            return False
        kp = sp.layer_kpad
        a2, a1 = sp.acts[L - 1], sp.acts[L - 2]
        return bool(kp[L] == 256 and kp[L - 1] == 512 and a1 == a2 and
                    ACT_IDS[a1] in ACT_DERIV_FROM_OUTPUT and a1 != "ptanh")

    def _chunk_hip(self, data: TrainData, r0: int, r1: int, wb, wt, x_dev=None, lane: int = 0, fwd_event=None):
        from ..ops import _native as nat
        sp, kp = self.spec, self.spec.layer_kpad
        L = len(sp.hidden)
        mc = r1 - r0
        ws = self._workspace(min(self.chunk_rows, data.n), lane)
        gv = self.params.views(self.grad)
        wv = self.params.views(self._wflat)
        x = data.x[r0:r1] if x_dev is None else x_dev
        st = nat.stream_of(x)
        acts = [x] + [a[:mc] for a in ws["acts"]]
        dels = [None] + [d[:mc] for d in ws["deltas"]]
        ders = [None] + [(d[:mc] if d is not None else None) for d in ws["derivs"]]
        head = self.fused_head and mc >= 65536
        y = data.y[r0:r1]
        s = data.s[r0:r1] if data.s is not None else None
        for l in range(L - 1 if head else L):
            a_in, a_out = acts[l], acts[l + 1]
            act = ACT_IDS[sp.acts[l]]
            nat.call_hip("shifu_gemm_nt", a_in.data_ptr(), kp[l], wb[l].data_ptr(), kp[l], sp.hidden[l],
                         a_out.data_ptr(), kp[l + 1], nat.ptr(ders[l + 1]), kp[l + 1], None, 0, None, 0,
                         mc, kp[l + 1], kp[l], 0, act, sp.hidden[l], 1, sp.flat_spot(sp.acts[l]), st)
        fused_dgrad = False
        # the strip head addresses the chunk's H1 / DZ1 / D2 with 32-bit buffer offsets: chunks of
        # 4M+ rows at K1 = 512 take the 8-phase head + the dgrad kernel instead
        strip = self.strip_head and mc * max(kp[L - 1], kp[L]) * 2 < (1 << 32) if L >= 1 else False
        if head and strip:
            # last hidden forward + output + loss + deltas + output wgrad + the dgrad of the layer
            # below in one persistent kernel (the head deltas never leave the chip)
            lh = L - 1
            nat.call_hip("shifu_strip_head", acts[lh], kp[lh], wb[lh], kp[lh], sp.hidden[lh], wt[lh], kp[L],
                              dels[L], kp[L], dels[lh], kp[lh], mc, kp[lh], sp.hidden[lh], sp.hidden[lh - 1],
                              wv[L].data_ptr(), kp[L], y, s, ws["gw_slab"], ws["err_slab"], self.err_acc,
                              ACT_IDS[sp.acts[lh]], ACT_IDS[sp.acts[lh - 1]], ACT_IDS[sp.out_act], sp.loss_id,
                              sp.flat_spot(sp.out_act), sp.flat_spot(sp.acts[lh]), sp.flat_spot(sp.acts[lh - 1]),
                              st)
            nat.call_hip("shifu_colsum_fixed", ws["gw_slab"], nat.hip().shifu_strip_head_rows(mc), kp[L],
                         ws["gw_part"], gv[L].data_ptr(), st)
            fused_dgrad = True
        elif head:
            # last hidden forward + output layer + loss + deltas + output wgrad in one GEMM epilogue
            lh = L - 1
            nat.call_hip("shifu_gemm_head", acts[lh].data_ptr(), kp[lh], wb[lh].data_ptr(), kp[lh], sp.hidden[lh],
                         dels[L].data_ptr(), kp[L], mc, kp[L], kp[lh], ACT_IDS[sp.acts[lh]], sp.hidden[lh],
                         wv[L].data_ptr(), y.data_ptr(), nat.ptr(s), gv[L].data_ptr(), self.err_acc.data_ptr(),
                         kp[L], ACT_IDS[sp.out_act], sp.loss_id, sp.flat_spot(sp.out_act),
                         sp.flat_spot(sp.acts[lh]), nat.ptr(ws["gw_slab"]), nat.ptr(ws["err_slab"]), st)
            if ws["gw_slab"] is not None:
                nat.call_hip("shifu_colsum_fixed", ws["gw_slab"], -(-mc // 256), kp[L], ws["gw_part"],
                             gv[L].data_ptr(), st)
        elif self.wide_out:
            # any-shape output layer: row kernel (deltas, errors) + output wgrad on the TN GEMM
            nat.call_hip("shifu_mlp_output_wide", acts[L], kp[L], ders[L], kp[L], wv[L].data_ptr(), y,
                         sp.n_out, s, dels[L] if L else None, kp[L], ws["outd"], ws["ldl"], gv[L].data_ptr(),
                         self.err_acc, None, 0, mc, kp[L], sp.layer_in[L], sp.n_out, ACT_IDS[sp.out_act],
                         ACT_IDS[sp.acts[L - 1]] if L else 2, sp.loss_id, sp.flat_spot(sp.out_act),
                         sp.flat_spot(sp.acts[L - 1]) if L else 0.0, st)
        else:
            # output layer + loss + last hidden delta + output wgrad
            nat.call_hip("shifu_mlp_output", acts[L].data_ptr(), kp[L], nat.ptr(ders[L]), kp[L],
                         wv[L].data_ptr(), y.data_ptr(), sp.n_out, nat.ptr(s),
                         nat.ptr(dels[L]) if L else None, kp[L], gv[L].data_ptr(), self.err_acc.data_ptr(),
                         None, 0, mc, kp[L], sp.layer_in[L], sp.n_out, ACT_IDS[sp.out_act],
                         ACT_IDS[sp.acts[L - 1]] if L else 2, sp.loss_id, sp.flat_spot(sp.out_act),
                         sp.flat_spot(sp.acts[L - 1]) if L else 0.0, st)
        if fwd_event is not None:
            fwd_event.record()                     # forward + head of this chunk enqueued
        self._grad_ready(L)
        splits = self.wgrad_splits
        for l in range(L - 1, -1, -1):
            # wgrad of layer l: G_l[h_l, K_l] += D_{l+1}^T A_l
            if splits is None:
                ntiles = math.ceil(sp.hidden[l] / 128) * (kp[l] // 128)
                spl = max(1, min(mc // 256, 1024 // max(1, ntiles)))
            else:
                spl = splits
            if self.wgrad_ring and ws["slab"] is not None and mc >= 4096:
                nat.call_hip("shifu_wgrad_ring", dels[l + 1], kp[l + 1], acts[l], kp[l], gv[l], kp[l],
                             mc, sp.hidden[l], kp[l], ws["slab"], ws["slab"].numel() * 4, st)
            else:
                nat.call_hip("shifu_wgrad_tn", dels[l + 1].data_ptr(), kp[l + 1], acts[l].data_ptr(), kp[l],
                             gv[l].data_ptr(), kp[l], mc, sp.hidden[l], kp[l], spl, st)
            self._grad_ready(l)
            if l >= 1 and not (fused_dgrad and l == L - 1):
                # dgrad: D_l = (D_{l+1} W_l) * (f'(A_l)+flat)
                act = ACT_IDS[sp.acts[l - 1]]
                nat.call_hip("shifu_gemm_nt", dels[l + 1].data_ptr(), kp[l + 1], wt[l].data_ptr(), kp[l + 1],
                             kp[l], dels[l].data_ptr(), kp[l], None, 0, acts[l].data_ptr(), kp[l],
                             nat.ptr(ders[l]), kp[l], mc, kp[l], kp[l + 1], 1, act, sp.hidden[l - 1],
                             0, sp.flat_spot(sp.acts[l - 1]), st)

    def _chunk_torch(self, data: TrainData, r0: int, r1: int):
        """fp32 CPU oracle with exactly the HIP path's structure."""
        sp, kp = self.spec, self.spec.layer_kpad
        L = len(sp.hidden)
        wv = self.params.views(self._wflat)
        gv = self.params.views(self.grad)
        x = data.x[r0:r1].float()
        acts, zs = [x], [None]
        for l in range(L):
            z = acts[l] @ wv[l].t()
            a = act_fwd(sp.acts[l], z)
            ap = torch.zeros(a.shape[0], kp[l + 1], dtype=a.dtype)
            ap[:, : sp.hidden[l]] = a
            ap[:, sp.hidden[l]] = 1
            acts.append(ap)
            zs.append(z)
        zo = acts[L] @ wv[L].t()
        p = act_fwd(sp.out_act, zo)
        y = data.y[r0:r1]
        s = data.s[r0:r1].unsqueeze(1) if data.s is not None else torch.ones(r1 - r0, 1)
        e = y - p
        if sp.loss == "log":
            dl = e * s
            pc = p.clamp(1e-7, 1 - 1e-7)
            if sp.tf_objective:
                err = (-(torch.log(p + 1e-7) * y + torch.log(1 - p + 1e-7) * (1 - y)) * s).sum()
            elif sp.n_out == 1:
                err = -(torch.log(pc) * y + torch.log(1 - pc) * (1 - y)).sum()
            else:
                err = -(torch.log(pc) * y * s).sum()
        elif sp.loss == "absolute":
            dl = torch.where(y < p, torch.ones_like(p), -torch.ones_like(p)) * \
                (act_deriv(sp.out_act, zo, p) + sp.flat_spot(sp.out_act)) * s
            err = (e.abs() * s).sum()
        else:
            dl = (act_deriv(sp.out_act, zo, p) + sp.flat_spot(sp.out_act)) * e * s
            err = (e * e * s).sum() if sp.tf_objective else ((e * s) ** 2).sum()
        self.err_acc[0] += float(err)
        self.err_acc[1] += float(s.sum())
        gv[L].add_(dl.t() @ acts[L])
        self._grad_ready(L)
        d = dl
        for l in range(L - 1, -1, -1):
            # delta of hidden layer l+1 (acts[l+1]) from the layer above
            back = d @ wv[l + 1][:, : sp.hidden[l]]
            dh = back * (act_deriv(sp.acts[l], zs[l + 1], acts[l + 1][:, : sp.hidden[l]]) + sp.flat_spot(sp.acts[l]))
            gv[l].add_(dh.t() @ acts[l])
            self._grad_ready(l)
            d = dh

    # --------------------------------------------------------------------------------------
    def _dropout_scale(self) -> torch.Tensor:
        sp = self.spec
        scale = torch.ones(self.params.numel, dtype=torch.float32)
        for l, (o, k) in enumerate(self.params.shapes):
            n_src = sp.layer_in[l]                      # inputs (l = 0) or hidden layer l outputs
            rate = self.dropout_rate * (0.4 if l == 0 else 1.0)
            if rate <= 0:
                continue
            keep = (torch.rand(n_src, generator=self._drop_gen) >= rate).float() / (1.0 - rate)
            off = self.params.offsets[l]
            scale[off: off + o * k].view(o, k)[:, :n_src] *= keep
        return scale.to(self.device)

    def compute_gradients(self, data: TrainData, row_lo=0, row_hi=None):
        """Local gradient pass + one fused all-reduce (grads ++ [err, wsum])."""
        self.grad.zero_()
        self.err_acc.zero_()
        if self.dropout_rate > 0:
            self._scale = self._dropout_scale()
            self._wflat = self.params.flat * self._scale
        else:
            self._wflat = self.params.flat
        self.accumulate_gradients(data, row_lo, row_hi)
        ev0 = None
        if self.comm_events is not None:
            if self.gpu:
                ev0 = torch.cuda.Event(enable_timing=True)
                ev0.record()
            else:
                ev0 = time.perf_counter()
        with trace_range("nn.grad_allreduce"):
            if self._reducer is not None:
                self._reducer.wait()                    # launches any bucket not yet in flight
            else:
                dist.all_reduce_(self.grad)
            # [error sum, weight sum] stay fp64 end to end: an fp32 tail rounds the
            # weight sum once a rank holds > 2^24 rows (the bench's 125M rows per rank)
            dist.all_reduce_(self.err_acc)
        self.gbuf[-2:] = self.err_acc.to(torch.float32)     # fp32 view for callers of the flat buffer
        if ev0 is not None:                             # span of the (final) gradient all-reduce
            if self.gpu:
                ev1 = torch.cuda.Event(enable_timing=True)
                ev1.record()
            else:
                ev1 = time.perf_counter()
            self.comm_events.append((ev0, ev1))
        if self.dropout_rate > 0:
            self.grad.mul_(self._scale)                 # d(loss)/dW of the scaled connections
        self._wflat = self.params.flat
        return self.gbuf

    def step(self, data: TrainData, row_lo=0, row_hi=None, num_train_global: float | None = None) -> float:
        """One epoch (iteration): full gradient over the shard, all-reduce, optimizer update.
        Returns the global training error (squared error / (records x outputs))."""
        self.compute_gradients(data, row_lo, row_hi)
        tail = self.err_acc
        n_local = (data.n if row_hi is None else row_hi) - row_lo
        if num_train_global is None:
            t = torch.tensor([float(n_local)], dtype=torch.float64, device=self.device)
            dist.all_reduce_(t)
            num_train_global = float(t.item())
        self.opt.step(self.params.flat, self.grad, num_train_global)
        err = float(tail[0].item()) / max(1.0, num_train_global * self.spec.n_out)
        self.last_error = err
        return err

    @torch.no_grad()
    def evaluate(self, data: TrainData) -> float:
        """Validation error (forward only), global over ranks."""
        sp = self.spec
        p = self.predict_rows(data.x)
        y = data.y
        s = data.s.unsqueeze(1) if data.s is not None else torch.ones_like(y[:, :1])
        e = (y - p.to(y.dtype))
        if sp.loss == "log":
            pc = p.clamp(1e-7, 1 - 1e-7)
            err = -(torch.log(pc) * y + torch.log(1 - pc) * (1 - y)).sum()
        elif sp.loss == "absolute":
            err = (e.abs() * s).sum()
        else:
            err = ((e * s) ** 2).sum()
        t = torch.tensor([float(err), float(data.n)], dtype=torch.float64, device=self.device)
        dist.all_reduce_(t)
        return float(t[0] / max(1.0, t[1] * sp.n_out))

    @torch.no_grad()
    def predict_rows(self, xpad: torch.Tensor) -> torch.Tensor:
        """Forward pass on padded rows -> [N, n_out] fp32 (HIP kernels on GPU)."""
        sp, kp = self.spec, self.spec.layer_kpad
        L = len(sp.hidden)
        if isinstance(xpad, HostRows):          # out-of-core rows: forward each streamed chunk
            parts = [self.predict_rows(xd.clone()) for _, _, xd in
                     xpad.chunks(0, len(xpad), self.chunk_rows, kp[0], self.device)]
            return torch.cat(parts) if parts else torch.empty(0, sp.n_out, device=self.device)
        n = xpad.shape[0]
        out = torch.empty(n, sp.n_out, dtype=torch.float32, device=self.device)
        if not self.gpu:
            wv = self.params.views()
            a = xpad.float()
            for l in range(L):
                h = act_fwd(sp.acts[l], a @ wv[l].t())
                ap = torch.zeros(n, kp[l + 1])
                ap[:, : sp.hidden[l]] = h
                ap[:, sp.hidden[l]] = 1
                a = ap
            return act_fwd(sp.out_act, a @ wv[L].t())
        from ..ops import _native as nat
        wb, _ = self._weights_bf16(train=False)
        wv = self.params.views()
        st = nat.stream_of(xpad)
        ws = self._workspace(min(self.chunk_rows, n))
        gscratch = torch.zeros(sp.n_out, kp[L], dtype=torch.float32, device=self.device)
        escratch = torch.zeros(2, dtype=torch.float64, device=self.device)
        ydummy = torch.zeros(min(self.chunk_rows, n), sp.n_out, dtype=torch.float32, device=self.device)
        for r0 in range(0, n, self.chunk_rows):
            r1 = min(n, r0 + self.chunk_rows)
            mc = r1 - r0
            acts = [xpad[r0:r1]] + [a[:mc] for a in ws["acts"]]
            for l in range(L):
                nat.call_hip("shifu_gemm_nt", acts[l].data_ptr(), kp[l], wb[l].data_ptr(), kp[l], sp.hidden[l],
                             acts[l + 1].data_ptr(), kp[l + 1], None, 0, None, 0, None, 0, mc, kp[l + 1], kp[l],
                             0, ACT_IDS[sp.acts[l]], sp.hidden[l], 1, 0.0, st)
            if self.wide_out:
                nat.call_hip("shifu_mlp_output_wide", acts[L], kp[L], None, kp[L], wv[L].data_ptr(), ydummy,
                             sp.n_out, None, None, kp[L], None, 0, None, escratch, out[r0:r1], sp.n_out, mc,
                             kp[L], sp.layer_in[L], sp.n_out, ACT_IDS[sp.out_act],
                             ACT_IDS[sp.acts[L - 1]] if L else 2, 0, 0.0, 0.0, st)
                continue
            nat.call_hip("shifu_mlp_output", acts[L].data_ptr(), kp[L], None, kp[L], wv[L].data_ptr(),
                         ydummy.data_ptr(), sp.n_out, None, None, kp[L], gscratch.data_ptr(),
                         escratch.data_ptr(), out[r0:r1].data_ptr(), sp.n_out, mc, kp[L], sp.layer_in[L],
                         sp.n_out, ACT_IDS[sp.out_act], ACT_IDS[sp.acts[L - 1]] if L else 2, 0, 0.0, 0.0, st)
        return out

    # convenience ---------------------------------------------------------------------------
    def encog_weights(self) -> np.ndarray:
        return self.params.to_encog_flat()

    def state_dict(self):
        return {"flat": self.params.flat.detach().cpu(), "opt": self.opt.state_dict(),
                "spec": self.spec.__dict__.copy()}

    def load_state_dict(self, d):
        self.params.flat.copy_(d["flat"].to(self.device))
        self.opt.load_state_dict(d["opt"])
