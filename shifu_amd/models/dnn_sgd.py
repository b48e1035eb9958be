"""``train.algorithm = TENSORFLOW`` (E5): the reference's Python DNN trainer, re-built on the
device with PyTorch autograd and synchronous data-parallel SGD over RCCL.

Reference behaviour (``src/main/python/train.py``; launched by ``TensorflowTrainer``
J/core/alg/TensorflowTrainer.java:163-266 in LOCAL mode, and by ``ssgd_monitor.py`` with a
parameter server + ``SyncReplicasOptimizer`` in DIST mode):

* network: the normalized selected columns -> ``NumHiddenNodes`` dense layers with
  ``ActivationFunc`` (sigmoid / tanh / relu / leakyrelu, anything else leakyrelu) -> 1 sigmoid
  output; weights and biases drawn U(-1, 1) (train.py:82-97) unless ``WeightInitializer`` is
  ``gaussian`` (N(0, 1)) or ``xavier``;
* loss ``TF.loss`` squared (default, mean squared error) / absolute / log, weighted by the sample
  weight column, + L2 regularization 0.01 * sum(W^2)/2 on every weight matrix
  (tf.contrib.layers.l2_regularizer(0.01));
* optimizer ``TF.optimizer`` adam (default) / gradientdescent / rmsprop at ``LearningRate``;
* mini-batch training: the training rows are split into len/``MiniBatchs`` batches (default 10
  rows per batch, as ``TensorflowTrainer`` :151); ``validSetRate`` of the rows held out;
* every ``CheckpointInterval`` epochs a checkpoint model, and the final model, saved with a
  ``GenericModelConfig.json`` (train.py:349-363) under ``models/<ModelSetName>/``.

MI355X realization (``train_dnn``): the network runs on the framework's own MLP engine
(``models/nn.py`` MLPTrainer: bf16 rows resident in HBM -- no fp32 copy of the shard -- and the
hand-written MFMA forward / dgrad / wgrad kernels), with the Encog flat spot off, tf.nn.leaky_relu
(alpha 0.2) as activation id 9, and the TF update rules of ``optimizer_kernel``
(``shifu_optimizer_step_tf``: ADAM, plain gradient descent, RMSProp rho 0.9) applied to the batch's
mean-loss gradient plus the L2 term in one fused pass.  Each rank owns a row shard and every
mini-batch's gradient is all-reduced before the replicated update -- synchronous SGD with no
parameter server (F9 -> F1).  ``train_dnn_autograd`` is the torch-autograd formulation of the same
objective, kept as the test oracle.  The saved model is a ``safetensors_mlp`` generic model
(``scoring/generic.py``), scored on the GPU by ``eval``.
"""
from __future__ import annotations

import json
import math
import os

import numpy as np
import torch

from ..parallel import dist
from ..utils.log import get_logger

_log = get_logger("models.dnn_sgd")

_ACTS = {"sigmoid": torch.sigmoid, "tanh": torch.tanh, "relu": torch.relu}


def _act(name):
    n = (name or "").lower()
    if n in _ACTS:
        return n, _ACTS[n]
    return "leakyrelu", lambda z: torch.nn.functional.leaky_relu(z, 0.2)   # tf.nn.leaky_relu alpha


def _loss(name, p, y, w):
    n = (name or "squared").lower()
    if n == "absolute":
        e = (p - y).abs()
    elif n == "log":
        eps = 1e-7                                          # tf.losses.log_loss epsilon
        e = -(y * torch.log(p + eps) + (1 - y) * torch.log(1 - p + eps))
    else:
        e = (p - y) ** 2
    # tf.losses.* with weights: sum(w * e) / count(w != 0)  (Reduction.SUM_BY_NONZERO_WEIGHTS)
    return (e * w).sum(), (w != 0).sum()


class DNN(torch.nn.Module):
    def __init__(self, n_in, hidden, acts, init="default", seed=0):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        dims = [n_in] + list(hidden) + [1]
        self.W = torch.nn.ParameterList()
        self.b = torch.nn.ParameterList()
        for i in range(len(dims) - 1):
            fan_in, fan_out = dims[i], dims[i + 1]
            if (init or "").lower() == "gaussian":
                w = torch.randn(fan_out, fan_in, generator=g)
            elif (init or "").lower() == "xavier":
                a = math.sqrt(6.0 / (fan_in + fan_out))
                w = (torch.rand(fan_out, fan_in, generator=g) * 2 - 1) * a
            else:
                w = torch.rand(fan_out, fan_in, generator=g) * 2 - 1
            self.W.append(torch.nn.Parameter(w))
            self.b.append(torch.nn.Parameter(torch.rand(fan_out, generator=g) * 2 - 1))
        self.act_names, self.acts = [], []
        for i in range(len(hidden)):
            nm, fn = _act(acts[i] if i < len(acts) else None)
            self.act_names.append(nm)
            self.acts.append(fn)

    def forward(self, x):
        for i in range(len(self.acts)):
            x = self.acts[i](torch.nn.functional.linear(x, self.W[i], self.b[i]))
        return torch.sigmoid(torch.nn.functional.linear(x, self.W[-1], self.b[-1]))


def _optimizer(name, params, lr):
    n = (name or "adam").lower()
    if n == "gradientdescent":
        return torch.optim.SGD(params, lr=lr)
    if n == "rmsprop":        # tf.train.RMSPropOptimizer defaults: decay 0.9, epsilon 1e-10
        return torch.optim.RMSprop(params, lr=lr, alpha=0.9, eps=1e-10)
    return torch.optim.Adam(params, lr=lr, betas=(0.9, 0.999), eps=1e-8)


def save_generic(model: DNN, out_dir: str, input_names, meta: dict | None = None):
    """models/<name>/{model.safetensors, GenericModelConfig.json} (generic model, safetensors_mlp)."""
    from safetensors.torch import save_file
    os.makedirs(out_dir, exist_ok=True)
    t = {}
    for i, (W, b) in enumerate(zip(model.W, model.b)):
        t[f"W{i}"] = W.detach().float().cpu().contiguous()
        t[f"b{i}"] = b.detach().float().cpu().contiguous()
    save_file(t, os.path.join(out_dir, "model.safetensors"))
    cfg = {"inputnames": list(input_names),
           "properties": {"algorithm": "safetensors_mlp", "trainer": "tensorflow-compatible DNN (torch)",
                          "tags": ["serve"], "outputnames": "shifu_output_0", "normtype": "ZSCALE",
                          "weights": "model.safetensors", "activations": model.act_names + ["sigmoid"],
                          **(meta or {})}}
    path = os.path.join(out_dir, "GenericModelConfig.json")
    with open(path, "w") as f:
        json.dump(cfg, f, indent=2)
    return path


def train_dnn_autograd(X: np.ndarray, y: np.ndarray, w: np.ndarray, valid: np.ndarray, params: dict, epochs: int,
                       device, seed: int = 0, log_fn=None, checkpoint_fn=None, grad_hook=None):
    """torch-autograd oracle of ``train_dnn`` (same batches, objective and optimizer)."""
    hidden = [int(h) for h in (params.get("NumHiddenNodes") or [])]
    acts = list(params.get("ActivationFunc") or [])
    lr = float(params.get("LearningRate", 0.1))
    batch = int(params.get("MiniBatchs", 10) or 10)
    ckpt = int(params.get("CheckpointInterval", 0) or 0)
    model = DNN(X.shape[1], hidden, acts, params.get("WeightInitializer"), seed).to(device)
    if dist.info().world_size > 1:          # identical init everywhere (rank 0 broadcast)
        for p in model.parameters():
            dist.broadcast_(p.data, 0)
    opt = _optimizer(params.get("TF.optimizer"), model.parameters(), lr)
    loss_name = params.get("TF.loss")
    Xt = torch.tensor(np.asarray(X, dtype=np.float32), device=device)   # copy: caches are read-only memmaps
    yt = torch.as_tensor(np.asarray(y, dtype=np.float32).reshape(-1, 1), device=device)
    wt = torch.as_tensor(np.asarray(w, dtype=np.float32).reshape(-1, 1), device=device)
    vmask = torch.as_tensor(np.asarray(valid, dtype=bool), device=device)
    tr_idx = torch.nonzero(~vmask).flatten()
    va_idx = torch.nonzero(vmask).flatten()
    n_tr = int(tr_idx.numel())
    # every rank runs the same number of synchronous steps (global batch count from the largest shard)
    n_batches = max(1, n_tr // batch)
    if dist.info().world_size > 1:
        t = torch.tensor([n_batches], dtype=torch.float64, device=device)
        dist.all_reduce_(t, "max")
        n_batches = int(t.item())
    splits = torch.tensor_split(tr_idx, n_batches) if n_tr else [tr_idx] * n_batches
    params_list = list(model.parameters())
    hist = []
    for ep in range(1, epochs + 1):
        tot = torch.zeros(2, dtype=torch.float64, device=device)
        for idx in splits:
            opt.zero_grad(set_to_none=False)
            p = model(Xt[idx])
            s, cnt = _loss(loss_name, p, yt[idx], wt[idx])
            # SUM_BY_NONZERO_WEIGHTS over the GLOBAL batch: local sums are all-reduced with the grads
            s.backward()
            flat = torch.cat([q.grad.reshape(-1) for q in params_list] +
                             [torch.stack([cnt.double().float(), s.detach().float()])])
            if dist.info().world_size > 1:
                dist.all_reduce_(flat)
            gcnt = float(flat[-2].clamp(min=1))
            off = 0
            for q in params_list:
                q.grad.copy_(flat[off:off + q.numel()].view_as(q) / gcnt)
                off += q.numel()
            with torch.no_grad():                 # L2 0.01 * sum(W^2) / 2 (replicated weights)
                for W in model.W:
                    W.grad.add_(W, alpha=0.01)
            if grad_hook:
                grad_hook(model)
            opt.step()
            tot += torch.stack([flat[-1].double(), torch.tensor(gcnt, dtype=torch.float64, device=device)])
        with torch.no_grad():
            if va_idx.numel():
                pv = model(Xt[va_idx])
                vs, vc = _loss(loss_name, pv, yt[va_idx], wt[va_idx])
                v = torch.stack([vs.double(), vc.double()])
            else:
                v = torch.zeros(2, dtype=torch.float64, device=device)
            if dist.info().world_size > 1:
                dist.all_reduce_(v)
        terr = float(tot[0] / tot[1].clamp(min=1))
        verr = float(v[0] / v[1].clamp(min=1)) if float(v[1]) > 0 else float("nan")
        hist.append((ep, terr, verr))
        if log_fn:
            log_fn(ep, terr, verr)
        if checkpoint_fn and ckpt > 0 and ep % ckpt == 0:
            checkpoint_fn(model, ep)
    return model, hist


# ------------------------------------------------------------------------------------------------
# the TENSORFLOW algorithm on the framework's MLP engine
# ------------------------------------------------------------------------------------------------
_TF_RULES = {"adam": 4, "gradientdescent": 7, "rmsprop": 9}    # optimizer_kernel rule ids


def _mlp_act(name):
    n, _ = _act(name)
    return "leakyrelu_tf" if n == "leakyrelu" else n


def _tf_step_torch(rule, w, g, s0, s1, lr, gscale, l2, l2mask, it):
    """CPU oracle of optimizer_kernel's TF path (fp32; Encog ascent direction g)."""
    g = g * gscale - l2 * w * l2mask
    if rule == 4:
        s0.mul_(0.9).add_(0.1 * g)
        s1.mul_(0.999).add_(0.001 * g * g)
        w.add_(lr * (s0 / (1 - 0.9 ** it)) / ((s1 / (1 - 0.999 ** it)).sqrt() + 1e-8))
    elif rule == 9:
        s0.mul_(0.9).add_(0.1 * g * g)
        w.add_(lr * g / (s0.sqrt() + 1e-10))
    else:
        w.add_(lr * g)


def train_dnn(X, y: np.ndarray, w: np.ndarray, valid: np.ndarray, params: dict, epochs: int,
              device, seed: int = 0, log_fn=None, checkpoint_fn=None, grad_hook=None):
    """Train on this rank's rows with the MLP engine; returns (DNN module, [(epoch, train_err,
    valid_err)]).  Batches, initialisation, objective and update equal ``train_dnn_autograd``."""
    from .nn import MLPSpec, MLPTrainer
    hidden = [int(h) for h in (params.get("NumHiddenNodes") or [])]
    acts = list(params.get("ActivationFunc") or [])
    lr = float(params.get("LearningRate", 0.1))
    batch = int(params.get("MiniBatchs", 10) or 10)
    ckpt = int(params.get("CheckpointInterval", 0) or 0)
    loss = (params.get("TF.loss") or "squared").lower()
    loss = loss if loss in ("squared", "absolute", "log") else "squared"
    rule = _TF_RULES.get((params.get("TF.optimizer") or "adam").lower(), 4)
    device = torch.device(device)
    n_in = int(np.shape(X)[1])
    ref = DNN(n_in, hidden, acts, params.get("WeightInitializer"), seed)      # the TF initialisation
    spec = MLPSpec(n_in, hidden, [_mlp_act(a) for a in acts[: len(hidden)]] or ["sigmoid"], 1, "sigmoid", loss,
                   flat=False, tf_objective=True)
    if len(spec.acts) < len(hidden):
        spec.acts += [_mlp_act(None)] * (len(hidden) - len(spec.acts))
    tr = MLPTrainer(spec, device=device, propagation="R", seed=seed, chunk_rows=max(1 << 16, batch))
    with torch.no_grad():
        for l, wv in enumerate(tr.params.views()):
            i = spec.layer_in[l]
            wv.zero_()
            wv[:, :i].copy_(ref.W[l].detach())
            wv[:, i].copy_(ref.b[l].detach())
    dist.broadcast_(tr.params.flat, 0)
    l2mask = torch.zeros(tr.params.numel, dtype=torch.uint8)
    for off, (o, k), i in zip(tr.params.offsets, tr.params.shapes, spec.layer_in):
        l2mask[off: off + o * k].view(o, k)[:, :i] = 1                          # weights, not biases
    l2mask = l2mask.to(device)
    s0 = torch.zeros(tr.params.numel, dtype=torch.float32, device=device)
    s1 = torch.zeros_like(s0)
    vmask = np.asarray(valid, dtype=bool)
    tri, vai = np.nonzero(~vmask)[0], np.nonzero(vmask)[0]
    yv = np.asarray(y, dtype=np.float32).reshape(-1)
    wv_ = np.asarray(w, dtype=np.float32).reshape(-1)

    def rows(idx):
        # bf16 NormalizedData (data/rowstore.Bf16Rows) goes to HBM as its bf16 bits, rows gathered
        # on the device; other inputs as fp32 host rows (prepare() casts them to bf16 on the GPU)
        if hasattr(X, "device_rows") and device.type == "cuda":
            return X.device_rows(device, rows=None if len(idx) == len(yv) else idx)
        return torch.from_numpy(np.asarray(X if len(idx) == len(yv) else X[idx], dtype=np.float32))
    data = tr.prepare(rows(tri), yv[tri].reshape(-1, 1), wv_[tri])
    vdata = tr.prepare(rows(vai), yv[vai].reshape(-1, 1), wv_[vai]) if len(vai) else None
    n_tr = len(tri)
    n_batches = max(1, n_tr // batch)
    if dist.info().world_size > 1:          # every rank runs the same number of synchronous steps
        t = torch.tensor([n_batches], dtype=torch.float64, device=device)
        dist.all_reduce_(t, "max")
        n_batches = int(t.item())
    bounds = [(int(a[0]), int(a[-1]) + 1) if len(a) else (0, 0)
              for a in np.array_split(np.arange(n_tr), n_batches)]
    # SUM_BY_NONZERO_WEIGHTS over the GLOBAL batch: per-batch counts of non-zero weights, summed once
    nz = (wv_[tri] != 0).astype(np.float64)
    cnts = torch.tensor([nz[a:b].sum() for a, b in bounds], dtype=torch.float64, device=device)
    dist.all_reduce_(cnts)
    cnts = cnts.clamp(min=1).cpu().numpy()
    sign = {"squared": 2.0, "log": 1.0, "absolute": -1.0}[loss]   # Encog delta -> -d(mean loss)/dW
    hist, it = [], 0
    from ..ops import _native as nat
    for ep in range(1, epochs + 1):
        # sum(w * loss) of every batch (TF objective, kept on the device: one host read per epoch)
        terr_sum, tcnt = torch.zeros((), dtype=torch.float64, device=device), 0.0
        for bi, (a, b) in enumerate(bounds):
            it += 1
            tr.compute_gradients(data, a, b)
            gscale = sign / float(cnts[bi])
            if grad_hook:
                grad_hook(tr)
            if device.type == "cuda":
                nat.call_hip("shifu_optimizer_step_tf", tr.params.flat, tr.grad, s0, s1, tr.params.numel, rule,
                             lr, 0.9, 0.999, 0.9, gscale, 0.01, l2mask, it, nat.stream_of(tr.params.flat))
            else:
                _tf_step_torch(rule, tr.params.flat, tr.grad, s0, s1, lr, gscale, 0.01, l2mask.float(), it)
            terr_sum += tr.err_acc[0]
            tcnt += float(cnts[bi])
        terr = float(terr_sum) / max(tcnt, 1.0)
        v = torch.zeros(2, dtype=torch.float64, device=device)
        if vdata is not None:
            with torch.no_grad():
                p = tr.predict_rows(vdata.x)[:, :1].float()
                vs, vc = _loss(loss, p, vdata.y[:, :1].float(), vdata.s.reshape(-1, 1).float())
                v = torch.stack([vs.double(), vc.double()])
        dist.all_reduce_(v)
        verr = float(v[0] / v[1].clamp(min=1)) if float(v[1]) > 0 else float("nan")
        hist.append((ep, terr, verr))
        if log_fn:
            log_fn(ep, terr, verr)
        if checkpoint_fn and ckpt > 0 and ep % ckpt == 0:
            checkpoint_fn(_to_dnn(tr, ref), ep)
    return _to_dnn(tr, ref), hist


def _to_dnn(tr, ref: DNN) -> DNN:
    """The MLP engine's weights as the DNN module (save_generic's layout: W[l] [out, in], b[l])."""
    m = DNN.__new__(DNN)
    torch.nn.Module.__init__(m)
    m.W, m.b = torch.nn.ParameterList(), torch.nn.ParameterList()
    for l, wv in enumerate(tr.params.views()):
        i = tr.spec.layer_in[l]
        m.W.append(torch.nn.Parameter(wv[:, :i].detach().float().cpu().clone()))
        m.b.append(torch.nn.Parameter(wv[:, i].detach().float().cpu().clone()))
    m.act_names, m.acts = list(ref.act_names), list(ref.acts)
    return m
