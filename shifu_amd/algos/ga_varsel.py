"""Voted (genetic wrapper) variable selection, ``varSelect.filterBy = V`` (H13 "voted").

Reference: ``WrapperMasterConductor`` (J/core/dvarsel/wrapper/WrapperMasterConductor.java:30-130),
``CandidateGenerator`` (J/core/dvarsel/wrapper/CandidateGenerator.java:30-290),
``WrapperWorkerConductor`` (:30-80) and ``ValidationConductor.runValidate`` (:48-76):

* variables = the good candidate columns; a *seed* is a list of ``expect_variable_cnt`` of them;
  ``population_live_size`` random seeds start the search;
* each generation every seed is scored by the validation error of an NN trained on its columns
  with the model set's NN settings (each worker evaluates a seed with probability
  ``worker_sample_rate``; a seed's error is the mean over the workers that evaluated it, 999 if
  none did);
* next generation (sorted by error): the best ``100 - hybrid - mutation`` % are inherited, the
  middle ``hybrid_percent`` % are replaced by children of two random parents of that band (genes
  drawn without replacement from the parents' union), the worst ``mutation_percent`` % are mutated
  (every gene swapped for an unselected variable with probability 0.05);
* each generation credits the first 5 seeds of the new population 5, 4, 3, 2, 1 in a queue of
  the last 25 credits; after ``population_multiply_cnt`` generations the seed with the most
  credit wins and its columns become ``finalSelect``.

MI355X realization: the whole population trains at once on the framework's own kernels
(``PopulationTrainer``).  Seed p's first layer is a masked [H, F] slice of one [P*H, F] weight, so
the population's forward is ONE bf16 MFMA GEMM X @ W^T of shape [N, F] x [F, P*H] and its
first-layer gradient one ring wgrad, instead of P separate Encog trainings; the per-seed output
neurons run in ``ga_kernels.hip`` and the update is ``optimizer_kernel``'s RPROP with the masked
weights frozen.  The rows are staged on the device once as bf16 and reused by every generation.
(The dense masked weight multiplies (F - expect) / F zeros; at the reference defaults that is
cheaper on the matrix cores than gathering each seed's columns, which would turn one GEMM with a
shared operand into P narrow ones.)  Every rank holds a row shard, the population gradient is
all-reduced once per epoch, and seeds are sampled per rank (``worker_sample_rate``; every seed
is evaluated by at least rank ``id % world``).  Deliberate deviation: ``randomVariable`` in the reference never draws the last
variable ((int)(rand * (n - 1))); here every variable can be drawn.
"""
from __future__ import annotations

import numpy as np
import torch

from ..parallel import dist
from ..utils.log import get_logger

_log = get_logger("algos.ga_varsel")

DEFAULTS = {"worker_sample_rate": 0.1, "population_multiply_cnt": 100, "population_live_size": 500,
            "expect_variable_cnt": 300, "hybrid_percent": 60, "mutation_percent": 30}
BEST_SEED_CNT, MAX_ITERATIONS_TO_KEEP = 5, 5


class Seed:
    __slots__ = ("id", "genes")

    def __init__(self, sid, genes):
        self.id, self.genes = sid, list(genes)


class CandidateGenerator:
    def __init__(self, params: dict, variables: list, rng: np.random.Generator):
        p = {**DEFAULTS, **{k: v for k, v in (params or {}).items() if k in DEFAULTS}}
        self.iterations = int(p["population_multiply_cnt"])
        self.live = int(p["population_live_size"])
        self.expect = int(p["expect_variable_cnt"])
        self.cross = int(p["hybrid_percent"])
        mutation = int(p["mutation_percent"])
        if self.live < 1 or self.expect < 1:
            raise ValueError("population_live_size and expect_variable_cnt must be >= 1")
        if not (0 <= self.cross <= 100 and 0 <= mutation <= 100) or self.cross + mutation > 100:
            raise ValueError("hybrid_percent / mutation_percent must be in [0, 100] and sum to <= 100")
        self.inherit = 100 - self.cross - mutation
        self.variables = list(variables)
        self.expect = min(self.expect, len(self.variables))
        self.rng = rng
        self.next_id = 1

    def _sid(self):
        self.next_id += 1
        return self.next_id - 1

    def init_seeds(self):
        return [Seed(self._sid(), self.rng.choice(self.variables, self.expect, replace=False).tolist())
                for _ in range(self.live)]

    def next_generation(self, seeds, errors: dict):
        order = sorted(seeds, key=lambda s: errors.get(s.id, 999.0))
        n = len(order)
        last_best = n * self.inherit // 100
        first_worst = n * (100 - self.cross) // 100
        best, ordinary, worst = order[:last_best + 1], order[last_best + 1:first_worst], order[first_worst:]
        out = list(best)
        for _ in range(len(ordinary)):
            f = ordinary[self.rng.integers(len(ordinary))]
            m = ordinary[self.rng.integers(len(ordinary))]
            pool = list(dict.fromkeys(f.genes + m.genes))
            idx = self.rng.permutation(len(pool))[:len(f.genes)]
            out.append(Seed(self._sid(), [pool[i] for i in idx]))
        for s in worst:
            keep = [g for g in s.genes if self.rng.random() >= 0.05]
            rest = [v for v in self.variables if v not in set(s.genes)]
            self.rng.shuffle(rest)
            out.append(Seed(self._sid(), keep + rest[:len(s.genes) - len(keep)]))
        return out


ACT_OK = ("sigmoid", "tanh", "relu")       # hidden activations with f' from the output (kernel + oracle)


def _deriv_out(act: str, h: torch.Tensor) -> torch.Tensor:
    if act == "tanh":
        return 1.0 - h * h
    if act == "relu":
        return (h > 0).to(h.dtype)
    return h * (1.0 - h)


def _pad(k: int, m: int) -> int:
    return (k + m - 1) // m * m


class PopulationData:
    """The varsel rows as GEMM operands, built once per selection run and reused by every
    generation: bf16 rows [n, kx] with a ones column at F (the first-layer bias) and zero padding
    to a multiple of 256, split into training and validation rows; targets and weights fp32."""

    def __init__(self, X, y, w, valid, device):
        dev = torch.device(device)
        X = np.asarray(X, dtype=np.float32)
        n, F = X.shape
        self.F, self.kx, self.dev = F, _pad(F + 1, 256), dev
        vm = np.asarray(valid, dtype=bool)

        def rows(sel):
            idx = np.flatnonzero(sel)
            Xb = torch.zeros(len(idx), self.kx, dtype=torch.bfloat16, device=dev)
            for a in range(0, len(idx), 1 << 18):           # bounded host staging, bf16 on the device
                Xb[a:a + (1 << 18), :F] = torch.as_tensor(X[idx[a:a + (1 << 18)]]).to(dev).to(torch.bfloat16)
            Xb[:, F] = 1.0
            yy = torch.as_tensor(np.asarray(y, np.float32).reshape(-1)[idx], device=dev)
            ww = torch.as_tensor(np.asarray(w, np.float32).reshape(-1)[idx], device=dev)
            return Xb, yy, ww
        self.Xt, self.yt, self.wt = rows(~vm)
        self.Xv, self.yv, self.wv = rows(vm)


class PopulationTrainer:
    """P one-hidden-layer MLPs (H hidden units, sigmoid output, squared error) over column subsets,
    trained together with the framework's RPROP (``models.nn.Optimizer``, Encog semantics: the
    reference trains each seed's NN with the model set's propagation).  Seed p's first layer is
    rows [p*H, (p+1)*H) of ONE dense weight [P*H, kx] whose masked entries are frozen at zero, so:

    * forward: the own bf16 MFMA GEMM (``shifu_gemm_nt``, activation in the epilogue) X W1^T ->
      H [n, P*H] bf16;
    * per-seed output neuron, loss and deltas: ``ga_kernels.hip`` (one thread per seed);
    * first-layer gradient: the ring wgrad dH^T X (``shifu_wgrad_ring``, fixed-order reduction);
    * update: ``optimizer_kernel`` over the flat [W1 | W2 | b2] vector.

    The CPU backend runs the same arithmetic in torch (bf16-rounded operands, fp32 sums) as the
    oracle of the GPU one."""

    CHUNK = 1 << 17

    def __init__(self, data: PopulationData, masks, hidden: int, act: str, lr: float, gen: torch.Generator):
        masks = torch.as_tensor(np.asarray(masks, dtype=bool))
        P, F = masks.shape
        self.P, self.H, self.F, self.kx = P, int(hidden), F, data.kx
        self.act = act if act in ACT_OK else "sigmoid"
        self.data, self.dev = data, data.dev
        PH = P * self.H
        self.PH, self.php = PH, _pad(PH, 256)
        # initial weights: uniform, first layer scaled by each seed's fan-in and masked
        fan = masks.sum(1).clamp(min=1).repeat_interleave(self.H).unsqueeze(1).float()
        mrow = masks.float().repeat_interleave(self.H, 0)                           # [PH, F]
        w1 = (torch.rand(PH, F, generator=gen) * 2 - 1) / fan.sqrt() * mrow
        w2 = (torch.rand(P, self.H, generator=gen) * 2 - 1) / self.H ** 0.5
        self.n1 = PH * self.kx
        flat = torch.zeros(self.n1 + PH + P, dtype=torch.float32)
        flat[: self.n1].view(PH, self.kx)[:, :F] = w1
        flat[self.n1: self.n1 + PH] = w2.reshape(-1)
        fixed = torch.zeros(flat.numel(), dtype=torch.bool)
        fv = fixed[: self.n1].view(PH, self.kx)
        fv[:, :F] = ~mrow.bool()                      # unselected columns stay zero
        fv[:, F + 1:] = True                          # padding (column F is the bias)
        self.flat = flat.to(self.dev)
        if dist.info().world_size > 1:
            dist.broadcast_(self.flat, 0)
        self.grad = torch.zeros_like(self.flat)
        from ..models.nn import Optimizer
        self.opt = Optimizer(self.flat.numel(), self.dev, "R", learning_rate=lr, fixed_mask=fixed)
        self.gpu = self.dev.type == "cuda"
        if self.gpu:
            self.w1b = torch.zeros(self.php, self.kx, dtype=torch.bfloat16, device=self.dev)
            self._bufs = {}

    # ---- views
    @property
    def W1(self):
        return self.flat[: self.n1].view(self.PH, self.kx)

    @property
    def W2(self):
        return self.flat[self.n1: self.n1 + self.PH].view(self.P, self.H)

    @property
    def b2(self):
        return self.flat[self.n1 + self.PH:]

    # ---- GPU
    def _buf(self, name, shape, dtype):
        b = self._bufs.get(name)
        if b is None or b.numel() < int(np.prod(shape)):
            b = self._bufs[name] = torch.zeros(int(np.prod(shape)), dtype=dtype, device=self.dev)
        return b[: int(np.prod(shape))].view(*shape)

    def _hidden_gpu(self, X):
        from ..models.nn import ACT_IDS
        from ..ops import _native as nat
        n = X.shape[0]
        Hs = self._buf("H", (n, self.php), torch.bfloat16)
        nat.call_hip("shifu_gemm_nt", X, self.kx, self.w1b, self.kx, self.PH, Hs, self.php, None, 0, None, 0, None,
                     0, n, self.php, self.kx, 0, ACT_IDS[self.act], self.PH, 0, 0.0, nat.stream_of(X))
        return Hs

    def _epoch_gpu(self):
        from ..models.nn import ACT_IDS
        from ..ops import _native as nat
        d = self.data
        st = nat.stream_of(self.flat)
        nat.call_hip("shifu_cast_bf16", self.W1, self.kx, self.w1b, self.kx, self.PH, self.kx, st)
        self.grad.zero_()
        g2 = self.grad[self.n1:]
        n = d.Xt.shape[0]
        for c, a in enumerate(range(0, n, self.CHUNK)):
            X = d.Xt[a:a + self.CHUNK]
            m = X.shape[0]
            Hs = self._hidden_gpu(X)
            dH = self._buf("dH", (m, self.php), torch.bfloat16)
            part = self._buf("part", (nat.hip().shifu_ga_part_floats(m, self.P, self.H, 1),), torch.float32)
            nat.call_hip("shifu_ga_head", Hs, self.php, m, self.P, self.H, self.W2, self.b2, d.yt[a:a + m],
                         d.wt[a:a + m], ACT_IDS[self.act], dH, self.php, part, g2, 1, int(c > 0), st)
            if m >= 32:
                ws = self._buf("ws", (max(4, nat.hip().shifu_wgrad_ring_ws(m, self.PH, self.kx) // 4),), torch.float32)
                nat.call_hip("shifu_wgrad_ring", dH, self.php, X, self.kx, self.grad, self.kx, m, self.PH, self.kx,
                             ws, ws.numel() * 4, st)
            else:                                   # a tail below one ring step
                self.grad[: self.n1].view(self.PH, self.kx).add_(dH[:, : self.PH].float().t() @ X.float())
        return n

    def _valid_gpu(self):
        from ..models.nn import ACT_IDS
        from ..ops import _native as nat
        d = self.data
        st = nat.stream_of(self.flat)
        nat.call_hip("shifu_cast_bf16", self.W1, self.kx, self.w1b, self.kx, self.PH, self.kx, st)
        err = torch.zeros(self.P, dtype=torch.float32, device=self.dev)
        n = d.Xv.shape[0]
        for c, a in enumerate(range(0, n, self.CHUNK)):
            X = d.Xv[a:a + self.CHUNK]
            m = X.shape[0]
            Hs = self._hidden_gpu(X)
            part = self._buf("vpart", (nat.hip().shifu_ga_part_floats(m, self.P, self.H, 0),), torch.float32)
            nat.call_hip("shifu_ga_head", Hs, self.php, m, self.P, self.H, self.W2, self.b2, d.yv[a:a + m],
                         d.wv[a:a + m], ACT_IDS[self.act], None, 0, part, err, 0, int(c > 0), st)
        return err

    # ---- CPU oracle (same roundings: bf16 operands / activations / deltas, fp32 sums)
    def _forward_cpu(self, X):
        from ..models.nn import act_fwd
        W1b = self.W1.to(torch.bfloat16).float()
        return act_fwd(self.act, X.float() @ W1b.t()).to(torch.bfloat16).float()    # [n, PH]

    def _head_cpu(self, Hs, y):
        z = (Hs.view(-1, self.P, self.H) * self.W2).sum(-1) + self.b2
        return torch.sigmoid(z), y.view(-1, 1)

    def _epoch_cpu(self):
        d = self.data
        self.grad.zero_()
        Hs = self._forward_cpu(d.Xt)
        o, y = self._head_cpu(Hs, d.yt)
        dz = (y - o) * o * (1 - o) * d.wt.view(-1, 1)                                  # [n, P]
        h3 = Hs.view(-1, self.P, self.H)
        dH = (dz.unsqueeze(-1) * self.W2 * _deriv_out(self.act, h3)).to(torch.bfloat16).float()
        self.grad[: self.n1].view(self.PH, self.kx).copy_(dH.view(-1, self.PH).t() @ d.Xt.float())
        self.grad[self.n1: self.n1 + self.PH] = (dz.unsqueeze(-1) * h3).sum(0).reshape(-1)
        self.grad[self.n1 + self.PH:] = dz.sum(0)
        return d.Xt.shape[0]

    def _valid_cpu(self):
        d = self.data
        o, y = self._head_cpu(self._forward_cpu(d.Xv), d.yv)
        return (((o - y) ** 2) * d.wv.view(-1, 1)).sum(0)

    # ---- training
    def train(self, epochs: int) -> np.ndarray:
        """``epochs`` full-batch RPROP epochs (gradients all-reduced), then each seed's validation
        error sum w (o - y)^2 / sum w over every rank's validation rows."""
        for _ in range(epochs):
            n = self._epoch_gpu() if self.gpu else self._epoch_cpu()
            cnt = torch.tensor([float(n)], dtype=torch.float64, device=self.dev)
            if dist.info().world_size > 1:
                dist.all_reduce_(self.grad)
                dist.all_reduce_(cnt)
            self.opt.step(self.flat, self.grad, float(cnt.item()))
        err = (self._valid_gpu() if self.gpu else self._valid_cpu()).double()
        s = torch.cat([err, self.data.wv.double().sum().reshape(1)])
        if dist.info().world_size > 1:
            dist.all_reduce_(s)
        return (s[:-1] / s[-1].clamp(min=1e-12)).cpu().numpy()


def population_errors(X, y, w, valid, masks, hidden=10, act="sigmoid", epochs=20, lr=0.1, seed=0, device="cpu",
                      data: PopulationData | None = None):
    """Validation MSE of each of the P masked MLPs (``PopulationTrainer``); ``data``: the rows
    already staged on the device (reused across generations)."""
    data = data or PopulationData(X, y, w, valid, device)
    g = torch.Generator().manual_seed(seed)
    return PopulationTrainer(data, masks, hidden, act, lr, g).train(epochs)


def voted_selection(X, y, w, variables, params, nn_params, epochs, valid_rate=0.2, seed=0, device="cpu",
                    log=None):
    """Run the GA; returns (best seed's variables, history of best errors)."""
    info = dist.info()
    rng = np.random.default_rng(seed)                     # identical on every rank (replicated master)
    gen = CandidateGenerator(params, list(range(len(variables))), rng)
    rate = float({**DEFAULTS, **(params or {})}["worker_sample_rate"])
    n = X.shape[0]
    valid = np.random.default_rng(seed + 7 + info.rank).random(n) < valid_rate
    hidden = int((nn_params.get("NumHiddenNodes") or [10])[0])
    act = str((nn_params.get("ActivationFunc") or ["sigmoid"])[0]).lower()
    lr = float(nn_params.get("LearningRate", 0.1))
    seeds = gen.init_seeds()
    data = PopulationData(X, y, w, valid, device)
    queue, hist = [None] * (BEST_SEED_CNT * MAX_ITERATIONS_TO_KEEP), []
    qn = 0
    for it in range(gen.iterations + 1):
        masks = np.zeros((len(seeds), len(variables)), dtype=bool)
        for i, s in enumerate(seeds):
            masks[i, s.genes] = True
        errs = population_errors(X, y, w, valid, masks, hidden, act, epochs, lr, seed + it, device, data=data)
        # worker sampling: each rank evaluates a seed with probability worker_sample_rate (rank
        # id % world always does); error = mean over the ranks that evaluated it, 999 if none
        srng = np.random.default_rng(seed * 1000003 + it * 131 + info.rank)
        took = (srng.random(len(seeds)) < rate) | (np.array([s.id for s in seeds]) % info.world_size == info.rank)
        acc = torch.tensor(np.stack([np.where(took, errs, 0.0), took.astype(float)]), dtype=torch.float64)
        if info.world_size > 1:
            acc = acc.to(device)
            dist.all_reduce_(acc)
            acc = acc.cpu()
        acc = acc.numpy()
        errors = {s.id: (acc[0, i] / acc[1, i] if acc[1, i] > 0 else 999.0) for i, s in enumerate(seeds)}
        best_err = min(errors.values())
        hist.append(best_err)
        if log:
            log(it, best_err)
        if it == gen.iterations:
            break
        seeds = gen.next_generation(seeds, errors)
        for i in range(min(BEST_SEED_CNT, len(seeds))):
            queue[qn % len(queue)] = (BEST_SEED_CNT - i, seeds[i])
            qn += 1
    credit = {}
    for e in queue:
        if e is not None:
            credit[e[1]] = credit.get(e[1], 0) + e[0]
    best = max(credit.items(), key=lambda kv: kv[1])[0] if credit else min(seeds, key=lambda s: errors[s.id])
    return [variables[g] for g in best.genes], hist
