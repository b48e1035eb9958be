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

MI355X realization: the whole population trains at once.  Seed p's first layer is a masked
[H, F] slice of one [P*H, F] weight, so the population's forward is ONE GEMM X @ W^T of shape
[N, F] x [F, P*H] (and the backward two more), instead of P separate Encog trainings.  Every
rank holds a row shard, the population gradient is all-reduced once per epoch, and seeds are
sampled per rank (``worker_sample_rate``; every seed is evaluated by at least rank
``id % world``).  Deliberate deviation: ``randomVariable`` in the reference never draws the last
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


class PopulationMLP(torch.nn.Module):
    """P one-hidden-layer MLPs over column subsets, trained together (masked first layer)."""

    def __init__(self, masks: torch.Tensor, hidden: int, act: str, gen: torch.Generator):
        super().__init__()
        P, F = masks.shape
        self.P, self.H = P, hidden
        self.register_buffer("mask", masks.float().repeat_interleave(hidden, 0))           # [P*H, F]
        fan = masks.sum(1).clamp(min=1).repeat_interleave(hidden).unsqueeze(1)
        w1 = (torch.rand(P * hidden, F, generator=gen) * 2 - 1) / fan.sqrt()
        self.W1 = torch.nn.Parameter(w1 * self.mask)
        self.b1 = torch.nn.Parameter(torch.zeros(P * hidden))
        self.W2 = torch.nn.Parameter((torch.rand(P, hidden, generator=gen) * 2 - 1) / hidden ** 0.5)
        self.b2 = torch.nn.Parameter(torch.zeros(P))
        self.act = {"tanh": torch.tanh, "relu": torch.relu}.get(act, torch.sigmoid)

    def forward(self, x):
        h = self.act(x @ (self.W1 * self.mask).t() + self.b1)                 # one [N, P*H] GEMM
        z = (h.view(-1, self.P, self.H) * self.W2).sum(-1) + self.b2          # [N, P]
        return torch.sigmoid(z)


def population_errors(X, y, w, valid, masks, hidden=10, act="sigmoid", epochs=20, lr=0.1, seed=0, device="cpu"):
    """Validation MSE of each of the P masked MLPs (full-batch RPROP epochs, gradients all-reduced)."""
    dev = torch.device(device)
    g = torch.Generator().manual_seed(seed)
    model = PopulationMLP(torch.as_tensor(masks), hidden, act, g).to(dev)
    if dist.info().world_size > 1:
        for p in model.parameters():
            dist.broadcast_(p.data, 0)
    Xt = torch.as_tensor(X, dtype=torch.float32, device=dev)
    yt = torch.as_tensor(y, dtype=torch.float32, device=dev).view(-1, 1)
    wt = torch.as_tensor(w, dtype=torch.float32, device=dev).view(-1, 1)
    vm = torch.as_tensor(valid, device=dev)
    opt = torch.optim.Rprop(model.parameters(), lr=lr, etas=(0.5, 1.2), step_sizes=(1e-6, 50.0))
    params = list(model.parameters())
    for _ in range(epochs):
        opt.zero_grad(set_to_none=False)
        p = model(Xt[~vm])
        (((p - yt[~vm]) ** 2) * wt[~vm]).sum().backward()
        if dist.info().world_size > 1:
            flat = torch.cat([q.grad.reshape(-1) for q in params])
            dist.all_reduce_(flat)
            off = 0
            for q in params:
                q.grad.copy_(flat[off:off + q.numel()].view_as(q))
                off += q.numel()
        model.W1.grad.mul_(model.mask)
        opt.step()
    with torch.no_grad():
        pv = model(Xt[vm])
        s = torch.cat([((((pv - yt[vm]) ** 2) * wt[vm]).sum(0)).double(),
                       wt[vm].sum().double().expand(1)])
        if dist.info().world_size > 1:
            dist.all_reduce_(s)
    return (s[:-1] / s[-1].clamp(min=1e-12)).cpu().numpy()


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
    queue, hist = [None] * (BEST_SEED_CNT * MAX_ITERATIONS_TO_KEEP), []
    qn = 0
    for it in range(gen.iterations + 1):
        masks = np.zeros((len(seeds), len(variables)), dtype=bool)
        for i, s in enumerate(seeds):
            masks[i, s.genes] = True
        errs = population_errors(X, y, w, valid, masks, hidden, act, epochs, lr, seed + it, device)
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
