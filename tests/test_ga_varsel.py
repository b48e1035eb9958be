"""Voted (GA wrapper) variable selection: CandidateGenerator semantics
(J/core/dvarsel/wrapper/CandidateGenerator.java:113-250), the batched population trainer against
independent per-seed models, and `varsel` with filterBy V end to end."""
import json
import os

import numpy as np
import torch


def test_generator_bands_and_sizes():
    from shifu_amd.algos.ga_varsel import CandidateGenerator
    rng = np.random.default_rng(0)
    g = CandidateGenerator({"population_live_size": 20, "expect_variable_cnt": 4, "hybrid_percent": 60,
                            "mutation_percent": 30}, list(range(30)), rng)
    seeds = g.init_seeds()
    assert len(seeds) == 20 and all(len(set(s.genes)) == 4 for s in seeds)
    errors = {s.id: float(i) for i, s in enumerate(seeds)}        # seed i has error i
    nxt = g.next_generation(seeds, errors)
    assert len(nxt) == 20
    # inherit band: 20 * 10 / 100 + 1 = 3 best seeds kept as the same objects, in error order
    assert [s.id for s in nxt[:3]] == [seeds[0].id, seeds[1].id, seeds[2].id]
    # children of the hybrid band draw genes only from the ordinary parents' union
    ordinary = set(g for s in seeds[3:14] for g in s.genes)
    assert all(set(s.genes) <= ordinary for s in nxt[3:14])
    assert all(len(set(s.genes)) == 4 for s in nxt)


def test_population_matches_independent_models():
    from shifu_amd.algos.ga_varsel import PopulationMLP, population_errors
    g = np.random.default_rng(1)
    X = g.normal(size=(300, 6)).astype(np.float32)
    y = (X[:, 0] + X[:, 3] > 0).astype(np.float32)
    w = np.ones(300, np.float32)
    valid = g.random(300) < 0.3
    masks = np.array([[1, 0, 0, 1, 0, 0], [0, 1, 1, 0, 0, 0], [1, 1, 1, 1, 1, 1]], bool)
    errs = population_errors(X, y, w, valid, masks, hidden=4, epochs=15, seed=3)
    # each seed alone (population of one with the same initial weights) gives the same error
    gen = torch.Generator().manual_seed(3)
    full = PopulationMLP(torch.as_tensor(masks), 4, "sigmoid", gen)
    for p in range(3):
        m = PopulationMLP(torch.as_tensor(masks[p:p + 1]), 4, "sigmoid", torch.Generator().manual_seed(0))
        with torch.no_grad():
            m.W1.copy_(full.W1[p * 4:(p + 1) * 4])
            m.W2.copy_(full.W2[p:p + 1])
        opt = torch.optim.Rprop(m.parameters(), lr=0.1, etas=(0.5, 1.2), step_sizes=(1e-6, 50.0))
        Xt, yt, vm = torch.tensor(X), torch.tensor(y)[:, None], torch.tensor(valid)
        for _ in range(15):
            opt.zero_grad()
            (((m(Xt[~vm]) - yt[~vm]) ** 2).sum()).backward()
            m.W1.grad.mul_(m.mask)
            opt.step()
        with torch.no_grad():
            e = float(((m(Xt[vm]) - yt[vm]) ** 2).mean())
        assert abs(e - errs[p]) < 1e-5
    assert errs[0] < errs[1]               # the informative subset wins


def test_varsel_voted_pipeline(tmp_path, monkeypatch):
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    from shifu_amd.cli import main
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.utils.synthetic import make_model_set
    root = make_model_set(str(tmp_path), "ga", "NN", n_rows=800)
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    mc.varSelect["filterBy"] = "V"
    mc.varSelect["params"] = {"population_live_size": 12, "population_multiply_cnt": 3, "expect_variable_cnt": 3,
                              "hybrid_percent": 50, "mutation_percent": 30, "worker_sample_rate": 1.0}
    mc.train["numTrainEpochs"] = 10
    mc.save()
    monkeypatch.chdir(root)
    for cmd in (["init"], ["stats"], ["varsel"]):
        assert main(cmd) == 0
    sel = [c for c in json.load(open("ColumnConfig.json")) if c["finalSelect"]]
    assert len(sel) == 3
