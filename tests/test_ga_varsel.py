"""Voted (GA wrapper) variable selection: CandidateGenerator semantics
(J/core/dvarsel/wrapper/CandidateGenerator.java:113-250), the batched population trainer against
independent per-seed models, and `varsel` with filterBy V end to end."""
import json
import os

import numpy as np
import pytest
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
    """The batched population (one dense masked first layer, RPROP per weight) trains every seed
    exactly as that seed alone would: same validation error from the same initial weights."""
    from shifu_amd.algos.ga_varsel import PopulationData, PopulationTrainer
    g = np.random.default_rng(1)
    X = g.normal(size=(300, 6)).astype(np.float32)
    y = (X[:, 0] + X[:, 3] > 0).astype(np.float32)
    w = np.ones(300, np.float32)
    valid = g.random(300) < 0.3
    masks = np.array([[1, 0, 0, 1, 0, 0], [0, 1, 1, 0, 0, 0], [1, 1, 1, 1, 1, 1]], bool)
    data = PopulationData(X, y, w, valid, "cpu")
    full = PopulationTrainer(data, masks, 4, "sigmoid", 0.1, torch.Generator().manual_seed(3))
    init = full.flat.clone()
    errs = full.train(15)
    W1 = init[: full.n1].view(full.PH, full.kx)
    W2 = init[full.n1: full.n1 + full.PH].view(3, 4)
    for p in range(3):
        one = PopulationTrainer(data, masks[p:p + 1], 4, "sigmoid", 0.1, torch.Generator().manual_seed(0))
        one.W1.copy_(W1[p * 4:(p + 1) * 4])
        one.W2.copy_(W2[p:p + 1])
        assert abs(float(one.train(15)[0]) - float(errs[p])) < 1e-6
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


@pytest.mark.gpu
@pytest.mark.parametrize("H", [10, 100])
def test_population_gpu_matches_cpu_oracle(H):
    """The population on the own kernels (MFMA forward, ga_kernels.hip heads, ring wgrad,
    optimizer_kernel RPROP) against the torch CPU oracle of the same arithmetic: per-seed
    validation errors within 1e-3 relative.  H = 100 runs the any-width head (> 64 hidden)."""
    from shifu_amd.algos.ga_varsel import PopulationData, PopulationTrainer
    g = np.random.default_rng(4)
    n, F, P, E = 20000, 300, 40, 60
    X = g.normal(size=(n, F)).astype(np.float32)
    y = (X[:, 0] - X[:, 7] + 0.5 * X[:, 11] > 0).astype(np.float32)
    w = (g.random(n) + 0.5).astype(np.float32)
    valid = g.random(n) < 0.2
    masks = np.zeros((P, F), bool)
    for p in range(P):
        masks[p, g.choice(F, E, replace=False)] = True
    errs = {}
    for dev in ("cpu", "cuda"):
        data = PopulationData(X, y, w, valid, dev)
        errs[dev] = PopulationTrainer(data, masks, H, "sigmoid", 0.1, torch.Generator().manual_seed(9)).train(5)
    rel = np.abs(errs["cuda"] - errs["cpu"]) / errs["cpu"]
    assert rel.max() < 1e-3, (rel.max(), errs)
