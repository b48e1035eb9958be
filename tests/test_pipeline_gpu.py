"""The full pipeline on the MI355X (HIP MFMA NN trainer, HIP histogram tree trainer) over a
synthetic model set generated in-test (the GPU box has no reference fixtures)."""
import json
import os

import pytest

pytestmark = pytest.mark.gpu


def _run(root, steps=("init", "stats", "varsel", "norm", "train", "eval")):
    from shifu_amd.cli import main
    cwd = os.getcwd()
    os.chdir(root)
    try:
        for s in steps:
            assert main(s.split()) == 0, s
    finally:
        os.chdir(cwd)


def _auc(root):
    return json.load(open(os.path.join(root, "evals/Eval1/EvalPerformance.json")))["areaUnderRoc"]


@pytest.mark.parametrize("alg,params,min_auc", [("NN", None, 0.85), ("LR", None, 0.85),
                                                ("GBT", {"TreeNum": 30, "MaxDepth": 5}, 0.8),
                                                ("RF", {"TreeNum": 10}, 0.75)])
def test_pipeline_on_gpu(tmp_path, alg, params, min_auc):
    import torch
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.utils.synthetic import make_model_set
    assert torch.cuda.is_available()
    root = make_model_set(str(tmp_path), "g", alg, n_rows=4000)
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    mc.train["numTrainEpochs"] = 60
    mc.train["baggingNum"] = 2
    if params:
        mc.train["params"].update(params)
    mc.save()
    _run(root)
    assert _auc(root) > min_auc, _auc(root)


def test_sensitivity_varsel_gpu(tmp_path):
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.utils.synthetic import make_model_set
    root = make_model_set(str(tmp_path), "g", "NN", n_rows=3000)
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    mc.varSelect["filterBy"] = "SE"
    mc.varSelect["filterNum"] = 10
    mc.train["numTrainEpochs"] = 20
    mc.save()
    _run(root, ("init", "stats", "varsel"))
    sel = [c for c in json.load(open(os.path.join(root, "ColumnConfig.json"))) if c["finalSelect"]]
    assert 0 < len(sel) <= 10


def test_posttrain_bin_avg_gpu_matches_cpu(tmp_path, monkeypatch):
    """posttrain binAvgScore through the HIP tree-inference + keyed-count kernels (K13, K18)
    equals the host numpy path on the same model set."""
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.utils.synthetic import make_model_set
    root = make_model_set(str(tmp_path), "g", "GBT", n_rows=4000)
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    mc.train["params"].update({"TreeNum": 10, "MaxDepth": 4})
    mc.save()
    _run(root, ("init", "stats", "norm", "train", "posttrain"))

    def avg():
        return {c["columnName"]: c["columnBinning"]["binAvgScore"]
                for c in json.load(open(os.path.join(root, "ColumnConfig.json")))
                if (c.get("columnBinning") or {}).get("binAvgScore")}
    gpu = avg()
    assert gpu and all(v for v in gpu.values())
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    _run(root, ("posttrain",))
    assert avg() == gpu


@pytest.mark.parametrize("wide,deep", [(True, True), (True, False), (False, True)])
def test_wdl_hip_gather_matches_torch(wide, deep, monkeypatch):
    """K20: the HIP wide-sum / deep-input gather (+ scatter backward) gives the torch path's
    logits and parameter gradients.  The 40000-category field puts the wide offsets of the
    deep-only case far past the 1-float placeholder table (the placeholder must never be
    scattered into)."""
    import numpy as np
    import torch
    from shifu_amd.models import wdl
    torch.manual_seed(0)
    sizes = [3, 40000, 7]
    net = wdl.WideDeepNet(5, sizes, [0, 2], 4, [16], ["relu"], wide=wide, deep=deep).cuda()
    with torch.no_grad():
        for t in net.wide_tables:
            t.normal_()
    n = 3001
    dense = torch.randn(n, 5, device="cuda")
    cats = torch.stack([torch.randint(0, s + 1, (n,)) for s in sizes], 1).cuda()
    out = {}
    monkeypatch.setattr(wdl, "WDL_DEEP_HIP", False)       # fp32 deep tower: the gather is under test
    for hip in (True, False):
        monkeypatch.setattr(wdl, "WDL_HIP", hip)
        net.zero_grad()
        logit = net(dense, cats)
        (logit.sin().sum()).backward()
        out[hip] = (logit.detach().clone(), [None if p.grad is None else p.grad.clone() for p in net.parameters()])
    torch.testing.assert_close(out[True][0], out[False][0], rtol=1e-5, atol=1e-5)
    for a, b in zip(out[True][1], out[False][1]):
        if b is None:
            assert a is None or float(a.abs().max()) == 0.0
        else:
            torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("acts", [["relu"], ["tanh", "sigmoid"], ["swish", "leakyrelu"]])
def test_wdl_deep_mfma_matches_fp32(acts, monkeypatch):
    """K20: the deep tower on the hand-written bf16 MFMA GEMMs (gemm_nt EPI_ACT / EPI_DACT +
    wgrad_tn) against the fp32 torch tower: logits and every parameter gradient within bf16
    accuracy (relative to each tensor's scale)."""
    import torch
    from shifu_amd.models import wdl
    torch.manual_seed(1)
    sizes = [3, 500, 7]
    hidden = [40, 24][: len(acts)]
    net = wdl.WideDeepNet(5, sizes, [0, 1, 2], 6, hidden, acts).cuda()
    n = 5000
    dense = torch.randn(n, 5, device="cuda")
    cats = torch.stack([torch.randint(0, s + 1, (n,)) for s in sizes], 1).cuda()
    out = {}
    for deep_hip in (True, False):
        monkeypatch.setattr(wdl, "WDL_DEEP_HIP", deep_hip)
        net.zero_grad()
        logit = net(dense, cats)
        ((logit.sigmoid() - 0.3) ** 2).sum().backward()
        out[deep_hip] = (logit.detach().clone(), [None if p.grad is None else p.grad.clone() for p in net.parameters()])
    a, b = out[True][0], out[False][0]
    assert float((a - b).abs().max()) <= 3e-2 * max(1.0, float(b.abs().max()))
    for ga, gb in zip(out[True][1], out[False][1]):
        if gb is None:
            continue
        # bf16 activations / deltas: relative Frobenius error (single entries that are sums of many
        # cancelling per-row terms, e.g. a frequent category's embedding row, keep bf16 noise)
        assert float((ga - gb).norm()) <= 3e-2 * max(float(gb.norm()), 1e-6)


def test_wdl_pipeline_on_gpu(tmp_path):
    """WDL through init/stats/norm/train/eval on the GPU (HIP gathers in the training loop)."""
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.utils.synthetic import make_model_set
    root = make_model_set(str(tmp_path), "w", "WDL", n_rows=3000)
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    mc.train["numTrainEpochs"] = 60
    mc.train["baggingNum"] = 1
    mc.train["params"] = {"NumHiddenLayers": 1, "NumHiddenNodes": [16], "ActivationFunc": ["relu"],
                          "LearningRate": 0.01, "NumEmbedOuputs": 4, "WDLL2Reg": 0.0}
    mc.save()
    _run(root, ("init", "stats", "varsel", "norm", "train", "eval"))
    assert _auc(root) > 0.8, _auc(root)
