"""``algorithm: TENSORFLOW`` (E5): the torch-native replacement of the reference's TF DNN
trainer (src/main/python/train.py + TensorflowTrainer) end to end: new -> init -> stats ->
norm -> varsel -> train (mini-batch DNN, generic model under models/<name>/) -> eval (generic
scorer), plus the world-size-2 gloo run training the identical model as one process."""
import json
import os

import numpy as np
import pytest
import torch


def _tf_model_set(tmp_path, name="tf"):
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.utils.synthetic import make_model_set
    root = make_model_set(str(tmp_path), name, "TENSORFLOW", n_rows=1500)
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    mc.train["numTrainEpochs"] = 6
    p = mc.train["params"]
    p.update({"NumHiddenNodes": [16], "ActivationFunc": ["tanh"], "LearningRate": 0.01, "MiniBatchs": 64,
              "TF.optimizer": "adam", "TF.loss": "log", "CheckpointInterval": 3})
    mc.save()
    return root


def test_tensorflow_pipeline(tmp_path, monkeypatch):
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    from shifu_amd.cli import main
    root = _tf_model_set(tmp_path)
    monkeypatch.chdir(root)
    for cmd in (["init"], ["stats"], ["norm"], ["varsel"], ["train"]):
        assert main(cmd) == 0, cmd
    cfg = json.load(open("models/tf/GenericModelConfig.json"))
    assert cfg["properties"]["algorithm"] == "safetensors_mlp"
    assert cfg["properties"]["activations"] == ["tanh", "sigmoid"]
    assert os.path.exists("models/tf-checkpoint-3/GenericModelConfig.json")
    assert main(["eval"]) == 0
    perf = json.load(open("evals/Eval1/EvalPerformance.json"))
    assert perf["areaUnderRoc"] > 0.75


def test_dnn_sgd_matches_manual_adam():
    """One mini-batch step of train_dnn equals torch's own Adam on the same MSE(+L2) objective."""
    from shifu_amd.models.dnn_sgd import DNN, train_dnn
    g = np.random.default_rng(0)
    X = g.normal(size=(40, 5)).astype(np.float32)
    y = (X[:, 0] > 0).astype(np.float32)
    w = np.ones(40, np.float32)
    valid = np.zeros(40, bool)
    params = {"NumHiddenNodes": [4], "ActivationFunc": ["sigmoid"], "LearningRate": 0.05, "MiniBatchs": 40}
    m, hist = train_dnn(X, y, w, valid, params, 1, torch.device("cpu"), seed=3)
    ref = DNN(5, [4], ["sigmoid"], None, 3)
    opt = torch.optim.Adam(ref.parameters(), lr=0.05)
    p = ref(torch.tensor(X))
    loss = ((p - torch.tensor(y)[:, None]) ** 2).mean() + 0.01 * sum((W ** 2).sum() for W in ref.W) / 2
    loss.backward()
    opt.step()
    for a, b in zip(m.parameters(), ref.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def _dp_run(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), SHIFU_FORCE_CPU="1")
    from shifu_amd.models.dnn_sgd import train_dnn
    from shifu_amd.parallel import dist
    dist.init_from_env("gloo")
    X, y = _dp_data()
    n = len(y)
    lo, hi = n * rank // world, n * (rank + 1) // world
    m, _ = train_dnn(X[lo:hi], y[lo:hi], np.ones(hi - lo, np.float32), np.zeros(hi - lo, bool), _DP_PARAMS, 3,
                     torch.device("cpu"), seed=5)
    torch.save([p.detach() for p in m.parameters()], os.path.join(out, f"r{rank}.pt"))
    dist.shutdown()


_DP_PARAMS = {"NumHiddenNodes": [6], "ActivationFunc": ["relu"], "LearningRate": 0.02, "MiniBatchs": 50,
              "TF.optimizer": "rmsprop", "TF.loss": "squared"}


def _dp_data():
    g = np.random.default_rng(1)
    X = g.normal(size=(400, 7)).astype(np.float32)
    return X, (X[:, 1] + 0.3 * X[:, 2] > 0).astype(np.float32)


def test_dnn_sgd_two_ranks_match_single(tmp_path):
    """World size 2 (gloo): per-batch gradient all-reduce == one process over the union batches."""
    import socket
    import torch.multiprocessing as mp
    from shifu_amd.models.dnn_sgd import train_dnn
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.start_processes(_dp_run, args=(2, port, str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    r0, r1 = (torch.load(os.path.join(tmp_path, f"r{r}.pt"), weights_only=True) for r in (0, 1))
    X, y = _dp_data()
    # single-process batches = union of the ranks' batch i (ranks hold rows [0,200) and [200,400))
    order = np.concatenate([np.r_[i * 50:(i + 1) * 50, 200 + i * 50:200 + (i + 1) * 50] for i in range(4)])
    p = dict(_DP_PARAMS, MiniBatchs=100)
    m, _ = train_dnn(X[order], y[order], np.ones(400, np.float32), np.zeros(400, bool), p, 3,
                     torch.device("cpu"), seed=5)
    for a, b, c in zip(r0, r1, m.parameters()):
        torch.testing.assert_close(a, b)
        torch.testing.assert_close(a, c.detach(), rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("opt,loss,act", [("adam", "squared", "sigmoid"), ("rmsprop", "log", "tanh"),
                                          ("gradientdescent", "absolute", "relu"),
                                          ("adam", "log", "leakyrelu")])
def test_mlp_engine_matches_autograd_oracle(opt, loss, act):
    """The MLP-engine TENSORFLOW trainer (own kernels' CPU oracle, no flat spot, TF leaky slope,
    optimizer_kernel's TF rules) trains the same weights as torch autograd + torch.optim."""
    from shifu_amd.models.dnn_sgd import train_dnn, train_dnn_autograd
    g = np.random.default_rng(4)
    X = g.normal(size=(300, 9)).astype(np.float32)
    y = (X[:, 0] - X[:, 3] > 0).astype(np.float32)
    w = (g.random(300) < 0.9).astype(np.float32) * 1.5         # some zero weights: nonzero-count mean
    valid = g.random(300) < 0.2
    p = {"NumHiddenNodes": [8, 5], "ActivationFunc": [act, act], "LearningRate": 0.02, "MiniBatchs": 32,
         "TF.optimizer": opt, "TF.loss": loss}
    m1, h1 = train_dnn(X, y, w, valid, p, 3, torch.device("cpu"), seed=7)
    m2, h2 = train_dnn_autograd(X, y, w, valid, p, 3, torch.device("cpu"), seed=7)
    for a, b in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(a.detach(), b.detach(), rtol=2e-4, atol=2e-5)
    np.testing.assert_allclose([v for _, _, v in h1], [v for _, _, v in h2], rtol=1e-4)
    # the per-epoch training error is the TF objective sum(w * loss) / count(w != 0) in both
    np.testing.assert_allclose([t for _, t, _ in h1], [t for _, t, _ in h2], rtol=1e-4)


@pytest.mark.gpu
def test_mlp_engine_tf_gpu_tracks_autograd():
    """On the GPU the TENSORFLOW trainer runs the bf16 MFMA kernels + shifu_optimizer_step_tf; it
    tracks the fp32 autograd oracle within bf16 rounding over a few epochs."""
    from shifu_amd.models.dnn_sgd import train_dnn, train_dnn_autograd
    from shifu_amd.ops import _native
    _native.require_gpu_native()
    g = np.random.default_rng(4)
    X = g.normal(size=(4000, 30)).astype(np.float32)
    y = (X[:, 0] - X[:, 3] > 0).astype(np.float32)
    w = np.ones(4000, np.float32)
    valid = g.random(4000) < 0.2
    p = {"NumHiddenNodes": [32, 16], "ActivationFunc": ["tanh", "leakyrelu"], "LearningRate": 0.01,
         "MiniBatchs": 256, "TF.optimizer": "adam", "TF.loss": "log"}
    m1, h1 = train_dnn(X, y, w, valid, p, 4, torch.device("cuda"), seed=2)
    m2, h2 = train_dnn_autograd(X, y, w, valid, p, 4, torch.device("cpu"), seed=2)
    v1, v2 = [v for _, _, v in h1], [v for _, _, v in h2]
    assert v1[-1] < v1[0]
    np.testing.assert_allclose(v1, v2, rtol=0.05)
    np.testing.assert_allclose([t for _, t, _ in h1], [t for _, t, _ in h2], rtol=0.05)
    for a, b in zip(m1.parameters(), m2.parameters()):
        assert float((a.detach() - b.detach()).abs().max()) < 0.05
