"""SVM (legacy LOCAL, SVMTrainer.java:38-185): the SMO/WSS3 solver matches libsvm (scikit-learn's
SVC wraps libsvm, the same solver Encog ports) on decision values for every kernel, the
reference's XOR test set is learned with its RBF params, and the .svm artifact round-trips."""
import numpy as np
import pytest


@pytest.mark.parametrize("kernel", ["linear", "poly", "rbf", "sigmoid"])
def test_svm_matches_libsvm(kernel):
    from sklearn.svm import SVC
    from shifu_amd.models import svm as S
    rng = np.random.default_rng(3)
    X = rng.normal(size=(300, 5)).astype(np.float32)
    y = ((X[:, 0] + 0.5 * X[:, 1] ** 2 + 0.3 * rng.normal(size=300)) > 0.4).astype(np.float64)
    gamma = 0.3 if kernel != "sigmoid" else 0.05
    m = S.train_svm(X, y, kernel, C=1.0, gamma=gamma, eps=1e-5)
    ref = SVC(C=1.0, kernel=kernel, gamma=gamma, degree=3, coef0=0.0, tol=1e-5, shrinking=False).fit(X, y)
    Xt = rng.normal(size=(200, 5)).astype(np.float32)
    d = m.decision(Xt)
    dr = ref.decision_function(Xt)
    sign = 1.0 if m.labels[0] == ref.classes_[1] else -1.0
    np.testing.assert_allclose(sign * d, dr, rtol=2e-3, atol=2e-3)
    assert (m.predict(Xt) == ref.predict(Xt)).mean() > 0.99


def test_svm_reference_xor_rbf(tmp_path):
    from shifu_amd.models import svm as S
    X = np.array([[0, 0]] * 5 + [[0, 1]] * 5 + [[1, 0]] * 5 + [[1, 1]] * 5, np.float32)
    y = np.array([0] * 5 + [1] * 10 + [0] * 5, np.float64)
    m = S.train_svm(X, y, S.kernel_name("rbf"), C=1.1, gamma=0.95)
    v = np.array([[0, 0], [0, 1], [1, 0], [1, 1]], np.float32)
    np.testing.assert_array_equal(m.predict(v), [0, 1, 1, 0])
    p = str(tmp_path / "model0.svm")
    S.write_svm(p, m, 2)
    assert open(p).readline().startswith("encog,SVM,java,3.0.0")
    m2 = S.read_svm(p)
    np.testing.assert_allclose(m2.decision(v), m.decision(v), rtol=1e-12, atol=1e-12)


def test_svm_train_step(tmp_path, monkeypatch):
    """`shifu train` with algorithm SVM writes models/model0.svm (CPU LOCAL path)."""
    import os
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.steps import api
    from shifu_amd.utils.synthetic import make_model_set
    root = make_model_set(str(tmp_path), "s", "SVM", n_rows=600, n_num=6, n_cat=1)
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    mc.train["baggingNum"] = 1
    mc.train["params"] = {"Kernel": "rbf", "Gamma": 0.2, "Const": 1.0}
    mc.save()
    for cls in (api.InitStep, api.StatsStep, api.NormStep, api.TrainStep):
        cls(root).process()
    from shifu_amd.models import svm as S
    m = S.read_svm(os.path.join(root, "models", "model0.svm"))
    assert len(m.coef) > 0 and m.kernel == "rbf"


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["linear", "rbf"])
def test_svm_gpu_batched_smo_matches_host_loop(kernel, monkeypatch):
    """svm_kernels.hip (SMO_BATCH iterations per launch, one host sync per batch) takes the same
    working sets as the host-driven loop: same iteration count, alphas and rho; and it matches
    libsvm's decision values like the CPU solver does."""
    import time
    import torch
    from sklearn.svm import SVC
    from shifu_amd.models import svm as S
    g = np.random.default_rng(3)
    X = g.normal(size=(1500, 6)).astype(np.float32)
    y = ((X[:, 0] * X[:, 1] + 0.3 * X[:, 2]) > 0).astype(np.float64)
    logs = []
    t0 = time.perf_counter()
    m1 = S.train_svm(X, y, kernel, C=1.0, gamma=0.5, eps=1e-4, device="cuda", log=logs.append)
    t1 = time.perf_counter()
    monkeypatch.setenv("SHIFU_SVM_HOST_LOOP", "1")
    logs2 = []
    m2 = S.train_svm(X, y, kernel, C=1.0, gamma=0.5, eps=1e-4, device="cuda", log=logs2.append)
    t2 = time.perf_counter()
    print(f"batched {t1 - t0:.3f}s vs host loop {t2 - t1:.3f}s: {logs[-1]} | {logs2[-1]}")
    assert logs[-1].split(",")[0] == logs2[-1].split(",")[0]          # same iteration count
    np.testing.assert_allclose(m1.coef, m2.coef, rtol=1e-9, atol=1e-12)
    assert abs(m1.rho - m2.rho) < 1e-9
    ref = SVC(kernel=kernel, C=1.0, gamma=0.5, tol=1e-4).fit(X.astype(np.float64), y)
    d_ref = ref.decision_function(X.astype(np.float64))
    d = m1.decision(X, device="cuda")
    sgn = 1.0 if ref.classes_[1] == m1.labels[0] else -1.0
    np.testing.assert_allclose(sgn * d, d_ref, atol=5e-3 * max(1.0, float(np.abs(d_ref).max())))


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["linear", "poly", "sigmoid", "rbf"])
def test_gram_gpu_own_gemm_fp32_accurate(kernel):
    """The GPU kernel matrix runs on the own split-bf16 MFMA GEMM (6 terms, fp32-accurate products):
    within fp32 rounding of an fp64 reference."""
    import torch
    from shifu_amd.models import svm as S
    g = np.random.default_rng(5)
    A = g.normal(size=(3000, 37)).astype(np.float32)
    B = g.normal(size=(1100, 37)).astype(np.float32)
    K = S.gram(torch.as_tensor(A).cuda(), torch.as_tensor(B).cuda(), kernel, 0.05, 3, 0.5).cpu().double().numpy()
    ref = S.gram(torch.as_tensor(A).double(), torch.as_tensor(B).double(), kernel, 0.05, 3, 0.5).numpy()
    np.testing.assert_allclose(K, ref, rtol=2e-5, atol=2e-5 * max(1.0, float(np.abs(ref).max())))
