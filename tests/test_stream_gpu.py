"""Out-of-core MLP training: host-resident rows (numpy memmap) streamed through HBM give the same
gradients / errors / optimizer trajectory as fully resident rows."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_host_streamed_training_matches_resident(tmp_path):
    from shifu_amd.models.nn import HostRows, MLPSpec, MLPTrainer
    rng = np.random.default_rng(0)
    n, f = 70000, 300
    path = str(tmp_path / "x.npy")
    np.save(path, rng.normal(size=(n, f)).astype(np.float32))
    xm = np.load(path, mmap_mode="r")
    y = (xm[:, 0] - xm[:, 1] > 0).astype(np.float32)
    spec = MLPSpec(f, [64, 32], ["tanh", "sigmoid"], 1, "sigmoid")
    a = MLPTrainer(spec, "cuda", "R", 0.1, seed=5, chunk_rows=16384)
    b = MLPTrainer(spec, "cuda", "R", 0.1, seed=5, chunk_rows=16384)
    da = a.prepare(torch.from_numpy(np.asarray(xm)), y, stream=False)
    db = b.prepare(xm, y, stream=True)
    assert isinstance(db.x, HostRows)
    for _ in range(4):
        ea, eb = a.step(da), b.step(db)
        assert eb == pytest.approx(ea, rel=1e-5, abs=1e-7)
    torch.testing.assert_close(a.params.flat, b.params.flat, rtol=1e-5, atol=1e-6)
    assert b.evaluate(db) == pytest.approx(a.evaluate(da), rel=1e-5)
