"""Failure handling: a job killed by the fault hook on ONE process resumes on TWO
gloo ranks (elastic world-size change: rows re-sharded on load, replicated optimizer / tree
state from the checkpoint) and ends with the uninterrupted model; a rank that stops making
progress is aborted by the iteration watchdog."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from tests.test_synthetic_models import _mc, _run


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_train(rank, world, port, root):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), SHIFU_FORCE_CPU="1")
    os.environ.pop("SHIFU_FAULT_AT_ITER", None)
    os.chdir(root)
    from shifu_amd.cli import main
    rc = main(["train"])
    if rc != 0:
        raise SystemExit(rc)


def _setup(tmp_path, alg, names):
    from shifu_amd.utils.synthetic import make_model_set
    roots = []
    for name in names:
        root = make_model_set(str(tmp_path), name, alg, n_rows=600)
        mc = _mc(root)
        mc.train["numTrainEpochs"] = 12
        mc.train["baggingNum"] = 1
        mc.train["validSetRate"] = 0.0
        if alg == "GBT":
            mc.train["params"].update({"TreeNum": 12, "MaxDepth": 3, "CheckpointInterval": 4})
        else:
            mc.train["params"]["CheckpointInterval"] = 4
        mc.save()
        _run(root, ["init", "stats", "norm"])
        roots.append(root)
    return roots


@pytest.mark.parametrize("alg", ["NN", "GBT"])
def test_fault_on_one_rank_resume_on_two(tmp_path, alg):
    a, b = _setup(tmp_path, alg, ("a", "b"))
    env = dict(os.environ, SHIFU_FORCE_CPU="1", SHIFU_FAULT_AT_ITER="8", PYTHONPATH=os.getcwd())
    r = subprocess.run([sys.executable, "-m", "shifu_amd.cli", "train"], cwd=a, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 17, r.stderr[-2000:]
    mp.start_processes(_rank_train, args=(2, _port(), a), nprocs=2, join=True, start_method="spawn")
    _run(b, ["train"])                               # uninterrupted single-process reference
    if alg == "NN":
        from shifu_amd.formats.nn_format import read_encog
        wa = read_encog(os.path.join(a, "models/model0.nn")).weights
        wb = read_encog(os.path.join(b, "models/model0.nn")).weights
        for x, y in zip(wa, wb):
            np.testing.assert_allclose(x, y, rtol=1e-4, atol=1e-5)
    else:
        from shifu_amd.formats.tree_format import read_tree_model
        ta = read_tree_model(os.path.join(a, "models/model0.gbt"))
        tb = read_tree_model(os.path.join(b, "models/model0.gbt"))
        assert len(ta.bags[0]) == len(tb.bags[0]) == 12
        x = {c: np.linspace(-3, 3, 50) for c in ta.names}
        np.testing.assert_allclose(ta.score(x, 50), tb.score(x, 50), rtol=1e-5)


def test_watchdog_aborts_hung_rank(tmp_path):
    (a,) = _setup(tmp_path, "NN", ("w",))
    env = dict(os.environ, SHIFU_FORCE_CPU="1", SHIFU_FAULT_HANG_AT_ITER="3", SHIFU_ITERATION_TIMEOUT="2",
               PYTHONPATH=os.getcwd())
    r = subprocess.run([sys.executable, "-m", "shifu_amd.cli", "train"], cwd=a, env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 18, r.stderr[-2000:]
    assert "watchdog" in r.stderr


def test_watchdog_stops_when_training_raises(tmp_path, monkeypatch):
    """A training error raised inside the loop (check_finite) ends the watchdog thread too, so a
    process that catches the error is not aborted one timeout later."""
    import threading
    import time
    from shifu_amd.steps import train as train_mod
    (a,) = _setup(tmp_path, "NN", ("x",))
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    monkeypatch.setenv("SHIFU_ITERATION_TIMEOUT", "1")

    def boom(name, value, it):
        raise FloatingPointError("forced")
    monkeypatch.setattr(train_mod, "check_finite", boom)
    with pytest.raises((FloatingPointError, AssertionError)):   # raised, or a non-zero exit code
        _run(a, ["train"])
    time.sleep(1.5)
    assert not [t for t in threading.enumerate() if t.name == "shifu-watchdog" and t.is_alive()]
