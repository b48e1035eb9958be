"""The whole node for ``init -autotype``, ``encode`` and ``combo`` (reference: the auto-type MR job
InitModelProcessor.java:289-376, one Guagua job per combo sub model ComboModelProcessor.java:278-356,
the encode Pig UDF ModelDataEncodeProcessor.java:77): ``bin/shifu`` starts them under torchrun
with SHIFU_GPUS ranks (gloo on the CPU here, RCCL on a GPU node) and their outputs equal a single
process; combo children started side by side in one process each hold a GPU of their own."""
import json
import os
import socket
import subprocess
import threading
import time

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DS = "example/cancer-judgement/DataStore"


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shifu(cwd, *args, gpus=4):
    env = dict(os.environ, SHIFU_FORCE_CPU="1", SHIFU_GPUS=str(gpus), SHIFU_MASTER_PORT=str(_port()),
               OMP_NUM_THREADS="1")
    r = subprocess.run([os.path.join(REPO, "bin", "shifu"), *args], cwd=cwd, env=env, capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, (args, r.stdout[-3000:], r.stderr[-3000:])
    return r


def _model_set(tmp_path, ref_resources, name, alg="LR"):
    from shifu_amd.cli import main
    from shifu_amd.config.model_config import ModelConfig
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        assert main(["new", name, "-t", alg]) == 0
    finally:
        os.chdir(cwd)
    root = str(tmp_path / name)
    R = os.path.join(ref_resources, DS)
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    mc.dataSet["dataPath"] = R + "/DataSet1"
    mc.dataSet["headerPath"] = R + "/DataSet1/.pig_header"
    mc.evals[0].dataSet["dataPath"] = R + "/EvalSet1"
    mc.evals[0].dataSet["headerPath"] = R + "/EvalSet1/.pig_header"
    mc.train["numTrainEpochs"] = 10
    mc.train["baggingNum"] = 1
    mc.save()
    return root


def _in(root, argv):
    from shifu_amd.cli import main
    cwd = os.getcwd()
    os.chdir(root)
    try:
        return main(argv)
    finally:
        os.chdir(cwd)


def _parts(d):
    return b"".join(open(os.path.join(d, f), "rb").read() for f in sorted(os.listdir(d)) if f.startswith("part-"))


def test_launcher_world4_init_autotype_and_encode_equal_one_process(tmp_path, ref_resources, monkeypatch):
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    root = _model_set(tmp_path, ref_resources, "w4")
    _shifu(root, "init", "-autotype")
    cc4 = json.load(open(os.path.join(root, "ColumnConfig.json")))
    os.remove(os.path.join(root, "ColumnConfig.json"))
    assert _in(root, ["init", "-autotype"]) == 0
    cc1 = json.load(open(os.path.join(root, "ColumnConfig.json")))
    assert [(c["columnName"], c["columnType"], c["columnFlag"]) for c in cc4] == \
        [(c["columnName"], c["columnType"], c["columnFlag"]) for c in cc1]
    # a GBT for the encode (single process), then encode under 4 ranks vs one process
    from shifu_amd.config.model_config import ModelConfig
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    mc.train["algorithm"] = "GBT"
    mc.train["params"] = {"TreeNum": 5, "MaxDepth": 3, "LearningRate": 0.1, "Loss": "squared",
                          "Impurity": "variance", "FeatureSubsetStrategy": "ALL", "MinInstancesPerNode": 5}
    mc.save()
    for v in (["stats"], ["varsel"], ["norm"], ["train"]):
        assert _in(root, v) == 0, v
    _shifu(root, "encode")
    out = os.path.join(root, "tmp", "encodedTrainData")
    assert sum(f.startswith("part-") for f in os.listdir(out)) == 4
    four, hdr4 = _parts(out), open(os.path.join(out, ".pig_header")).read()
    assert _in(root, ["encode"]) == 0
    assert sum(f.startswith("part-") for f in os.listdir(out)) == 1
    assert _parts(out) == four and open(os.path.join(out, ".pig_header")).read() == hdr4


def test_launcher_world4_combo_run_matches_one_process(tmp_path, ref_resources, monkeypatch):
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    roots = {}
    for tag in ("one", "four"):
        root = _model_set(tmp_path, ref_resources, f"c{tag}")
        for v in (["init"], ["stats"], ["varsel"], ["combo", "-new", "LR,GBT,LR"], ["combo", "-init"]):
            assert _in(root, v) == 0, v
        roots[tag] = root
    assert _in(roots["one"], ["combo", "-run"]) == 0
    _shifu(roots["four"], "combo", "-run")
    _shifu(roots["four"], "combo", "-eval")
    assert _in(roots["one"], ["combo", "-eval"]) == 0

    def joined(tag):
        d = os.path.join(roots[tag], f"c{tag}_assemble", "data")
        hdr = open(os.path.join(d, ".pig_header")).read().strip().split("|")
        rows = [l.split("|") for l in _parts(d).decode().strip().split("\n")]
        return hdr, rows
    h1, r1 = joined("one")
    h4, r4 = joined("four")
    assert h1[:-2] == h4[:-2] and len(r1) == len(r4)
    assert [h.replace("cone_", "") for h in h1[-2:]] == [h.replace("cfour_", "") for h in h4[-2:]]
    assert [r[:-2] for r in r1] == [r[:-2] for r in r4]           # raw columns, same row order
    for j in (-2, -1):                                              # the two sub-model score columns
        a = np.array([float(r[j]) for r in r1])
        b = np.array([float(r[j]) for r in r4])
        assert np.abs(a - b).max() < 5.0                           # x1000 scores: sums in another order
    for tag in roots:
        for d in (f"c{tag}_LR_0", f"c{tag}_GBT_1"):
            assert any(f.startswith("model0.") for f in os.listdir(os.path.join(roots[tag], d, "models")))
    auc = [json.load(open(os.path.join(roots[t], f"c{t}_assemble", "evals", "Eval1", "EvalPerformance.json")))
           ["areaUnderRoc"] for t in ("one", "four")]
    assert abs(auc[0] - auc[1]) < 0.02 and min(auc) > 0.8


def test_combo_children_get_distinct_gpus(monkeypatch):
    """Side-by-side combo children (shifu.combo.parallel > 1, one process): each child holds one
    GPU of the node for all its verbs, and no two running children ever share one."""
    from shifu_amd.runtime import executor
    seen, lock = [], threading.Lock()

    def fake_run_cli(args, cwd, env=None, log_path=None):
        t0 = time.perf_counter()
        time.sleep(0.05)
        with lock:
            seen.append((cwd, env["HIP_VISIBLE_DEVICES"], env["LOCAL_RANK"], t0, time.perf_counter()))
        return 0
    monkeypatch.setattr(executor, "run_cli", fake_run_cli)
    pool = executor.DevicePool(["3", "5", "6"])
    tasks = [executor.cli_task(["stats", "norm", "train"], f"sub{i}", devices=pool) for i in range(7)]
    executor.ExecutorManager(len(pool), 0).run(tasks)
    assert len(seen) == 21
    by_task = {}
    for cwd, dev, lr, _, _ in seen:
        assert "," not in dev and lr == "0"
        by_task.setdefault(cwd, set()).add(dev)
    assert all(len(v) == 1 for v in by_task.values())            # one GPU for the whole task
    spans = {}
    for cwd, dev, _, t0, t1 in seen:
        a, b, _ = spans.get(cwd, (t0, t1, dev))
        spans[cwd] = (min(a, t0), max(b, t1), dev)
    items = list(spans.values())
    for i in range(len(items)):
        for j in range(i + 1, len(items)):
            (a0, a1, da), (b0, b1, db) = items[i], items[j]
            if a0 < b1 and b0 < a1:
                assert da != db                                     # overlapping children: distinct GPUs
    assert sorted(pool.ids) == ["3", "5", "6"] and pool._free.qsize() == 3


def test_device_pool_follows_visible_devices(monkeypatch):
    import torch
    from shifu_amd.runtime.executor import DevicePool
    monkeypatch.delenv("SHIFU_FORCE_CPU", raising=False)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 3)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "4,6,7")
    assert DevicePool.for_node().ids == ["4", "6", "7"]
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    monkeypatch.delenv("CUDA_VISIBLE_DEVICES", raising=False)
    assert DevicePool.for_node().ids == ["0", "1", "2"]
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 0)
    assert DevicePool.for_node() is None
