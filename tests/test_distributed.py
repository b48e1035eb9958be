"""Multi-process data parallelism on the CPU (gloo, world_size 2, 127.0.0.1): the all-reduced
training of 2 ranks over row shards must equal single-process training over all rows
(parity model: the reference's Guagua master/worker sums — NNMaster.doCompute :240-249,
DTMaster.doCompute :298-315)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(n=600, f=12, seed=0):
    rng = np.random.default_rng(seed)
    x = rng.normal(size=(n, f)).astype(np.float32)
    y = (x[:, 0] - 0.5 * x[:, 1] + 0.3 * rng.normal(size=n) > 0).astype(np.float32)
    return x, y


def _mlp_run(rank, world, port, out, steps):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), SHIFU_FORCE_CPU="1")
    from shifu_amd.models.nn import MLPSpec, MLPTrainer
    from shifu_amd.parallel import dist
    dist.init_from_env("gloo")
    x, y = _data()
    n = len(y)
    lo, hi = n * rank // world, n * (rank + 1) // world
    tr = MLPTrainer(MLPSpec(x.shape[1], [8], ["tanh"], 1, "sigmoid"), "cpu", "R", 0.1, seed=3)
    d = tr.prepare(torch.from_numpy(x[lo:hi]), y[lo:hi].reshape(-1, 1))
    errs = [tr.step(d, num_train_global=float(n)) for _ in range(steps)]
    if rank == 0:
        torch.save({"w": tr.params.flat.clone(), "errs": errs}, out)
    dist.shutdown()


def _gbdt_run(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), SHIFU_FORCE_CPU="1")
    from shifu_amd.models.gbdt import BinnedData, TreeConfig, TreeTrainer
    from shifu_amd.parallel import dist
    dist.init_from_env("gloo")
    rng = np.random.default_rng(1)
    n, f = 800, 6
    codes = rng.integers(0, 16, size=(n, f))
    y = ((codes[:, 0] > 7) ^ (codes[:, 1] > 11)).astype(np.float32)
    lo, hi = n * rank // world, n * (rank + 1) // world
    d = BinnedData.from_codes(torch.from_numpy(codes[lo:hi]), y[lo:hi], np.full(f, 16))
    cfg = TreeConfig("GBT", tree_num=3, max_depth=4, learning_rate=0.1, feature_subset_strategy="ALL",
                     min_instances_per_node=2)
    tt = TreeTrainer(cfg, d)
    tt.train()
    if rank == 0:
        torch.save({"feat": [t.feat.copy() for t in tt.trees], "thr": [t.thr.copy() for t in tt.trees],
                    "value": [t.value.copy() for t in tt.trees], "err": tt.train_errors}, out)
    dist.shutdown()


def _spawn(fn, world, *args):
    ctx = mp.get_context("spawn")
    port = _free_port()
    ps = [ctx.Process(target=fn, args=(r, world, port) + args) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]


def test_mlp_data_parallel_matches_single(tmp_path):
    a, b = str(tmp_path / "w1.pt"), str(tmp_path / "w2.pt")
    _spawn(_mlp_run, 1, a, 5)
    _spawn(_mlp_run, 2, b, 5)
    r1, r2 = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    np.testing.assert_allclose(r1["errs"], r2["errs"], rtol=1e-4)
    torch.testing.assert_close(r1["w"], r2["w"], rtol=1e-4, atol=1e-5)


def test_gbdt_data_parallel_matches_single(tmp_path):
    a, b = str(tmp_path / "t1.pt"), str(tmp_path / "t2.pt")
    _spawn(_gbdt_run, 1, a)
    _spawn(_gbdt_run, 2, b)
    r1, r2 = torch.load(a, weights_only=False), torch.load(b, weights_only=False)
    for k in range(3):
        np.testing.assert_array_equal(r1["feat"][k], r2["feat"][k])
        np.testing.assert_array_equal(r1["thr"][k], r2["thr"][k])
        np.testing.assert_allclose(r1["value"][k], r2["value"][k], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(r1["err"], r2["err"], rtol=1e-5)


@pytest.mark.skipif(not hasattr(torch.distributed, "is_available") or not torch.distributed.is_available(),
                    reason="no torch.distributed")
def test_bucketed_allreducer_two_ranks(tmp_path):
    _spawn(_bucket_run, 2, str(tmp_path / "b.pt"))
    r = torch.load(str(tmp_path / "b.pt"), weights_only=True)
    torch.testing.assert_close(r["a"], torch.full((1000,), 3.0))
    torch.testing.assert_close(r["b"], torch.full((7, 5), 3.0))


def _bucket_run(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), SHIFU_FORCE_CPU="1")
    from shifu_amd.parallel import dist
    dist.init_from_env("gloo")
    flat = torch.full((1035,), float(rank + 1))
    red = dist.BucketedAllReducer(flat, bucket_bytes=1024)
    red.launch_from(600)          # back-to-front partial launch, then the rest
    red.wait()
    if rank == 0:
        torch.save({"a": flat[:1000].clone(), "b": flat[1000:].view(7, 5).clone()}, out)
    dist.shutdown()


def _mlp_overlap_run(rank, world, port, out, overlap):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), SHIFU_FORCE_CPU="1")
    if overlap:
        os.environ["SHIFU_GRAD_OVERLAP"] = "1"
        os.environ["SHIFU_GRAD_BUCKET_MB"] = "0.0002"        # ~200 B buckets: many per layer
    from shifu_amd.models.nn import MLPSpec, MLPTrainer
    from shifu_amd.parallel import dist
    dist.init_from_env("gloo")
    x, y = _data()
    n = len(y)
    lo, hi = n * rank // world, n * (rank + 1) // world
    tr = MLPTrainer(MLPSpec(x.shape[1], [16, 8], ["tanh", "sigmoid"], 1, "sigmoid"), "cpu", "R", 0.1, seed=3,
                    chunk_rows=64)
    assert (tr._reducer is not None) == bool(overlap)
    d = tr.prepare(torch.from_numpy(x[lo:hi]), y[lo:hi].reshape(-1, 1))
    errs = [tr.step(d, num_train_global=float(n)) for _ in range(4)]
    if rank == 0:
        torch.save({"w": tr.params.flat.clone(), "errs": errs}, out)
    dist.shutdown()


def test_mlp_bucketed_overlap_equals_single_allreduce(tmp_path):
    """Buckets launched back-to-front during the last chunk's backward (BucketedAllReducer) give
    bitwise the same training as one all-reduce after the backward."""
    a, b = str(tmp_path / "o0.pt"), str(tmp_path / "o1.pt")
    _spawn(_mlp_overlap_run, 2, a, False)
    _spawn(_mlp_overlap_run, 2, b, True)
    r1, r2 = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    assert r1["errs"] == r2["errs"]
    assert torch.equal(r1["w"], r2["w"])
