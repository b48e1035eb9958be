"""GBT on the GPU over 2 ranks (gloo collectives on device tensors, both ranks on cuda:0 of the
one-GPU box; the 8-GPU RCCL run is the driver's): the device-decision level loop
(TreeTrainer._grow_levels_dev -- split decisions on the device, histogram items sized from each
rank's own estimated child sizes) must grow the same trees, byte for byte, as one process over
all rows (DTMaster.doCompute :298-315 sums the workers' histograms the same way)."""
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


def _rows(n=60001, f=70, seed=21):
    rng = np.random.default_rng(seed)
    codes = rng.integers(0, 64, size=(n, f))
    score = codes[:, :8].astype(np.float64) @ rng.normal(size=8) + 4.0 * np.isin(codes[:, 5], [3, 17, 40])
    y = (score > np.median(score)).astype(np.float32)
    is_cat = np.zeros(f, np.uint8)
    is_cat[[5, 9]] = 1
    return codes, y, is_cat


def _run(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    from shifu_amd.models import gbdt as gb
    from shifu_amd.models.gbdt import BinnedData, TreeConfig, TreeTrainer
    from shifu_amd.parallel import dist
    dist.init_from_env("gloo")
    codes, y, is_cat = _rows()
    n = len(y)
    lo, hi = n * rank // world, n * (rank + 1) // world
    d = BinnedData.from_codes(torch.from_numpy(codes[lo:hi]), y[lo:hi], np.full(codes.shape[1], 64), is_cat,
                              device="cuda")
    cfg = TreeConfig("GBT", tree_num=3, max_depth=6, learning_rate=0.1, feature_subset_strategy="ALL",
                     min_instances_per_node=2)
    tt = TreeTrainer(cfg, d)
    assert tt._pipelined(1) and gb.DEV_DECIDE
    tt.train()
    if rank == 0:
        np.savez(out, feat=np.stack([t.feat for t in tt.trees]), thr=np.stack([t.thr for t in tt.trees]),
                 value=np.stack([t.value for t in tt.trees]), cat=np.stack([t.cat_left for t in tt.trees]),
                 err=np.asarray(tt.train_errors))
    dist.shutdown()


def _spawn(world, out):
    ctx = mp.get_context("spawn")
    port = _free_port()
    ps = [ctx.Process(target=_run, args=(r, world, port, out)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(240)
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]


@pytest.mark.gpu
def test_gpu_gbt_two_ranks_match_one(tmp_path):
    a, b = str(tmp_path / "w1.npz"), str(tmp_path / "w2.npz")
    _spawn(1, a)
    _spawn(2, b)
    r1, r2 = np.load(a), np.load(b)
    for k in ("feat", "thr", "value", "cat"):
        np.testing.assert_array_equal(r1[k], r2[k])
    assert (r1["cat"] != 0).any()
    np.testing.assert_allclose(r1["err"], r2["err"], rtol=1e-9)
