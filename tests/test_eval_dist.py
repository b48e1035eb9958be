"""K16 multi-rank EvalPerformance (algos/eval_dist.py): rows sharded over 2 / 3 gloo ranks (rank-
major = the single-process row order) give the single-process ``evaluation.performance`` result:
identical buckets, positions and counts, weighted sums within summation-order rounding.  Cases:
heavy ties straddling rank boundaries, NaN / -inf scores, a rank with no rows, no negatives."""
import json
import os

import numpy as np
import pytest
import torch

from test_distributed import _free_port, _spawn


def _case(seed, n):
    rng = np.random.default_rng(seed)
    s = np.round(rng.random(n) * 40.0) * 25.0               # integer-ish scores: heavy ties
    if seed % 2:
        s[rng.random(n) < 0.03] = np.nan
        s[rng.random(n) < 0.02] = -np.inf
    y = (rng.random(n) < 0.3).astype(np.float64)
    if seed == 3:
        y[:] = 1.0                                           # no negatives: NaN roc curve
    w = rng.random(n) * 2.0
    return s, y, w


def _run(rank, world, port, out, seed, n, cuts):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), SHIFU_FORCE_CPU="1")
    from shifu_amd.algos import eval_dist
    from shifu_amd.parallel import dist
    dist.init_from_env("gloo")
    s, y, w = _case(seed, n)
    lo, hi = cuts[rank], cuts[rank + 1]
    res = eval_dist.performance(s[lo:hi], y[lo:hi], w[lo:hi], 10, max_score=1000.0, device=torch.device("cpu"))
    if rank == 0:
        with open(out, "w") as f:
            json.dump(res, f)
    dist.shutdown()


def _close(a, b, path="", weighted=False):
    if isinstance(a, dict):
        assert a.keys() == b.keys(), path
        for k in a:
            _close(a[k], b[k], path + "/" + k, weighted or k.lower().startswith("weight") or "Wgt" in k)
    elif isinstance(a, list):
        assert len(a) == len(b), path
        for i, (x, z) in enumerate(zip(a, b)):
            _close(x, z, f"{path}[{i}]", weighted)
    elif isinstance(a, float):
        if np.isnan(a):
            assert np.isnan(b), path
        elif a == b:
            pass
        elif weighted:
            assert abs(a - b) <= 1e-12 * max(1.0, abs(a)), (path, a, b)
        else:
            assert a == b, (path, a, b)
    else:
        assert a == b, path


@pytest.mark.parametrize("seed,n,cuts", [(0, 3000, [0, 1400, 3000]), (1, 2500, [0, 900, 900, 2500]),
                                         (2, 4000, [0, 1000, 2500, 4000]), (3, 1200, [0, 600, 1200])])
def test_dist_performance_matches_single(tmp_path, seed, n, cuts):
    from shifu_amd.algos import evaluation as E
    s, y, w = _case(seed, n)
    ref = json.loads(json.dumps(E.performance(s, y, w, 10, max_score=1000.0, device=torch.device("cpu"))))
    out = str(tmp_path / "p.json")
    _spawn(_run, len(cuts) - 1, out, seed, n, cuts)
    got = json.load(open(out))
    _close(ref, got)
