"""Device-decision GBDT path vs host path: first differing tree / level, pred after each tree."""
import sys, os, json
sys.path.insert(0, os.getcwd())
import numpy as np
import torch
from shifu_amd.models import gbdt as gb
from shifu_amd.models.gbdt import BinnedData, TreeConfig, TreeTrainer

rng = np.random.default_rng(5)
n, f, nb = 20000, 40, 64
codes = rng.integers(0, nb, size=(n, f))
y = ((codes[:, 0] > nb // 2) ^ (codes[:, 1] < 3)).astype(np.float32)
y = np.where(rng.random(n) < 0.05, 1 - y, y)
is_cat = np.zeros(f, np.uint8)
is_cat[3] = int(sys.argv[1]) if len(sys.argv) > 1 else 1
data = BinnedData.from_codes(codes, y, np.full(f, nb), is_cat, device="cuda")
cfg = TreeConfig("GBT", tree_num=4, max_depth=5, learning_rate=0.2, feature_subset_strategy="ALL")
trs = {}
for dd in (True, False):
    gb.DEV_DECIDE = dd
    tr = TreeTrainer(cfg, data)
    preds = []
    for t in range(4):
        tr.train(1)
        preds.append(tr.pred.clone())
    trs[dd] = (tr, preds)
a, pa = trs[True]
b, pb = trs[False]
for t in range(4):
    x, z = a.trees[t], b.trees[t]
    out = {"tree": t, "feat_eq": bool((x.feat == z.feat).all()), "thr_eq": bool((x.thr == z.thr).all()),
           "val_eq": bool(np.array_equal(x.value, z.value)), "pred_eq": bool(torch.equal(pa[t], pb[t])),
           "pred_maxdiff": float((pa[t] - pb[t]).abs().max())}
    if not out["feat_eq"]:
        out["feat_dev"] = x.feat.tolist(); out["feat_host"] = z.feat.tolist()
    if not out["val_eq"]:
        out["val_dev"] = x.value.tolist(); out["val_host"] = z.value.tolist()
    print(json.dumps(out), flush=True)
print(json.dumps({"levels_dev": a.last_tree_stats["levels"], "levels_host": b.last_tree_stats["levels"]}))
