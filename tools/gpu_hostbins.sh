# out-of-core trees: host-resident pinned bins vs HBM bins (GPU tests) + 20M-row timing of both
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gbdt.py > gpurun_out/t_hb.log 2>&1 || { echo TESTS_FAILED; exit 1; }
timeout -k 10 300 python -u - > gpurun_out/hostbins_timing.txt 2>&1 <<'PY'
import time, torch, numpy as np
from shifu_amd.models.gbdt import BinnedData, TreeConfig, TreeTrainer, synthetic_binned
d = synthetic_binned(20_000_000, 200, "cuda", seed=3)
codes = d.codes().cpu().numpy()
h = BinnedData.host_resident(codes, d.y.cpu().numpy(), d.nbins, d.is_cat, device="cuda")
for name, data in (("hbm", d), ("host_pinned", h)):
    tr = TreeTrainer(TreeConfig("GBT", tree_num=3, max_depth=7, feature_subset_strategy="ALL"), data)
    tr.train(1); torch.cuda.synchronize()
    t0 = time.perf_counter(); tr.train(2); torch.cuda.synchronize()
    print(name, "ms/round", (time.perf_counter() - t0) / 2 * 1e3, "err", tr.train_errors[-1], flush=True)
PY
echo EXIT $?
