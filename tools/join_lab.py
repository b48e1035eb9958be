"""Stage timings of the streamed row join (data/join.py) and the auto-type scan
(algos/autotype.py) on a generated '|'-delimited text set (native generator).

    python tools/join_lab.py --rows 200000 --cols 1600 [--work /tmp/join_lab] [--steps scan,join]
"""
import argparse
import json
import os
import shutil
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=200000)
    ap.add_argument("--cols", type=int, default=1600)
    ap.add_argument("--work", default="/tmp/join_lab")
    ap.add_argument("--steps", default="read,scan,join")
    ap.add_argument("--block-mb", type=int, default=256)
    ap.add_argument("--threads", type=int, default=min(16, os.cpu_count() or 4))
    ap.add_argument("--parse-cols", type=int, default=200, help="numeric columns the join's compute reads")
    a = ap.parse_args()
    from shifu_amd.data.join import FIXED6, STATS, raw_blocks, stream_join
    from shifu_amd.data.purifier import DatasetPlan
    from shifu_amd.data.reader import column_kinds
    from shifu_amd.ops import _native
    shutil.rmtree(a.work, ignore_errors=True)
    d = os.path.join(a.work, "data")
    os.makedirs(d)
    t0 = time.perf_counter()
    if _native.rt().shifu_gen_csv(d.encode(), a.rows, a.cols, 3, 11, 0.02, 20, a.threads):
        raise SystemExit("generation failed")
    hdr = ["id", "diagnosis", "wgt"] + [f"num_{j}" for j in range(a.cols)] + [f"cat_{j}" for j in range(3)]
    gen = time.perf_counter() - t0
    size = sum(os.path.getsize(os.path.join(d, f)) for f in os.listdir(d))
    nums = [f"num_{j}" for j in range(min(a.parse_cols, a.cols))]
    plan = DatasetPlan(data_path=d, delim="|", header=hdr, skip_header_line=False, target="diagnosis", weight=None,
                       filt=None, nums=nums, strs=[], seg_names=[], seg_exprs=[], missing=["", "?"])
    out = {"rows": a.rows, "cols": a.cols, "gb": round(size / 1e9, 2), "gen_s": round(gen, 2), "threads": a.threads}
    steps = a.steps.split(",")
    block = a.block_mb << 20
    if "read" in steps:
        t0 = time.perf_counter()
        nb = sum(len(x[2]) for x in raw_blocks(plan, 0, 1, block))
        out["read_s"] = round(time.perf_counter() - t0, 2)
        out["read_gbs"] = round(nb / 1e9 / out["read_s"], 2)
    if "scan" in steps:
        from shifu_amd.algos import autotype
        from shifu_amd.config.model_config import ModelConfig
        from shifu_amd.utils.synthetic import make_model_set
        root = make_model_set(a.work, "m", "NN", n_rows=100)
        mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
        for k, v in dict(dataPath=d, headerPath=None, targetColumnName="diagnosis", posTags=["M"], negTags=["B"],
                         weightColumnName=None, filterExpressions=None).items():
            mc.dataSet[k] = v
        autotype.STATS.clear()
        t0 = time.perf_counter()
        autotype.scan(mc, hdr, list(range(len(hdr))), nthreads=a.threads, block_bytes=block)
        out["scan_s"] = round(time.perf_counter() - t0, 2)
        out["scan_native_s"] = round(autotype.STATS.get("feed_s", 0.0), 2)
        out["scan_finish_s"] = round(autotype.STATS.get("finish_s", 0.0), 2)
        out["scan_gbs"] = round(size / 1e9 / out["scan_s"], 2)
    if "join" in steps:
        kinds = column_kinds(hdr, nums, [])
        STATS.clear()

        def compute(table, n):
            s = np.zeros(n)
            for c in nums:
                s += np.nan_to_num(table[c].numeric())
            return [(FIXED6, s)]
        t0 = time.perf_counter()
        stream_join(plan, os.path.join(a.work, "joined"), ["s"], kinds, compute, block_bytes=block, nthreads=a.threads)
        out["join_s"] = round(time.perf_counter() - t0, 2)
        out["join_gbs"] = round(size / 1e9 / out["join_s"], 2)
        out["join_stages_s"] = {k: round(v, 2) for k, v in STATS.items()}
    print(json.dumps(out))
    shutil.rmtree(a.work, ignore_errors=True)


if __name__ == "__main__":
    main()
