"""Prepare a GBT model set for tracing ``shifu train`` (init + stats + norm done here):

    python tools/gbt_model_set.py <dir> [--rows 1000000] [--num 60] [--trees 20] [--depth 7]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--num", type=int, default=60)
    ap.add_argument("--trees", type=int, default=20)
    ap.add_argument("--depth", type=int, default=7)
    a = ap.parse_args()
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.steps.create import run_init
    from shifu_amd.steps.norm import run_norm
    from shifu_amd.steps.stats import run_stats
    from shifu_amd.utils.synthetic import make_model_set
    root = make_model_set(a.dir, "gbt", "GBT", n_rows=a.rows, n_num=a.num, n_cat=3)
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    mc.train["params"].update({"TreeNum": a.trees, "MaxDepth": a.depth})
    mc.train["baggingNum"] = 1
    mc.save()
    run_init(root)
    run_stats(root)
    run_norm(root)
    print(root)


if __name__ == "__main__":
    main()
