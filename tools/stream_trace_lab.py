"""Per-stage timeline of the streamed, GPU-parsed norm pass (SHIFU_STREAM_TRACE=1): for each
stage (read, h2d, parse, purify, consume, write_wait) its busy time, and for the pass how long
1, 2, 3... stages were active at once -- whether the threads overlap or take turns.

    python tools/stream_trace_lab.py [--rows 1000000] [--cols 1600]
"""
import argparse
import json
import os
import shutil
import sys
import time

os.environ["SHIFU_STREAM_TRACE"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def overlap_table(ev):
    t0 = min(e[2] for e in ev)
    pts = sorted([(e[2], 1) for e in ev] + [(e[3], -1) for e in ev])
    busy, last, k = {}, t0, 0
    for t, d in pts:
        busy[k] = busy.get(k, 0.0) + (t - last)
        k += d
        last = t
    return {str(k): round(v, 3) for k, v in sorted(busy.items())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--cols", type=int, default=1600)
    ap.add_argument("--work", default="/tmp/stream_trace_lab")
    a = ap.parse_args()
    from shifu_amd.config import environment
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.data import stream as DS
    from shifu_amd.ops import _native
    from shifu_amd.steps import api
    from shifu_amd.steps.create import create_model_set
    environment.props()["shifu.norm.dtype"] = "bf16"
    shutil.rmtree(a.work, ignore_errors=True)
    os.makedirs(a.work)
    root = create_model_set("pipe", "NN", parent=a.work)
    d = os.path.join(root, "data", "DataSet1")
    os.makedirs(d)
    if _native.rt().shifu_gen_csv(d.encode(), a.rows, a.cols, 3, 11, 0.02, 20, 16):
        raise SystemExit("generation failed")
    hdr = ["id", "diagnosis", "wgt"] + [f"num_{j}" for j in range(a.cols)] + [f"cat_{j}" for j in range(3)]
    with open(os.path.join(d, ".pig_header"), "w") as f:
        f.write("|".join(hdr) + "\n")
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    sec = mc.dataSet
    sec["dataPath"], sec["headerPath"] = d, os.path.join(d, ".pig_header")
    sec["targetColumnName"], sec["posTags"], sec["negTags"], sec["weightColumnName"] = "diagnosis", ["M"], ["B"], "wgt"
    mc.save()
    with open(os.path.join(root, "columns", "meta.column.names"), "w") as f:
        f.write("id\n")
    with open(os.path.join(root, "columns", "categorical.column.names"), "w") as f:
        f.write("cat_0\ncat_1\ncat_2\n")
    api.InitStep(root).process()
    out = {"rows": a.rows, "cols": a.cols}
    for step in ("stats", "norm"):
        DS.TRACE.clear()
        t0 = time.perf_counter()
        (api.StatsStep if step == "stats" else api.NormStep)(root).process()
        wall = time.perf_counter() - t0
        ev = list(DS.TRACE)
        if not ev:
            out[step] = {"wall_s": round(wall, 3), "note": "no traced stages (not streamed)"}
            continue
        busy = {}
        for st, _, s0, s1 in ev:
            busy[st] = busy.get(st, 0.0) + (s1 - s0)
        span = max(e[3] for e in ev) - min(e[2] for e in ev)
        out[step] = {"wall_s": round(wall, 3), "traced_span_s": round(span, 3),
                     "busy_s": {k: round(v, 3) for k, v in busy.items()},
                     "seconds_with_k_stages_active": overlap_table(ev), "events": len(ev)}
        with open(os.path.join("gpurun_out" if os.path.isdir("gpurun_out") else a.work, f"stream_trace_{step}.json"),
                  "w") as f:
            json.dump([list(e) for e in ev], f)
        print(json.dumps({step: out[step]}), flush=True)
    print(json.dumps(out))
    shutil.rmtree(a.work, ignore_errors=True)


if __name__ == "__main__":
    main()
