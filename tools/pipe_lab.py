"""Where the time of the CLI pipeline steps goes (bench.py --model pipeline data set): generates
the same synthetic text data, runs init, then each requested step under cProfile, and prints the
step's wall time plus the top functions by cumulative time.

    python tools/pipe_lab.py [--rows 500000] [--cols 1600] [--steps stats norm varsel train eval] [--top 25]
(eval runs on an eval set of --rows / 4 rows, as in the pipeline bench)
"""
import argparse
import cProfile
import io
import os
import pstats
import shutil
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=500_000)
    ap.add_argument("--cols", type=int, default=1600)
    ap.add_argument("--steps", nargs="*", default=["stats", "norm"])
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--stream", action="store_true", help="force the streamed stats / norm paths")
    ap.add_argument("--prefetch", type=int, default=None, help="shifu.data.prefetch (parsed chunks queued ahead)")
    ap.add_argument("--props", nargs="*", default=[], help="extra shifu properties k=v (e.g. shifu.data.gpuParse=false)")
    a = ap.parse_args()
    from shifu_amd.config import environment
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.ops import _native
    from shifu_amd.steps import api
    from shifu_amd.steps.create import create_model_set
    environment.props()["shifu.norm.dtype"] = "bf16"
    if a.prefetch is not None:
        environment.props()["shifu.data.prefetch"] = str(a.prefetch)
    for kv in a.props:
        k, v = kv.split("=", 1)
        environment.props()[k] = v
    if a.stream:
        environment.props()["shifu.stats.streaming"] = "true"
        environment.props()["shifu.norm.streaming"] = "true"
    work = os.path.join(tempfile.gettempdir(), "shifu_pipe_lab")
    shutil.rmtree(work, ignore_errors=True)
    os.makedirs(work)
    root = create_model_set("pipe", "NN", parent=work)
    d = os.path.join(root, "data", "DataSet1")
    os.makedirs(d)
    t0 = time.perf_counter()
    if _native.rt().shifu_gen_csv(d.encode(), a.rows, a.cols, 3, 11, 0.02, 20, 16):
        raise SystemExit("generation failed")
    e = os.path.join(root, "data", "EvalSet1")
    os.makedirs(e)
    if "eval" in a.steps and _native.rt().shifu_gen_csv(e.encode(), max(1, a.rows // 4), a.cols, 3, 12, 0.02, 20, 16):
        raise SystemExit("generation failed")
    print(f"generated {a.rows} x {a.cols} in {time.perf_counter() - t0:.1f}s", flush=True)
    for dd in (d, e):
        with open(os.path.join(dd, ".pig_header"), "w") as f:
            f.write("|".join(["id", "diagnosis", "wgt"] + [f"num_{j}" for j in range(a.cols)] +
                             [f"cat_{j}" for j in range(3)]) + "\n")
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    for sec, dd in ((mc.dataSet, d), (mc.evals[0].dataSet, e)):
        sec["dataPath"], sec["headerPath"] = dd, os.path.join(dd, ".pig_header")
        sec["targetColumnName"], sec["posTags"], sec["negTags"] = "diagnosis", ["M"], ["B"]
        sec["weightColumnName"] = "wgt"
    with open(os.path.join(root, "columns", "meta.column.names"), "w") as f:
        f.write("id\n")
    with open(os.path.join(root, "columns", "categorical.column.names"), "w") as f:
        f.write("cat_0\ncat_1\ncat_2\n")
    mc.varSelect["filterBy"] = "SE"
    mc.varSelect["filterNum"] = 200
    mc.train["numTrainEpochs"] = 10
    mc.save()
    api.InitStep(root).process()
    mc.varSelect["autoFilterEnable"] = False
    mc.train["baggingNum"] = 1
    mc.save()
    steps = {"stats": api.StatsStep, "norm": api.NormStep, "varsel": api.VarSelStep, "train": api.TrainStep,
             "eval": api.EvalStep}
    for name in a.steps:
        pr = cProfile.Profile()
        t0 = time.perf_counter()
        pr.enable()
        steps[name](root).process()
        pr.disable()
        dt = time.perf_counter() - t0
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(a.top)
        print(f"==== {name}: {dt:.2f}s", flush=True)
        print(s.getvalue(), flush=True)
    shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
