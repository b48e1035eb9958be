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


def read_back(path):
    """Seconds to bring the written NormalizedData to HBM: Bf16Rows.device_rows (mmap + threaded
    copies into page-locked buffers + H2D), and plain 8-thread preads of the segment files into
    page-locked memory (no page faults) for comparison."""
    import glob
    from concurrent.futures import ThreadPoolExecutor
    import numpy as np
    import torch
    from shifu_amd.steps.base import load_dataset_cache
    res = {}
    _, arr = load_dataset_cache(path)
    t = time.perf_counter()
    x = arr["X"].device_rows(torch.device("cuda"))
    torch.cuda.synchronize()
    res["device_rows_s"] = round(time.perf_counter() - t, 3)
    res["gb"] = round(x.numel() * 2 / 1e9, 2)
    del x
    files = sorted(glob.glob(os.path.join(path, "part-*", "Xb*.npy")))
    sizes = [os.path.getsize(f) for f in files]
    buf = torch.empty(max(sizes), dtype=torch.uint8, pin_memory=True)
    bufs = [torch.empty(max(sizes), dtype=torch.uint8, pin_memory=True) for _ in range(8)]

    def rd(i):
        f, n = files[i], sizes[i]
        mv = memoryview(bufs[i % 8].numpy())[:n]
        fd = os.open(f, os.O_RDONLY)
        off = 0
        while off < n:
            off += os.preadv(fd, [mv[off:]], off)
        os.close(fd)
    t = time.perf_counter()
    with ThreadPoolExecutor(8) as ex:
        list(ex.map(rd, range(len(files))))
    res["pread8_s"] = round(time.perf_counter() - t, 3)
    res["files"] = len(files)
    del buf
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--cols", type=int, default=1600)
    ap.add_argument("--work", default="/tmp/stream_trace_lab")
    ap.add_argument("--shm-tmp", action="store_true", help="model set tmp/ (NormalizedData) on /dev/shm")
    ap.add_argument("--read-back", action="store_true",
                    help="then time reading the NormalizedData rows back to HBM (device_rows, preads)")
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
    if a.shm_tmp:
        shm = "/dev/shm/stream_trace_lab_tmp"
        shutil.rmtree(shm, ignore_errors=True)
        os.makedirs(shm)
        shutil.rmtree(os.path.join(root, "tmp"), ignore_errors=True)
        os.symlink(shm, os.path.join(root, "tmp"))
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
    if a.read_back:
        out["read_back"] = read_back(os.path.join(root, "tmp", "NormalizedData"))
        print(json.dumps({"read_back": out["read_back"]}), flush=True)
    print(json.dumps(out))
    shutil.rmtree(a.work, ignore_errors=True)
    shutil.rmtree("/dev/shm/stream_trace_lab_tmp", ignore_errors=True)


if __name__ == "__main__":
    main()
