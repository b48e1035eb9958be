#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): rows/sec (whole node) of Shifu NN training,
MLP 1000-500-200-1 binary classifier, bf16, 125M rows x 1000 cols per MI355X (256 GB of rows
resident in HBM; 8 GPUs = the metric's 1B-row x 1k-col table).

One step = one full training iteration of the reference's NN algorithm
(``J/core/dtrain/nn/AbstractNNWorker.java:521-588`` + ``NNMaster.java:207-319``): forward +
backward over every resident row of the local shard, one RCCL all-reduce of the fp32
gradient (+ error scalars), and the replicated RPROP update - nothing skipped.

Weak scaling: every rank owns ``--rows`` rows (synthetic, generated on device, random-init
weights).  ``value`` = total rows processed per second over all ranks.

    python bench.py --gpus 1 --steps 5 --warmup 2
    torchrun --nproc-per-node 8 bench.py --gpus 8 ...
    python bench.py --model gbdt    # GBDT rounds/sec (500 trees depth 7, 256 bins) config alone

The default line carries both halves of the metric: ``value`` = MLP rows/s, and after the MLP
rows are freed the same process times ``--gbdt-steps`` boosting rounds on 100M x 1000 uint8 codes
per GPU (``gbdt_rounds_per_s`` / ``gbdt_ms_per_round``; ``--gbdt-steps 0`` skips it).
    python bench.py --model varsel  # 10k-feature MLP + SE varselect config (sparse planted rule, recall@20)
    python bench.py --model lr      # LR 100k-row CSV local (CPU plumbing) config
    python bench.py --model stats   # stats (K4 exact cuts + histograms) 100M x 1000 per GPU
    python bench.py --model treeinfer   # eval scoring, 500-tree depth-7 GBT, 20M x 1000 fp64 rows
    python bench.py --model pipeline    # CLI steps on disk data, 2M x 1600 per GPU (reference: 20M x 1600)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def _launch_ranks(argv) -> int | None:
    """``--gpus N > 1`` without a torchrun environment: start N fresh worker processes (one per
    GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set, rendezvous on 127.0.0.1) and relay rank 0's JSON
    line.  This parent never imports torch or touches the GPU and never execs: it only spawns
    children and waits (the Guagua client's role, ``J/core/processor/TrainModelProcessor.java:
    720-945``).  Returns the exit code, or None when this process should run the bench itself."""
    if "WORLD_SIZE" in os.environ:
        return None
    n = 1
    for i, a in enumerate(argv):
        if a == "--gpus" and i + 1 < len(argv):
            n = int(argv[i + 1])
        elif a.startswith("--gpus="):
            n = int(a.split("=", 1)[1])
    if n <= 1:
        return None
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), *argv], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL, text=True))
    # rank 0's stdout is drained on a thread; the parent polls EVERY child, so a rank that dies
    # (e.g. at init) ends the job at once instead of leaving rank 0 in a collective until the
    # process-group timeout: the surviving ranks get SIGTERM, then SIGKILL 10 s later
    import threading
    import time as _time
    buf = []
    reader = threading.Thread(target=lambda: buf.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    rc = 0
    failed_at = None
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad and failed_at is None:
            rc = bad[0]
            failed_at = _time.monotonic()
            for p, c in zip(procs, codes):
                if c is None:
                    p.terminate()
        if all(c is not None for c in codes):
            break
        if failed_at is not None and _time.monotonic() - failed_at > 10:
            for p in procs:
                if p.poll() is None:
                    p.kill()
        _time.sleep(0.2)
    reader.join(timeout=10)
    out = buf[0] if buf else ""
    sys.stdout.write(out)
    sys.stdout.flush()
    if rc:
        print(f"[bench] a rank failed (exit {rc})", file=sys.stderr, flush=True)
    return rc


if __name__ == "__main__":
    _rc = _launch_ranks(sys.argv[1:])
    if _rc is not None:
        sys.exit(_rc)

import numpy as np  # noqa: E402
import torch  # noqa: E402

# Derived reference throughput (CHANGES.txt:268): 20M rows x 200 epochs in
# 45 min on the Hadoop cluster = 1.48M row-epochs/s whole cluster (1600 inputs).
BASELINE_MLP_ROWS_PER_S = 20e6 * 200 / 2700.0
METRIC = "rows/sec (whole node) MLP train + GBDT rounds/sec on 1B-row×1k-col tabular"


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def strong_inputs(n_in, k):
    """The ``k`` inputs of a sparse planted rule (spread over the columns, fixed for every rank)."""
    step = max(1, n_in // k)
    return list(range(0, step * k, step))[:k]


def make_synthetic(rows, n_in, k0, device, seed, sparse_k=0):
    """bf16 rows [rows, k0]: N(0,1) features, bias column = 1, zero padding; labels from a hidden
    linear rule so the task is learnable -- dense (every input) or, ``sparse_k`` > 0, only over the
    ``strong_inputs`` (alternating signs, decaying weights), which a sensitivity analysis must
    recover."""
    g = torch.Generator(device=device).manual_seed(seed)
    x = torch.empty(rows, k0, dtype=torch.bfloat16, device=device)
    y = torch.empty(rows, 1, dtype=torch.float32, device=device)
    wt = torch.randn(n_in, 1, generator=torch.Generator(device=device).manual_seed(99), device=device,
                     dtype=torch.float32)
    if sparse_k:
        wt.zero_()
        for q, j in enumerate(strong_inputs(n_in, sparse_k)):
            wt[j, 0] = (1.0 if q % 2 == 0 else -1.0) / (1.0 + 0.15 * q)
    wt = wt.to(torch.bfloat16)
    step = 1 << 22
    for r0 in range(0, rows, step):
        r1 = min(rows, r0 + step)
        blk = x[r0:r1]
        blk[:, :n_in].normal_(generator=g)
        blk[:, n_in] = 1
        blk[:, n_in + 1:] = 0
        y[r0:r1] = (blk[:, :n_in] @ wt > 0).float()
    return x, y


def bench_mlp(a, dev, info):
    from shifu_amd.models.nn import MLPSpec, MLPTrainer, TrainData
    from shifu_amd.parallel import dist
    spec = MLPSpec(n_in=a.cols, hidden=[500, 200], acts=["sigmoid", "sigmoid"], n_out=1)
    tr = MLPTrainer(spec, device=dev, propagation=a.propagation, learning_rate=0.1, seed=7,
                    chunk_rows=a.chunk_rows)
    t0 = time.time()
    if dev.type == "cuda":
        x, y = make_synthetic(a.rows, a.cols, spec.layer_kpad[0], dev, 1234 + info.rank)
    else:
        g = torch.Generator().manual_seed(1234 + info.rank)
        xr = torch.randn(a.rows, a.cols, generator=g)
        y = (xr[:, :1] > 0).float()
        x = tr.prepare(xr, y).x
    data = TrainData(x, y, None, a.rows)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    log(f"[bench] data ready: {a.rows} rows x {a.cols} cols/rank ({x.numel() * x.element_size() / 1e9:.1f} GB) "
        f"in {time.time() - t0:.1f}s")
    n_global = float(a.rows * info.world_size)
    for i in range(a.warmup):
        e = tr.step(data, num_train_global=n_global)
        log(f"[bench] warmup {i} train error {e:.6f}")

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()
    dist.barrier(); sync()
    tr.comm_events = []
    t0 = time.perf_counter()
    errs = []
    for i in range(a.steps):
        errs.append(tr.step(data, num_train_global=n_global))
    sync()
    t_local = time.perf_counter() - t0          # this rank's compute + its all-reduce waits
    dist.barrier()
    dt = time.perf_counter() - t0
    if dev.type == "cuda":
        comm_ms = sum(e0.elapsed_time(e1) for e0, e1 in tr.comm_events)
    else:
        comm_ms = sum(e1 - e0 for e0, e1 in tr.comm_events) * 1e3
    tr.comm_events = None
    log(f"[bench] train errors {['%.6f' % e for e in errs]}")
    flops_row = 2 * (a.cols * 500 + 500 * 200 + 200) * 2 + 2 * 500 * 200   # fwd+wgrad all, dgrad layer2
    return dt, errs, flops_row, {"t_local": t_local, "comm_ms": comm_ms}


def gbdt_half(a, dev, info):
    """The metric's second half ("+ GBDT rounds/sec"), timed in the same process after the MLP
    rows are freed: BASELINE config 3 (GBT depth 7, 256-bin histograms, 100M rows x 1000 cols per
    GPU, uint8 codes), ``--gbdt-steps`` boosting rounds after ``--gbdt-warmup`` untimed ones, each
    bracketed like the MLP steps (barrier + synchronize, max over ranks)."""
    import gc
    gc.collect()
    if dev.type == "cuda":
        torch.cuda.empty_cache()
        torch.cuda.reset_peak_memory_stats(dev)
    from types import SimpleNamespace
    rows = a.gbdt_rows or (100_000_000 if dev.type == "cuda" else 2_000)
    kinds = ["favourable", "balanced"] if a.gbdt_data == "both" else [a.gbdt_data]
    out = {}
    for kind in kinds:
        g = SimpleNamespace(rows=rows, cols=a.cols, steps=a.gbdt_steps, warmup=a.gbdt_warmup, levels=a.gbdt_levels,
                            labels=kind, late=a.gbdt_late)
        t0 = time.time()
        res = bench_gbdt(g, dev, info)
        log(f"[bench] gbdt ({kind}): {res['ms_per_step']:.1f} ms/round, {res['hist_rows_per_round'] / 1e6:.0f}M "
            f"rows histogrammed per round ({time.time() - t0:.1f}s incl. data generation)")
        out[kind] = res
        del res
        gc.collect()
        if dev.type == "cuda":
            torch.cuda.empty_cache()
    # the headline GBDT number is the slowest workload (balanced splits when both ran)
    head = min(out.values(), key=lambda r: r["value"])
    ret = {"gbdt_rounds_per_s": head["value"], "gbdt_ms_per_round": head["ms_per_step"],
           "gbdt_labels": head["labels"], "gbdt_hist_rows_per_round": head["hist_rows_per_round"],
           "gbdt_steps": a.gbdt_steps, "gbdt_warmup": a.gbdt_warmup, "gbdt_late_rounds": a.gbdt_late,
           "gbdt_train_error": head.get("train_error"),
           "gbdt_config": {"model": head["config"]["model"], "rows_per_gpu": rows, "n_cols": a.cols,
                           "global_rows": rows * info.world_size, "dtype": head["dtype"],
                           "parallelism": head["config"]["parallelism"]}}
    for kind, r in out.items():
        ret[f"gbdt_{kind}"] = {"rounds_per_s": r["value"], "ms_per_round": r["ms_per_step"],
                               "hist_rows_per_round": r["hist_rows_per_round"], "train_error": r.get("train_error"),
                               **({"levels": r["levels"]} if r.get("levels") else {})}
    return ret


def bench_gbdt(a, dev, info):
    from shifu_amd.models.gbdt import bench_rounds
    return bench_rounds(a, dev, info)


class _Cycle:
    """Rows [0, n) served from a host buffer of fewer rows (row r -> buffer row r mod len):
    chunk slices never straddle the wrap (chunk size divides the buffer)."""

    def __init__(self, buf, n):
        self.buf, self.n = buf, n
        self.shape = (n, buf.shape[1])

    def __len__(self):
        return self.n

    def __getitem__(self, sl):
        m = len(self.buf)
        a = sl.start % m
        return self.buf[a: a + (sl.stop - sl.start)]


SE_K = 20     # planted strong inputs of the SE bench


def bench_varsel(a, dev, info):
    """BASELINE config 5: 10k-feature MLP + sensitivity-analysis variable selection.  Each rank
    holds ``--rows`` rows x 10000 features (bf16, HBM-resident: 2M rows = 40 GB), trains the
    SE model (10000-500-1, sigmoid, RPROP full-batch epochs; ``--steps`` timed epochs) and then
    runs one SE pass over every row (HIP kernel K14: cached first layer + rank-1 correction per
    input), all-reducing the per-input sums over ranks.  value = rows through the job per second
    (epochs x rows + one SE pass x rows, all ranks)."""
    from shifu_amd.algos.varsel import sensitivity
    from shifu_amd.formats.nn_format import NNNetwork
    from shifu_amd.models.nn import HostRows, MLPSpec, MLPTrainer, TrainData
    from shifu_amd.parallel import dist
    n_in = a.cols
    spec = MLPSpec(n_in=n_in, hidden=[500], acts=["sigmoid"], n_out=1)
    tr = MLPTrainer(spec, device=dev, propagation="R", learning_rate=0.1, seed=7, chunk_rows=a.chunk_rows)
    if a.stream:
        # out-of-core: rows live in host memory and stream to HBM chunk by chunk (pinned staging,
        # H2D on a copy stream overlapping the GEMMs / SE kernels).  The 288 GB-HBM box's host cap
        # (270 GiB) cannot hold 20M x 10k bf16 (400 GB), so --rows are served from a host buffer of
        # --host-rows rows cycled: every chunk is a real H2D copy, the row values repeat.
        hb = min(a.rows, a.host_rows)
        xd, yd = make_synthetic(hb, n_in, spec.layer_kpad[0], dev, 4321 + info.rank, sparse_k=SE_K)
        xh = xd[:, :n_in].cpu()
        del xd
        torch.cuda.empty_cache()
        reps = -(-a.rows // hb)
        x = HostRows(_Cycle(xh, a.rows), n_in)
        y = yd.repeat(reps, 1)[: a.rows].contiguous()
        if a.chunk_rows > hb or hb % a.chunk_rows:
            raise SystemExit("--host-rows must be a multiple of --chunk-rows")
    else:
        x, y = make_synthetic(a.rows, n_in, spec.layer_kpad[0], dev, 4321 + info.rank, sparse_k=SE_K)
    data = TrainData(x, y, None, a.rows)
    n_global = float(a.rows * info.world_size)
    log(f"[bench] varsel data ready ({'streamed from host' if a.stream else 'HBM-resident'})")
    for i in range(a.warmup):
        tr.step(data, num_train_global=n_global)
        log(f"[bench] varsel warmup epoch {i}")

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()
    dist.barrier(); sync()
    t0 = time.perf_counter()
    for i in range(a.steps):
        tr.step(data, num_train_global=n_global)
        log(f"[bench] varsel epoch {i}")
    sync(); dist.barrier()
    t_train = time.perf_counter() - t0
    ws = tr.params.views()
    net = NNNetwork([n_in, 500, 1], ["sigmoid", "sigmoid"],
                    [ws[l][:, : spec.layer_in[l] + 1].detach().double().cpu().numpy() for l in range(len(ws))])
    dist.barrier(); sync()
    t1 = time.perf_counter()
    mean, rms, _ = sensitivity(net, x if a.stream else x[:, :n_in], device=dev,
                               row_chunk=(a.chunk_rows // 16) if a.stream else 1 << 12)
    stats = torch.tensor(np.concatenate([mean, rms ** 2]) * a.rows, dtype=torch.float64, device=dev)
    dist.all_reduce_(stats)
    sync(); dist.barrier()
    t_se = time.perf_counter() - t1
    t = torch.tensor([t_train, t_se], dtype=torch.float64, device=dev)
    dist.all_reduce_(t, "max")
    t_train, t_se = float(t[0]), float(t[1])
    rows_total = a.rows * info.world_size
    value = rows_total * (a.steps + 1) / (t_train + t_se)
    rms_all = np.sqrt(stats[n_in:].cpu().numpy() / rows_total)
    # the result must be meaningful: non-degenerate RMS and the planted inputs ranked on top
    strong = set(strong_inputs(n_in, SE_K))
    top = np.argsort(-rms_all, kind="stable")[:SE_K]
    recall = len(strong & set(int(i) for i in top)) / SE_K
    distinct = int(np.unique(np.round(rms_all, 12)).size)
    if distinct < n_in // 2 or not np.isfinite(rms_all).all() or float(rms_all.max()) <= 0.0:
        raise SystemExit(f"degenerate SE result: {distinct} distinct RMS values over {n_in} inputs")
    return {
        "metric": METRIC + " [config: 10k-feature MLP + SE varselect]",
        "value": value, "unit": "rows/s", "n_gpus": info.world_size, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": (t_train + t_se) / (a.steps + 1) * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "bf16", "data": "synthetic (N(0,1) features, hidden linear rule), random-init weights",
        "config": {"model": f"MLP {n_in}-500-1 + SE sensitivity varselect", "global_batch": rows_total,
                   "seq_len": None, "n_cols": n_in, "rows_per_gpu": a.rows, "parallelism": f"dp{info.world_size}",
                   "streamed_from_host": bool(a.stream),
                   "host_buffer_rows": min(a.rows, a.host_rows) if a.stream else None},
        "train_ms_per_epoch": t_train / max(1, a.steps) * 1e3, "se_pass_ms": t_se * 1e3,
        "se_input_pairs_per_s": rows_total * n_in / t_se, "top5_inputs_by_rms": np.argsort(-rms_all)[:5].tolist(),
        "planted_rule": f"sparse, {SE_K} of {n_in} inputs", "recall_at_k": recall, "distinct_rms_values": distinct,
    }


def _stats_batch(C, n, k0, dev, seed):
    """Synthetic column batch [C, n] fp64 on the device: a mix of N(0,1) with ~2% missing,
    log-normal heavy tails, low-cardinality integers and 2-decimal values (many ties)."""
    g = torch.Generator(device=dev).manual_seed(seed)
    v = torch.empty(C, n, dtype=torch.float64, device=dev)
    v.normal_(generator=g)
    for k in range(C):
        t = (k0 + k) % 4
        col = v[k]
        if t == 0:
            col.masked_fill_(col > 2.0, float("nan"))
        elif t == 1:
            col.mul_(2.0).exp_()
        elif t == 2:
            col.mul_(3.0).floor_()
        else:
            col.mul_(100.0).round_().div_(100.0)
    return v


def bench_stats(a, dev, info):
    """``shifu stats`` over 100M rows x 1000 numeric columns per GPU (the reference's headline stats
    job is 100M x 1600 in 30 min on a Hadoop cluster, CHANGES.txt:233-234).  One step = the full
    per-column pass for every column: K4 exact equal-population cuts (qprep/qhist/qgather, 10 bins,
    EqualPositive over a binary target), K1+K2 bin histograms + moments with those cuts, distinct
    counts, and - for N > 1 - the all-reduces that merge the per-rank partials.  Columns are
    processed in HBM-resident batches of 64 (51 GB of fp64 at 100M rows), two batches in flight on
    one GPU (as `shifu stats` runs them); the batches are generated on the device before their
    timed section (generation time is reported, not counted).
    value = rows x (all columns) per second over all ranks, i.e. full-table stats passes x rows."""
    from shifu_amd.algos import quantile as Q
    from shifu_amd.algos.stats import batch_histograms, run_lanes
    from shifu_amd.parallel import dist
    n, F, C = a.rows, a.cols, 64
    g = torch.Generator(device=dev).manual_seed(99 + info.rank)
    y = (torch.rand(n, generator=g, device=dev) < 0.3).float()
    w = torch.ones(n, dtype=torch.float64, device=dev)
    multi = info.world_size > 1
    red = (lambda t, op: dist.all_reduce_(t, op)) if multi else None
    cat = dist.all_gather_cat if multi else None

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    # column batches in flight together (algos/stats.run_lanes: one HIP stream + host thread per
    # batch, so one batch's host planning overlaps the other's kernels), as `shifu stats` runs them
    lanes = 1 if multi else int(os.environ.get("SHIFU_STATS_LANES", "2"))

    def stats_of(v):
        bounds, _ = Q.column_cuts(v, y, w, 10, "EqualPositive", True, reduce=red, allgather=cat)
        return bounds, batch_histograms(v, y, w, bounds, True)

    def one_pass(step):
        t_stats = t_gen = 0.0
        nb_total = 0
        starts = list(range(0, F, C))
        for g0 in range(0, len(starts), lanes):
            group = starts[g0: g0 + lanes]
            t0 = time.perf_counter()
            vs = [_stats_batch(min(C, F - b0), n, b0, dev, 1000 * step + b0 + 7 * info.rank) for b0 in group]
            sync()
            dist.barrier()
            t1 = time.perf_counter()
            outs = run_lanes(stats_of, vs, dev, lanes)
            for bounds, res in outs:
                if multi:
                    h = np.concatenate([np.concatenate([r[0], r[1], r[2], r[3]]) for r in res])
                    dist.all_reduce_np(h)
                nb_total += sum(len(b) + 1 for b in bounds)
            sync()
            dist.barrier()
            t_stats += time.perf_counter() - t1
            t_gen += t1 - t0
            del vs
        return t_stats, t_gen, nb_total

    for i in range(a.warmup):
        ts, tg, nb = one_pass(i)
        log(f"[bench] stats warmup {i}: {ts:.2f}s stats, {tg:.2f}s generation, {nb} bins")
    times, gens = [], []
    for i in range(a.steps):
        ts, tg, nb = one_pass(100 + i)
        times.append(ts)
        gens.append(tg)
        log(f"[bench] stats step {i}: {ts:.3f}s stats, {tg:.2f}s generation")
    t = torch.tensor([sum(times)], dtype=torch.float64, device=dev)
    dist.all_reduce_(t, "max")
    dt = float(t.item())
    total_rows = n * info.world_size
    value = total_rows * a.steps / dt
    return {
        "metric": "rows/sec (whole node) shifu stats: exact 10-bin equal-population cuts + bin histograms + "
                  "moments + distinct counts over every column [config: 100M rows x 1000 numeric cols per GPU]",
        "value": value, "unit": "rows/s", "n_gpus": info.world_size, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": dt / a.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "fp64", "data": "synthetic, generated on the device per 64-column batch (not timed)",
        "config": {"model": "stats (EqualPositive, maxNumBin 10, binary target)", "global_batch": total_rows,
                   "seq_len": None, "n_cols": F, "rows_per_gpu": n, "parallelism": f"dp{info.world_size}"},
        "column_rows_per_s": value * F, "generation_s_per_step": sum(gens) / len(gens),
        "reference_note": "reference: 100M x 1600 stats in 30 min on a Hadoop cluster (CHANGES.txt:233-234) "
                          "= 5.6e4 rows/s",
    }


def bench_treeinfer(a, dev, info):
    """K13: eval-time scoring of a 500-tree depth-7 GBT (IndependentTreeModel.computeRegressionScore,
    J/core/dtrain/dt/IndependentTreeModel.java:387-441) over rows x 1000 raw fp64 columns resident
    in HBM (feature-major).  One step = every row scored by every tree (random-init trees with
    random raw-value thresholds; synthetic N(0,1) inputs)."""
    from shifu_amd.formats.tree_format import CONTINUOUS, Node, Split, TreeModelFile, TreeRecord
    from shifu_amd.scoring.tree_ensemble import FlatEnsemble
    rng = np.random.default_rng(7)
    n_trees, depth, C = 500, 7, a.cols

    def grow(d):
        nd = Node(0)
        if d == depth:
            nd.predict = float(rng.normal())
            return nd
        nd.split = Split(int(rng.integers(0, C)), CONTINUOUS, threshold=float(rng.normal() * 0.5))
        nd.left, nd.right = grow(d + 1), grow(d + 1)
        return nd
    cols = list(range(C))
    m = TreeModelFile("GBT", "squared", False, False, C, {c: 0.0 for c in cols}, {c: f"c{c}" for c in cols}, {},
                      {c: c for c in cols}, [[TreeRecord(t, 0, grow(0), 0.1) for t in range(n_trees)]])
    ens = FlatEnsemble(m, 0, cols, dev)
    XT = torch.empty(C, a.rows, dtype=torch.float64, device=dev)
    g = torch.Generator(device=dev).manual_seed(1)
    for c0 in range(0, C, 64):
        XT[c0:c0 + 64].normal_(generator=g)
    X = XT.t()                                  # [N, C] view of the feature-major matrix (no copy)
    from shifu_amd.parallel import dist
    for _ in range(a.warmup):
        ens.score(X)
    torch.cuda.synchronize(dev) if dev.type == "cuda" else None
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        s = ens.score(X)
    torch.cuda.synchronize(dev) if dev.type == "cuda" else None
    dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    dist.all_reduce_(t, "max")                  # every rank scores its own --rows (eval is row-sharded)
    ms = float(t.item()) / a.steps * 1e3
    total = a.rows * info.world_size
    return {
        "metric": "GBT scoring rows/s (500 trees depth 7, 1000 raw fp64 columns)", "value": total / (ms / 1e3),
        "unit": "rows/s", "n_gpus": info.world_size, "steps": a.steps, "warmup": a.warmup, "ms_per_step": ms,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp64",
        "data": "synthetic N(0,1) inputs, random-init trees",
        "config": {"model": "GBT 500 trees depth 7", "global_batch": total, "seq_len": None, "n_cols": C,
                   "rows_per_gpu": a.rows, "parallelism": f"dp{info.world_size}"},
        "node_visits_per_s": total * n_trees * depth / (ms / 1e3), "score_checksum": float(s.sum()),
    }


def bench_corr(a, dev, info):
    """K15: ``shifu stats -correlation`` sums (pairwise-complete Pearson, FastCorrelationMapper
    J/core/correlation/FastCorrelationMapper.java:171-278) over rows x cols fp64 values per GPU
    with 2% missing cells.  One step = every row through CorrAccumulator.update (int8 digit-plane
    GEMMs, method i8) + finalize (fold, reduce-scatter of the six sums, correlation rows, gather).
    Rows are drawn from a pool of device-resident 64K-row chunks (generated before the timed
    section) that is cycled through -- the pass is compute bound, so reuse does not flatter it.
    Also reported: the fp64 torch-addmm path (hipBLASLt fp64 GEMMs) over one pool pass, and the
    max |corr_i8 - corr_fp64| over the pool (same shift)."""
    from shifu_amd.algos.stats import CORR_CHUNK, CorrAccumulator
    from shifu_amd.parallel import dist
    n, F = a.rows, a.cols
    CH = CORR_CHUNK if dev.type == "cuda" else 1024
    npool = max(1, min(16, int(16e9 // (CH * F * 8)), -(-n // CH)))
    g = torch.Generator(device=dev).manual_seed(5 + info.rank)
    pool = []
    for k in range(npool):
        z = torch.randn(CH, F + 1, generator=g, device=dev, dtype=torch.float64)
        x = z[:, 1:] + 0.6 * z[:, :-1]                         # neighbouring columns correlated
        x[:, ::7] += 1000.0                                    # large-mean columns (shifted away)
        x[torch.rand(CH, F, generator=g, device=dev) < 0.02] = float("nan")
        pool.append(x.contiguous())
        del z
    shift = torch.zeros(F, dtype=torch.float64)
    shift[::7] = 1000.0

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    def one_pass(method, rows):
        acc = CorrAccumulator(F, dev, shift=shift.numpy(), method=method)
        k = 0
        for r0 in range(0, rows, CH):
            x = pool[k % npool]
            acc.update(x[: min(CH, rows - r0)])
            k += 1
        return acc.finalize(0)

    for _ in range(a.warmup):
        one_pass("i8" if dev.type == "cuda" else "fp64", n)
    sync()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        C = one_pass("i8" if dev.type == "cuda" else "fp64", n)
    sync()
    dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    dist.all_reduce_(t, "max")
    dt = float(t.item())
    total = n * info.world_size
    value = total * a.steps / dt
    out = {
        "metric": "correlation rows/s (whole node): pairwise-complete Pearson sums + finalize over every column pair",
        "value": value, "unit": "rows/s", "n_gpus": info.world_size, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": dt / a.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "fp64 values; exact int8 digit GEMMs (S=6 x 7-bit digits)" if dev.type == "cuda" else "fp64",
        "data": f"synthetic N(0,1) with neighbour correlation, 2% missing, every 7th column mean 1000; "
                f"{npool} device-resident 64K-row chunks cycled",
        "config": {"model": "stats -correlation", "global_batch": total, "seq_len": None, "n_cols": F,
                   "rows_per_gpu": n, "parallelism": f"dp{info.world_size}"},
        "column_pair_updates_per_s": value * F * F,
    }
    if dev.type == "cuda":
        # the previous path (four fp64 addmm per chunk) over one pool pass, and the agreement
        rows_ref = npool * CH
        sync()
        t1 = time.perf_counter()
        Cref = one_pass("fp64", rows_ref)
        sync()
        t_ref = time.perf_counter() - t1
        Ci8 = one_pass("i8", rows_ref)
        if info.rank == 0:
            out["fp64_addmm_rows_per_s"] = rows_ref * info.world_size / t_ref
            out["speedup_vs_fp64_addmm"] = value / out["fp64_addmm_rows_per_s"]
            out["max_abs_diff_vs_fp64"] = float(np.nanmax(np.abs(Ci8 - Cref)))
            out["corr_checksum"] = float(np.nansum(C))
    return out


def bench_eval(a, dev, info):
    """K16 ``shifu eval`` performance pass (EvalModelProcessor -> ConfusionMatrix
    .bufferedComputeConfusionMatrixAndPerformance, J/core/ConfusionMatrix.java:276-507) over
    rows scored (score, tag, weight) records per GPU: stable descending radix sort on the device
    (ops/csrc/sort_kernels.hip), cumulative confusion sweep, ROC / PR / gains bucket searches and
    the score buckets -- the EvalPerformance.json of that eval set.  Each rank evaluates its own
    eval set (N GPUs = N eval sets in parallel).  Reported also: the sort alone."""
    from shifu_amd.algos import evaluation as E
    from shifu_amd.parallel import dist
    n = a.rows
    g = torch.Generator(device=dev).manual_seed(11 + info.rank)
    z = torch.randn(n, generator=g, device=dev, dtype=torch.float64)
    y = (torch.rand(n, generator=g, device=dev, dtype=torch.float64) < torch.sigmoid(1.5 * z - 1.0)).double()
    score = torch.round(1000.0 * torch.sigmoid(z + 0.3 * torch.randn(n, generator=g, device=dev,
                                                                      dtype=torch.float64)))   # integer scores: ties
    w = 0.5 + torch.rand(n, generator=g, device=dev, dtype=torch.float64)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    res = None
    for _ in range(a.warmup):
        res = E.performance(score, y, w, 10, max_score=1000.0, device=dev)
    sync()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        res = E.performance(score, y, w, 10, max_score=1000.0, device=dev)
    sync()
    dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    dist.all_reduce_(t, "max")
    dt = float(t.item())
    total = n * info.world_size
    out = {
        "metric": "eval performance rows/s (whole node): sort + confusion sweep + ROC/PR/gains/score buckets",
        "value": total * a.steps / dt, "unit": "rows/s", "n_gpus": info.world_size, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": dt / a.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "fp64",
        "data": "synthetic scored records (integer scores 0..1000 -> heavy ties, logistic tags, U(0.5,1.5) weights)",
        "config": {"model": "eval performance (10 buckets)", "global_batch": total, "seq_len": None,
                   "rows_per_gpu": n, "parallelism": f"dp{info.world_size} (one eval set per rank)"},
        "auc": res["areaUnderRoc"] if res else None,
    }
    if dev.type == "cuda":
        sync()
        t1 = time.perf_counter()
        for _ in range(3):
            E.order_desc(score)
        sync()
        out["sort_rows_per_s"] = 3 * n / (time.perf_counter() - t1)
        t1 = time.perf_counter()
        torch.argsort(-score, stable=True)
        sync()
        out["torch_stable_argsort_rows_per_s"] = n / (time.perf_counter() - t1)
        # NN scoring (the eval's model pass) of the headline 1000-500-200-1 net: fp32 (default,
        # parity: split-bf16 on the own MFMA GEMM), the vendor fp32 GEMM, and bf16 on the
        # trainer's own MFMA kernels
        from shifu_amd.formats.nn_format import NNNetwork
        from shifu_amd.scoring.model_runner import nn_forward
        rng = np.random.default_rng(0)
        sizes = [1000, 500, 200, 1]
        net = NNNetwork(sizes, ["sigmoid", "sigmoid", "sigmoid"],
                        [rng.normal(size=(sizes[i + 1], sizes[i] + 1)) * 0.05 for i in range(3)])
        ns = min(n, 4_000_000)
        X = torch.randn(ns, 1000, generator=g, device=dev, dtype=torch.float32)
        a64 = X[:16384].double().cpu().numpy()
        for W in net.weights:                                   # fp64 oracle of the first rows
            a64 = 1.0 / (1.0 + np.exp(-(a64 @ W[:, :-1].T + W[:, -1])))
        ref64 = a64
        for prec in ("fp32", "fp32_torch", "bf16"):
            nn_forward(net, X[:65536], dev, precision=prec)
            sync()
            t1 = time.perf_counter()
            sc = nn_forward(net, X, dev, precision=prec)
            sync()
            out[f"nn_scoring_rows_per_s_{prec}"] = ns / (time.perf_counter() - t1)
            out[f"nn_scoring_checksum_{prec}"] = float(sc.sum())
            out[f"nn_scoring_maxabs_vs_fp64_{prec}"] = float(np.abs(sc[:16384] - ref64).max())
    return out


REF_PIPELINE_MIN = {"stats": 20.0, "eval": 13.0, "varsel_train_200ep": 45.0, "varsel_se": 25.0}
REF_PIPELINE_ROWS = 20_000_000


def bench_pipeline(a, dev, info):
    """The reference's only published numbers are CLI step wall times on 20M rows x 1600 variables
    (CHANGES.txt:233-237, 264-268): stats 20 min, eval 13 min, varsel SE 70 min = 45 min of
    200-epoch NN training + 25 min of sensitivity.  This runs the same CLI steps (Step API, the
    code `shifu <verb>` runs) on a generated '|'-delimited data set on disk (native generator,
    runtime/csrc/gen_csv.cpp, planted sparse rule on 20 of the columns) and times each step:
    init, stats, norm, varsel (filterBy SE: trains numTrainEpochs/2 epochs then the SE pass),
    train (numTrainEpochs = --pipeline-epochs of the default NN) and eval (an eval set a quarter of
    the training set).  The whole pipeline is one step.  Epoch counts below 200 are timed and the 200-epoch figure is projected
    linearly from the per-epoch time (labelled); the 20M-row projection scales each
    data-proportional step linearly (labelled).  value = rows/s of the whole pipeline."""
    import ctypes
    import shutil
    import tempfile
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.ops import _native
    from shifu_amd.parallel import dist
    from shifu_amd.steps import api
    from shifu_amd.steps.create import create_model_set
    rows, F = a.rows, a.cols
    # disk: the eval set is a quarter of the training set unless --pipeline-eval-rows says otherwise
    rows_eval = a.pipeline_eval_rows or max(1000, rows // 4)
    epochs = max(2, a.pipeline_epochs)
    from shifu_amd.config import environment
    environment.props()["shifu.norm.dtype"] = "bf16"     # GEMM-ready NormalizedData (half the bytes)
    work = a.workdir or os.path.join(tempfile.gettempdir(), "shifu_pipeline_bench")
    root = os.path.join(work, "pipe")
    t_gen = 0.0
    if info.rank == 0:
        shutil.rmtree(work, ignore_errors=True)
        os.makedirs(work)
        root = create_model_set("pipe", "NN", parent=work)
        lib = _native.rt()
        t0 = time.perf_counter()
        rep = max(1, a.pipeline_replicate)
        for name, seed, nr in (("DataSet1", 11, rows), ("EvalSet1", 12, rows_eval)):
            d = os.path.join(root, "data", name)
            os.makedirs(d, exist_ok=True)
            # --pipeline-replicate R: one generated part of rows/R rows, listed R times (symlinks):
            # the reference's 20M x 1600 text (268 GB) does not fit the box's disk
            g = d if rep == 1 else os.path.join(work, "gen_" + name)
            os.makedirs(g, exist_ok=True)
            rc = lib.shifu_gen_csv(g.encode(), -(-nr // rep), F, 3, seed, 0.02, 20, min(16, os.cpu_count() or 4))
            if rc:
                raise RuntimeError("data generation failed (disk full?)")
            if rep > 1:
                parts = sorted(f for f in os.listdir(g) if not f.startswith((".", "_")))
                for r_ in range(rep):
                    for f in parts:
                        os.symlink(os.path.join(g, f), os.path.join(d, f"r{r_:02d}-{f}"))
            hdr = ["id", "diagnosis", "wgt"] + [f"num_{j}" for j in range(F)] + [f"cat_{j}" for j in range(3)]
            with open(os.path.join(d, ".pig_header"), "w") as f:
                f.write("|".join(hdr) + "\n")
        t_gen = time.perf_counter() - t0
        mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
        for sec, key in ((mc.dataSet, "DataSet1"), (mc.evals[0].dataSet, "EvalSet1")):
            d = os.path.join(root, "data", key)
            sec["dataPath"], sec["headerPath"] = d, os.path.join(d, ".pig_header")
            sec["targetColumnName"], sec["posTags"], sec["negTags"] = "diagnosis", ["M"], ["B"]
            sec["weightColumnName"] = "wgt"
        with open(os.path.join(root, "columns", "meta.column.names"), "w") as f:
            f.write("id\n")
        with open(os.path.join(root, "columns", "categorical.column.names"), "w") as f:
            f.write("cat_0\ncat_1\ncat_2\n")
        mc.varSelect["filterBy"] = "SE"
        mc.varSelect["filterNum"] = 200
        mc.varSelect["autoFilterEnable"] = False
        mc.train["numTrainEpochs"] = epochs
        mc.train["baggingNum"] = 1
        mc.train["validSetRate"] = 0.1
        mc.save()
        if a.pipeline_tmp:                   # NormalizedData etc. on another filesystem (e.g. /dev/shm)
            tdir = os.path.join(a.pipeline_tmp, "shifu_pipe_tmp")
            shutil.rmtree(tdir, ignore_errors=True)
            os.makedirs(tdir)
            shutil.rmtree(os.path.join(root, "tmp"), ignore_errors=True)
            os.symlink(tdir, os.path.join(root, "tmp"))
        gb = sum(os.path.getsize(os.path.join(root, "data", "DataSet1", f))
                 for f in os.listdir(os.path.join(root, "data", "DataSet1")))
        log(f"[bench] pipeline data: {rows} rows x {F} numeric + 3 categorical, {gb / 1e9:.1f} GB text, "
            f"generated in {t_gen:.1f}s -> {root}")
    root = dist.all_gather_objects(root)[0]
    times = {}

    def step(name, fn):
        dist.barrier()
        if dev.type == "cuda":
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        if dev.type == "cuda":
            torch.cuda.synchronize()
        dist.barrier()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        dist.all_reduce_(t, "max")
        times[name] = float(t.item())
        log(f"[bench] pipeline {name}: {times[name]:.1f}s")
    step("init", lambda: api.InitStep(root).process())
    step("stats", lambda: api.StatsStep(root).process())
    step("norm", lambda: api.NormStep(root).process())
    step("varsel", lambda: api.VarSelStep(root).process())
    from shifu_amd.steps.varsel import PHASES as SE_PHASES
    step("train", lambda: api.TrainStep(root).process())
    step("eval", lambda: api.EvalStep(root).process())
    # --pipeline-extra: steps timed after the pipeline, outside its total (scale checks of the
    # data-parallel init -autotype scan and the combo score join, data/join.py)
    extra = {}
    for x in [e.strip() for e in (a.pipeline_extra or "").split(",") if e.strip()]:
        if x == "autotype":
            def _scan():
                from shifu_amd.algos import autotype
                from shifu_amd.config.model_config import ModelConfig
                from shifu_amd.data.reader import read_header
                mc_ = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
                hp = mc_.resolve(mc_.dataSet["headerPath"])
                hdr_ = read_header(hp, "|", mc_.resolve(mc_.dataSet["dataPath"]), "|")
                autotype.scan(mc_, hdr_, list(range(len(hdr_))), info.rank, info.world_size)
            step("x_autotype_scan", _scan)
        elif x == "join":
            def _join():
                from shifu_amd.steps.base import ModelSet
                from shifu_amd.steps.combo import _join_scores
                ms_ = ModelSet(root)
                _join_scores([("nn", ms_)], [ms_.mc.dataSet], os.path.join(root, "joined"))
            step("x_combo_join", _join)
        elif x == "encode":
            # a small GBT on the same data (setup, untimed), then the streamed leaf-path encode
            from shifu_amd.config.model_config import ModelConfig
            mc_ = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
            mc_.train["algorithm"] = "GBT"
            mc_.train["params"] = {"TreeNum": 10, "MaxDepth": 5, "LearningRate": 0.1, "Loss": "squared",
                                   "Impurity": "variance", "FeatureSubsetStrategy": "ALL", "MinInstancesPerNode": 5}
            mc_.save()
            step("x_encode_setup_norm", lambda: api.NormStep(root).process())
            step("x_encode_setup_train", lambda: api.TrainStep(root).process())

            def _enc():
                from shifu_amd.steps.misc import run_encode
                run_encode(root)
            step("x_encode", _enc)
            times.pop("x_encode_setup_norm")
            times.pop("x_encode_setup_train")
        else:
            raise ValueError(f"unknown --pipeline-extra step {x}")
        extra[x] = times.pop({"autotype": "x_autotype_scan", "join": "x_combo_join", "encode": "x_encode"}[x])
    recall = None
    if info.rank == 0:
        import numpy as np
        from shifu_amd.config.column_config import load_column_configs
        strong = np.zeros(20, np.int32)
        k = _native.rt().shifu_gen_strong_cols(F, 20, strong.ctypes.data)
        want = {f"num_{j}" for j in strong[:k]}
        se = [l.split("\t") for l in open(os.path.join(root, "varsel", "se.0")).read().strip().split("\n")]
        top = [r[1] for r in se[:k]]
        recall = len(want & set(top)) / max(1, k)
        perf = json.load(open(os.path.join(root, "evals", "Eval1", "EvalPerformance.json")))
    total = sum(times.values())
    scale20 = REF_PIPELINE_ROWS / float(rows * info.world_size)
    proj = {k: v * (REF_PIPELINE_ROWS / float(rows_eval * info.world_size) if k == "eval" else scale20) / 60.0
            for k, v in times.items()}
    # per-epoch time from the trainer's own metrics stream (one ts per epoch); the rest of the
    # train step is setup (NormalizedData load + H2D, model write)
    ep_train = times["train"] / epochs
    if info.rank == 0:
        try:
            ts = [json.loads(l)["ts"] for l in open(os.path.join(root, "tmp", "metrics.jsonl"))
                  if json.loads(l).get("trainer") == 0]
            ts = ts[-epochs:]
            if len(ts) >= 3:
                d = sorted(b - a_ for a_, b in zip(ts, ts[1:]))
                ep_train = d[len(d) // 2]
        except (OSError, ValueError, KeyError):
            pass
    train_setup = max(0.0, times["train"] - epochs * ep_train)
    out = {
        "metric": "rows/sec (whole pipeline init+stats+norm+varsel(SE)+train+eval, CLI steps on disk data)",
        "value": rows * info.world_size / total, "unit": "rows/s", "n_gpus": info.world_size, "steps": 1,
        "train_epochs": epochs,
        "warmup": 0, "ms_per_step": total * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "bf16 NN GEMMs / fp64 stats", "data": f"synthetic '|'-delimited text on disk, {rows} training + "
        f"{rows_eval} eval rows x {F} numeric + 3 categorical per GPU, planted rule on 20 columns (native generator)"
        + (f"; each set is one generated part listed {a.pipeline_replicate} times (symlinks: the box's disk cannot "
           f"hold the full-size text)" if a.pipeline_replicate > 1 else ""),
        "config": {"model": f"default NN {F}-50-1 (tanh), SE varsel filterNum 200", "global_batch": rows * info.world_size,
                   "seq_len": None, "n_cols": F, "rows_per_gpu": rows, "parallelism": f"dp{info.world_size}"},
        "step_seconds": {k: round(v, 2) for k, v in times.items()}, "generation_s": round(t_gen, 1),
        "extra_step_seconds (outside the total)": {k: round(v, 2) for k, v in extra.items()},
        "train_epoch_s (median epoch interval, metrics.jsonl)": round(ep_train, 4),
        "train_setup_s": round(train_setup, 2),
        "varsel_phases_s (SE: rows load, NN training, sensitivity)": {k: (round(v, 2) if isinstance(v, float) else v)
                                                                      for k, v in SE_PHASES.items()},
        "step_minutes": {k: round(v / 60.0, 2) for k, v in times.items()},
        "reference_minutes_20M_x_1600 (CHANGES.txt:233-237,264-268)": REF_PIPELINE_MIN,
        # a replicated input (one generated part listed R times, read from the page cache) is not
        # the reference's 268 GB of distinct text: never labelled as measured at its shape
        "measured_at_reference_shape": bool(rows * info.world_size >= REF_PIPELINE_ROWS and F >= 1600 and epochs >= 400
                                            and rows_eval * info.world_size >= REF_PIPELINE_ROWS
                                            and a.pipeline_replicate <= 1),
        "replicated_input": a.pipeline_replicate > 1,
        "reference_shape_rows_and_cols": bool(rows * info.world_size >= REF_PIPELINE_ROWS and F >= 1600),
        "se_recall_of_planted_columns": recall,
        "eval_auc": perf["areaUnderRoc"] if info.rank == 0 else None,
    }
    if not out["measured_at_reference_shape"]:        # smaller runs: labelled linear projections
        out["projected_20M_rows_minutes (linear in rows, labelled projection)"] = {k: round(v, 2)
                                                                                  for k, v in proj.items()}
        out["projected_20M_train_200_epochs_minutes ((setup + 200 x epoch) x rows, labelled projection)"] = \
            round((train_setup + ep_train * 200) * scale20 / 60.0, 2)
    if info.rank == 0 and not a.keep:
        shutil.rmtree(work, ignore_errors=True)
        if a.pipeline_tmp:
            shutil.rmtree(os.path.join(a.pipeline_tmp, "shifu_pipe_tmp"), ignore_errors=True)
    return out


def bench_lr(a, dev, info):
    """BASELINE config 1: logistic regression on a 100k-row CSV, local mode, CPU only (the
    plumbing path): shifu init -> stats -> norm -> train on a generated model set.  One step =
    one full pipeline run; value = pipeline runs per minute is not meaningful, so the line reports
    the pipeline wall time (lower is better) and the LR training rows/s."""
    import tempfile
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.steps import api
    from shifu_amd.utils.synthetic import make_model_set
    os.environ["SHIFU_FORCE_CPU"] = "1"
    times, train_t = [], []
    with tempfile.TemporaryDirectory(prefix="shifu_lr_bench_") as tmp:
        root = make_model_set(tmp, "lrbench", "LR", n_rows=a.rows, n_num=20, n_cat=3)
        mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
        mc.train["numTrainEpochs"] = 100
        mc.train["baggingNum"] = 1
        mc.save()
        for i in range(a.warmup + a.steps):
            t0 = time.perf_counter()
            for cls in (api.InitStep, api.StatsStep, api.NormStep):
                cls(root).process()
            t1 = time.perf_counter()
            api.TrainStep(root).process()
            t2 = time.perf_counter()
            if i >= a.warmup:
                times.append(t2 - t0)
                train_t.append(t2 - t1)
    ms = sum(times) / len(times) * 1e3
    return {
        "metric": "LR local pipeline wall time (init+stats+norm+train, 100 epochs) [config: LR 100k-row CSV, CPU]",
        "value": ms / 1e3, "unit": "s", "n_gpus": 0, "steps": a.steps, "warmup": a.warmup, "ms_per_step": ms,
        "higher_is_better": False, "scaling": "strong", "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic CSV (20 numeric + 3 categorical columns)",
        "config": {"model": "LR", "global_batch": a.rows, "seq_len": None, "parallelism": "local"},
        "train_rows_epochs_per_s": a.rows * 100 / (sum(train_t) / len(train_t)),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default="mlp", choices=["mlp", "gbdt", "varsel", "lr", "stats", "treeinfer", "pipeline", "corr", "eval"])
    ap.add_argument("--rows", type=int, default=None,
                    help="rows per GPU (default 125M on GPU: 256 GB of bf16 rows resident in one MI355X's "
                         "288 GB HBM, so 8 GPUs hold the metric's 1B-row x 1k-col table)")
    ap.add_argument("--cols", type=int, default=1000)
    ap.add_argument("--chunk-rows", type=int, default=1 << 21)   # 2M-row chunks: +1.6% vs 1M (profiles/r1d)
    ap.add_argument("--propagation", default="R")
    ap.add_argument("--gbdt-rows", type=int, default=None,
                    help="rows per GPU of the GBDT half of the default line (default 100M on GPU)")
    ap.add_argument("--gbdt-steps", type=int, default=5, help="timed boosting rounds (0 = MLP only)")
    ap.add_argument("--gbdt-warmup", type=int, default=1)
    ap.add_argument("--gbdt-data", default="both", choices=["both", "favourable", "balanced"],
                    help="GBDT labels: favourable (rule on two features: small non-root nodes), balanced (dense "
                         "linear rule at its median: ~N/2 rows per smaller child), both (headline = the slower)")
    ap.add_argument("--gbdt-late", type=int, default=0,
                    help="GBDT: untimed rounds before the timed window (time a later part of the ensemble)")
    ap.add_argument("--gbdt-levels", action="store_true",
                    help="GBDT: per-level histogram table (rows, bytes, ms, TB/s; HIP events around each level)")
    ap.add_argument("--stream", action="store_true", help="varsel: rows streamed from host memory (HostRows)")
    ap.add_argument("--host-rows", type=int, default=2_000_000, help="varsel --stream: host buffer rows")
    ap.add_argument("--workdir", default=None, help="pipeline: where the generated model set lives")
    ap.add_argument("--keep", action="store_true", help="pipeline: keep the generated model set")
    ap.add_argument("--pipeline-replicate", type=int, default=1,
                    help="pipeline: generate rows/R rows and list the part R times (disk-limited boxes)")
    ap.add_argument("--pipeline-tmp", default=None, help="pipeline: put the model set's tmp/ (NormalizedData) here")
    ap.add_argument("--pipeline-eval-rows", type=int, default=None,
                    help="pipeline: eval set rows (default a quarter of --rows; the reference's eval is 20M rows)")
    ap.add_argument("--pipeline-extra", default="",
                    help="pipeline: extra timed steps after it, comma list of autotype, join, encode")
    ap.add_argument("--pipeline-epochs", type=int, default=40,
                    help="pipeline: numTrainEpochs of the NN (varsel SE trains half of them)")
    a = ap.parse_args()

    from shifu_amd.parallel import dist
    info = dist.init_from_env()
    if os.environ.get("SHIFU_BENCH_FAIL_RANK") == str(info.rank):     # launcher fault-injection test
        log(f"[bench] rank {info.rank}: injected failure")
        sys.exit(3)
    if info.world_size != a.gpus and "WORLD_SIZE" in os.environ:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={info.world_size}")
    gpu = torch.cuda.is_available()
    dev = torch.device("cuda", torch.cuda.current_device()) if gpu else torch.device("cpu")
    if a.model == "varsel" and a.cols == 1000:
        a.cols = 10_000
    if a.model == "pipeline" and a.cols == 1000:
        a.cols = 1600 if gpu else 40
    if a.model == "corr" and a.cols == 1000:
        a.cols = 1600 if gpu else 40
    if a.rows is None:
        a.rows = {"varsel": 2_000_000 if gpu else 2_000, "lr": 100_000, "stats": 100_000_000 if gpu else 5_000,
                  "treeinfer": 20_000_000 if gpu else 5_000, "pipeline": 2_000_000 if gpu else 4_000,
                  "corr": 20_000_000 if gpu else 5_000, "eval": 100_000_000 if gpu else 20_000,
                  "gbdt": 100_000_000 if gpu else 20_000}.get(a.model, 125_000_000 if gpu else 20_000)
    if a.model == "gbdt":
        a.levels = a.gbdt_levels
        a.labels = "balanced" if a.gbdt_data == "both" else a.gbdt_data
        a.late = a.gbdt_late
        res = bench_gbdt(a, dev, info)
        out = res
    elif a.model == "varsel":
        out = bench_varsel(a, dev, info)
    elif a.model == "lr":
        out = bench_lr(a, dev, info)
    elif a.model == "treeinfer":
        out = bench_treeinfer(a, dev, info)
    elif a.model == "pipeline":
        out = bench_pipeline(a, dev, info)
    elif a.model == "corr":
        out = bench_corr(a, dev, info)
    elif a.model == "eval":
        out = bench_eval(a, dev, info)
    elif a.model == "stats":
        if not gpu and a.cols == 1000:
            a.cols = 64
        out = bench_stats(a, dev, info)
    else:
        dt, errs, flops_row, extra = bench_mlp(a, dev, info)
        # max over ranks of the timed span; per-rank step-time spread and all-reduce time
        tmax = torch.tensor([dt, extra["t_local"], extra["comm_ms"]], dtype=torch.float64, device=dev)
        tmin = tmax.clone()
        dist.all_reduce_(tmax, "max")
        dist.all_reduce_(tmin, "min")
        dt = float(tmax[0].item())
        ms = dt / a.steps * 1e3
        total_rows = a.rows * info.world_size
        value = total_rows * a.steps / dt
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "rows/s",
            "n_gpus": info.world_size,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": value / BASELINE_MLP_ROWS_PER_S,
            "dtype": "bf16",
            "data": "synthetic (N(0,1) features, labels from a hidden linear rule), random-init weights",
            "config": {"model": "MLP 1000-500-200-1 (sigmoid, RPROP, squared loss, full-batch epoch)",
                       "global_batch": total_rows, "seq_len": None, "n_cols": a.cols,
                       "rows_per_gpu": a.rows, "parallelism": f"dp{info.world_size}"},
            "achieved_tflops": value * flops_row / 1e12,
            "baseline_note": "baseline = 1.48M rows/s derived from CHANGES.txt:268 (SURVEY §6)",
            "final_train_error": errs[-1] if errs else None,
            "rank_step_ms_max": float(tmax[1]) / a.steps * 1e3, "rank_step_ms_min": float(tmin[1]) / a.steps * 1e3,
            "allreduce_ms_per_step": float(tmax[2]) / a.steps,
            "allreduce_ms_per_step_min_rank": float(tmin[2]) / a.steps,
        }
        if gpu:      # HBM headroom per rank (RCCL buffers for N > 1 must fit beside the rows)
            out["hbm_peak_gb"] = torch.cuda.max_memory_allocated(dev) / 1e9
            out["hbm_total_gb"] = torch.cuda.get_device_properties(dev).total_memory / 1e9
        if a.gbdt_steps > 0:
            out.update(gbdt_half(a, dev, info))
    if info.rank == 0:
        print(json.dumps(out), flush=True)
    dist.shutdown()


if __name__ == "__main__":
    main()
