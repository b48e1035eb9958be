"""Data-parallel `shifu stats` (algos/dist_stats.py): 2 gloo ranks over row shards must write the
same ColumnConfig as one process over all rows (exact distributed equal-population cuts,
global category order, merged histograms / moments / distinct counts)."""
import json
import os
import shutil
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_stats(rank, world, port, root):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), SHIFU_FORCE_CPU="1")
    from shifu_amd.parallel import dist
    from shifu_amd.steps.stats import run_stats
    dist.init_from_env("gloo")
    run_stats(root)
    dist.barrier()
    dist.shutdown()


@pytest.mark.parametrize("method", ["EqualTotal", "EqualPositive", "WeightEqualTotal", "EqualInterval"])
def test_stats_two_ranks_match_single(tmp_path, method, monkeypatch):
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.steps.create import run_init
    from shifu_amd.steps.stats import run_stats
    from shifu_amd.utils.synthetic import make_model_set
    a = make_model_set(str(tmp_path), "a", "NN", n_rows=1501, n_num=6, n_cat=3)
    mc = ModelConfig.load(os.path.join(a, "ModelConfig.json"))
    mc.stats["binningMethod"] = method
    mc.stats["maxNumBin"] = 12
    mc.save()
    run_init(a)
    b = str(tmp_path / "b")
    shutil.copytree(a, b)
    run_stats(a)
    mp.start_processes(_rank_stats, args=(2, _port(), b), nprocs=2, join=True, start_method="spawn")
    ca = json.load(open(os.path.join(a, "ColumnConfig.json")))
    cb = json.load(open(os.path.join(b, "ColumnConfig.json")))
    assert len(ca) == len(cb)
    for x, y in zip(ca, cb):
        bx, by = x["columnBinning"], y["columnBinning"]
        assert bx.get("binBoundary") == by.get("binBoundary"), x["columnName"]
        assert bx.get("binCategory") == by.get("binCategory"), x["columnName"]
        for k in ("binCountPos", "binCountNeg"):
            assert bx.get(k) == by.get(k), (x["columnName"], k)
        for k in ("binWeightedPos", "binWeightedNeg", "binCountWoe"):
            if bx.get(k) is not None:
                np.testing.assert_allclose(bx[k], by[k], rtol=1e-9, atol=1e-9)
        sx, sy = x["columnStats"], y["columnStats"]
        for k in ("totalCount", "missingCount", "distinctCount", "max", "min"):
            assert sx.get(k) == sy.get(k), (x["columnName"], k)
        for k in ("mean", "stdDev", "ks", "iv", "median", "skewness", "kurtosis"):
            if sx.get(k) is not None:
                np.testing.assert_allclose(sx[k], sy[k], rtol=1e-9, atol=1e-9, err_msg=f"{x['columnName']} {k}")


def test_hll_estimate_accuracy():
    import torch
    from shifu_amd.algos.dist_stats import hll_estimate, hll_registers
    v = torch.arange(200000, dtype=torch.float64) * 0.37
    est = hll_estimate(torch.maximum(hll_registers(v[:120000]), hll_registers(v[80000:])))
    assert abs(est - 200000) / 200000 < 0.03


def _rank_cli(rank, world, port, root, verb):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), SHIFU_FORCE_CPU="1")
    os.chdir(root)
    from shifu_amd.cli import main
    rc = main(verb.split())
    if rc != 0:
        raise SystemExit(rc)


def test_cli_pipeline_two_ranks(tmp_path):
    """stats, norm, varsel, train, posttrain and eval (all data parallel) driven through the CLI by
    2 gloo ranks, as `SHIFU_GPUS=2 shifu ...` does."""
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.steps.create import run_init
    from shifu_amd.utils.synthetic import make_model_set
    root = make_model_set(str(tmp_path), "d", "NN", n_rows=900, n_num=6, n_cat=2)
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    mc.train["numTrainEpochs"] = 15
    mc.train["baggingNum"] = 1
    mc.save()
    run_init(root)
    for verb in ("stats", "norm", "varsel", "train", "posttrain", "eval"):
        mp.start_processes(_rank_cli, args=(2, _port(), root, verb), nprocs=2, join=True, start_method="spawn")
    assert os.path.exists(os.path.join(root, "models", "model0.nn"))
    perf = json.load(open(os.path.join(root, "evals", "Eval1", "EvalPerformance.json")))
    assert perf["areaUnderRoc"] > 0.7
    # the 2-rank (sharded scoring + gather) eval equals a single-process eval of the same models
    def score_rows():
        p = os.path.join(root, "evals", "Eval1", "EvalScore")
        p = os.path.join(p, "part-00000") if os.path.isdir(p) else p
        return open(p).read()
    two = score_rows()
    cwd = os.getcwd()
    os.environ["SHIFU_FORCE_CPU"] = "1"
    try:
        os.chdir(root)
        from shifu_amd.cli import main
        assert main(["eval"]) == 0
    finally:
        os.chdir(cwd)
    one = score_rows()
    r1 = [l.split("|") for l in one.strip().split("\n")]
    r2 = [l.split("|") for l in two.strip().split("\n")]
    assert r1[0] == r2[0] and len(r1) == len(r2)
    j = r1[0].index("mean")
    m1, m2 = np.array([float(r[j]) for r in r1[1:]]), np.array([float(r[j]) for r in r2[1:]])
    np.testing.assert_allclose(m1, m2, atol=1e-3)        # fp32 GEMM blocking differs by batch shape
    assert sorted(r[0] for r in r1[1:]) == sorted(r[0] for r in r2[1:])
    perf1 = json.load(open(os.path.join(root, "evals", "Eval1", "EvalPerformance.json")))
    assert abs(perf1["areaUnderRoc"] - perf["areaUnderRoc"]) < 1e-3


def _rank_cli_guarded(rank, world, port, root, verb, gpu):
    """One CLI verb on one rank with SHIFU_ASSERT_DEVICE_COLLECTIVES=1 (every collective tensor on
    the rank's compute device, RCCL's contract).  gpu: both ranks share cuda:0 over gloo."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), SHIFU_ASSERT_DEVICE_COLLECTIVES="1", SHIFU_DIST_BACKEND="gloo")
    if not gpu:
        os.environ["SHIFU_FORCE_CPU"] = "1"
    os.chdir(root)
    from shifu_amd.cli import main
    rc = main(verb.split())
    if rc != 0:
        raise SystemExit(rc)


def _guarded_pipeline(tmp_path, gpu, world=2):
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.steps.create import run_init
    from shifu_amd.utils.synthetic import make_model_set
    root = make_model_set(str(tmp_path), "g", "NN", n_rows=900, n_num=6, n_cat=2)
    mc = ModelConfig.load(os.path.join(root, "ModelConfig.json"))
    mc.train["numTrainEpochs"] = 8
    mc.train["baggingNum"] = 1
    mc.evals[0]["scoreMetaColumnNameFile"] = "columns/Eval1score.meta.column.names"
    mc.save()
    with open(os.path.join(root, "columns", "Eval1score.meta.column.names"), "w") as f:
        f.write("id\n")                                 # a champion score column: the max goes over ranks
    run_init(root)
    for verb in ("stats", "norm", "varsel", "train", "posttrain", "eval"):
        mp.start_processes(_rank_cli_guarded, args=(world, _port(), root, verb, gpu), nprocs=world, join=True,
                           start_method="spawn")
    assert os.path.exists(os.path.join(root, "evals", "Eval1", "EvalMetaScore", "idEvalPerformance.json"))
    return root


def test_cli_two_ranks_device_collective_guard(tmp_path):
    """the data-parallel verbs incl. eval with score meta columns under the
    device-collective guard (host run: the guard's contract is the host device)."""
    _guarded_pipeline(tmp_path, gpu=False)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_cli_ranks_device_collectives_gpu(tmp_path, world):
    """2 or 4 ranks on one GPU (gloo transport, guard on): a collective over a host tensor,
    which RCCL would reject (the r3 eval champion-score crash), raises here."""
    import torch
    assert torch.cuda.is_available()
    _guarded_pipeline(tmp_path, gpu=True, world=world)


@pytest.mark.parametrize("alg,shuffle", [("NN", False), ("NN", True), ("GBT", False)])
def test_norm_two_ranks_match_single(tmp_path, alg, shuffle):
    """Data-parallel norm (each rank normalizes its output row range and writes it in place into
    the shared .npy caches) == single-process norm, with and without -shuffle."""
    from shifu_amd.steps.base import load_dataset_cache
    from shifu_amd.steps.create import run_init
    from shifu_amd.steps.norm import run_norm
    from shifu_amd.steps.stats import run_stats
    from shifu_amd.utils.synthetic import make_model_set
    os.environ["SHIFU_FORCE_CPU"] = "1"
    a = make_model_set(str(tmp_path), "a", alg, n_rows=1203, n_num=5, n_cat=2)
    run_init(a)
    run_stats(a)
    b = str(tmp_path / "b")
    shutil.copytree(a, b)
    run_norm(a, shuffle=shuffle)
    verb = "norm -shuffle" if shuffle else "norm"
    mp.start_processes(_rank_cli, args=(2, _port(), b, verb), nprocs=2, join=True, start_method="spawn")
    sub = "CleanedData" if alg == "GBT" else "NormalizedData"
    ma, xa = load_dataset_cache(os.path.join(a, "tmp", sub), mmap=False)
    mb, xb = load_dataset_cache(os.path.join(b, "tmp", sub), mmap=False)
    assert ma["n"] == mb["n"] and set(xa) == set(xb)
    for k in xa:
        np.testing.assert_array_equal(xa[k], xb[k], err_msg=k)


def test_varsel_se_and_posttrain_two_ranks_match_single(tmp_path):
    """Row-sharded SE sensitivity (all-reduced per-input sums, gradients all-reduced in the quick
    NN) and row-sharded posttrain (all-reduced per-bin score sums) == one process."""
    from shifu_amd.config.column_config import load_column_configs
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.steps.create import run_init
    from shifu_amd.steps.posttrain import run_posttrain
    from shifu_amd.steps.stats import run_stats
    from shifu_amd.steps.train import run_train
    from shifu_amd.steps.varsel import run_varsel
    from shifu_amd.utils.synthetic import make_model_set
    os.environ["SHIFU_FORCE_CPU"] = "1"
    a = make_model_set(str(tmp_path), "a", "NN", n_rows=1100, n_num=7, n_cat=2)
    mc = ModelConfig.load(os.path.join(a, "ModelConfig.json"))
    mc.varSelect["filterBy"] = "SE"
    mc.varSelect["filterNum"] = 5
    mc.varSelect["autoFilterEnable"] = False
    mc.train["numTrainEpochs"] = 12
    mc.train["baggingNum"] = 1
    mc.save()
    run_init(a)
    run_stats(a)
    b = str(tmp_path / "b")
    shutil.copytree(a, b)
    run_varsel(a)
    mp.start_processes(_rank_cli, args=(2, _port(), b, "varsel"), nprocs=2, join=True, start_method="spawn")
    def se(root):
        rows = [l.split("\t") for l in open(os.path.join(root, "varsel", "se.0")).read().strip().split("\n")]
        return {r[1]: float(r[3]) for r in rows}
    sa, sb = se(a), se(b)
    assert sa.keys() == sb.keys()
    np.testing.assert_allclose([sa[k] for k in sa], [sb[k] for k in sa], rtol=2e-3, atol=1e-6)
    fa = sorted(c.name for c in load_column_configs(os.path.join(a, "ColumnConfig.json")) if c.final_select)
    fb = sorted(c.name for c in load_column_configs(os.path.join(b, "ColumnConfig.json")) if c.final_select)
    assert fa == fb and len(fa) == 5
    # posttrain on the same model files
    run_train(a)
    shutil.rmtree(os.path.join(b, "models"), ignore_errors=True)
    shutil.copytree(os.path.join(a, "models"), os.path.join(b, "models"))
    run_posttrain(a)
    mp.start_processes(_rank_cli, args=(2, _port(), b, "posttrain"), nprocs=2, join=True, start_method="spawn")
    ba = {c.name: c.bin_avg_score for c in load_column_configs(os.path.join(a, "ColumnConfig.json")) if c.final_select}
    bb = {c.name: c.bin_avg_score for c in load_column_configs(os.path.join(b, "ColumnConfig.json")) if c.final_select}
    assert ba.keys() == bb.keys() and all(ba[k] for k in ba)
    for k in ba:
        assert np.max(np.abs(np.array(ba[k]) - np.array(bb[k]))) <= 1, k


def test_correlation_two_ranks_match_single(tmp_path):
    """`stats -c` data parallel: row-sharded pairwise-complete sums all-reduced once == one process."""
    from shifu_amd.steps.create import run_init
    from shifu_amd.steps.stats import read_correlation, run_stats
    from shifu_amd.utils.synthetic import make_model_set
    os.environ["SHIFU_FORCE_CPU"] = "1"
    a = make_model_set(str(tmp_path), "a", "NN", n_rows=1301, n_num=6, n_cat=2)
    run_init(a)
    run_stats(a)
    b = str(tmp_path / "b")
    shutil.copytree(a, b)
    run_stats(a, correlation=True)
    mp.start_processes(_rank_cli, args=(2, _port(), b, "stats -c"), nprocs=2, join=True, start_method="spawn")
    na, ca = read_correlation(os.path.join(a, "correlation.csv"))
    nb, cb = read_correlation(os.path.join(b, "correlation.csv"))
    assert na == nb and len(na) >= 6
    np.testing.assert_allclose(ca, cb, atol=1e-10)


def test_psi_two_ranks_match_single(tmp_path):
    """`stats -p` data parallel: global unit set + all-reduced (unit, bin) counts == one process."""
    from shifu_amd.config.column_config import load_column_configs
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.steps.create import run_init
    from shifu_amd.steps.stats import run_stats
    from shifu_amd.utils.synthetic import make_model_set
    os.environ["SHIFU_FORCE_CPU"] = "1"
    a = make_model_set(str(tmp_path), "a", "NN", n_rows=1250, n_num=5, n_cat=2)
    mc = ModelConfig.load(os.path.join(a, "ModelConfig.json"))
    mc.stats["psiColumnName"] = "cat_0"
    mc.save()
    run_init(a)
    run_stats(a)
    b = str(tmp_path / "b")
    shutil.copytree(a, b)
    from shifu_amd.config.column_config import save_column_configs
    ccb = load_column_configs(os.path.join(b, "ColumnConfig.json"))
    for c in ccb:                           # b's PSI must come from the 2-rank run
        c.stats["psi"] = None
    save_column_configs(ccb, os.path.join(b, "ColumnConfig.json"))
    run_stats(a, psi=True)
    mp.start_processes(_rank_cli, args=(2, _port(), b, "stats -p"), nprocs=2, join=True, start_method="spawn")
    pa = {c.name: c.stats.get("psi") for c in load_column_configs(os.path.join(a, "ColumnConfig.json"))}
    pb = {c.name: c.stats.get("psi") for c in load_column_configs(os.path.join(b, "ColumnConfig.json"))}
    keys = [k for k in pa if pa[k] is not None]
    assert keys and all(pb[k] is not None for k in keys)
    np.testing.assert_allclose([pa[k] for k in keys], [pb[k] for k in keys], rtol=1e-9, atol=1e-12)
    def unit_stats(root):            # {col: [(unit, mean, missing rate, count)]}
        out = {}
        for line in open(os.path.join(root, "tmp", "columnconfig.unitstats")).read().splitlines():
            col, rest = line.split("|", 1)
            out[col] = [(u, float(m), float(r), int(n)) for u, m, r, n in (x.split("^") for x in rest.split("\u0001"))]
        return out
    ua, ub = unit_stats(a), unit_stats(b)
    assert ua.keys() == ub.keys() and ua
    for k in ua:                    # value sums are all-reduced: equal up to summation order
        assert [(u, n) for u, _, _, n in ua[k]] == [(u, n) for u, _, _, n in ub[k]]
        np.testing.assert_allclose([x[1:3] for x in ua[k]], [x[1:3] for x in ub[k]], rtol=1e-12)


def _java_psi(expected, per_unit_counts):
    """PSICalculatorUDF.exec :70-97 transcribed literally (index advances only on added terms)."""
    import math
    psi = 0.0
    for sub in per_unit_counts:
        total = float(sum(sub))
        i = 0
        for s in sub:
            if total == 0:
                continue
            elif expected[i] == 0:
                continue
            else:
                log_num = (s / total) / expected[i]
                if log_num <= 0:
                    continue
                psi += (s / total - expected[i]) * math.log(log_num)
            i += 1
    return psi


def test_psi_reference_parity(tmp_path):
    """PSI from the ColumnConfig stats' expected distribution + the UDF's loop, and unit stats
    'unit^mean^missingRate^count' (sorted, \\u0001-joined) in tmp/columnconfig.unitstats."""
    from shifu_amd.algos import binning as B
    from shifu_amd.config.column_config import load_column_configs
    from shifu_amd.config.jsonio import java_double_str
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.steps.base import ModelSet
    from shifu_amd.steps.create import run_init
    from shifu_amd.steps.stats import run_stats
    from shifu_amd.utils.synthetic import make_model_set
    os.environ["SHIFU_FORCE_CPU"] = "1"
    a = make_model_set(str(tmp_path), "a", "NN", n_rows=900, n_num=4, n_cat=2)
    mc = ModelConfig.load(os.path.join(a, "ModelConfig.json"))
    mc.stats["psiColumnName"] = "cat_0"
    mc.save()
    run_init(a)
    run_stats(a)
    run_stats(a, psi=True)
    ccs = load_column_configs(os.path.join(a, "ColumnConfig.json"))
    ms = ModelSet(a)
    md = ms.load_raw([c for c in ms.ccs if c.name in ("num_0", "cat_0")])
    units_s = md.table["cat_0"].strings()
    units = sorted(set(units_s))
    cc = next(c for c in ccs if c.name == "num_0")
    v = md.table["num_0"].numeric()
    bidx = B.bin_index_numeric(v, cc.bin_boundary)
    nb = len(cc.bin_boundary) + 1
    per_unit = [np.bincount(bidx[units_s == u], minlength=nb) for u in units]
    tot = float(cc.stat("totalCount"))
    expected = [(n + p) / tot for n, p in zip(cc.bin_count_neg, cc.bin_count_pos)]
    assert abs(cc.stats["psi"] - _java_psi(expected, per_unit)) < 1e-12
    lines = dict(l.split("|", 1) for l in open(os.path.join(a, "tmp", "columnconfig.unitstats")).read().splitlines())
    stats = lines[str(cc.num)].split("\u0001")
    assert stats == sorted(stats) and len(stats) == len(units)
    u0 = units[0]
    m = units_s == u0
    n0, miss = int(m.sum()), int(np.isnan(v[m]).sum())
    mean = float("nan") if n0 == miss else float(np.nansum(v[m])) / n0
    want = f"{u0}^{java_double_str(mean)}^{java_double_str(miss / n0)}^{n0}"
    assert want in stats


def test_correlation_reuse_skips_data_pass(tmp_path, monkeypatch):
    """shifu.stats.corr.reuse=true with a cached matrix for the same columns rewrites
    correlation.csv from the cache (a sentinel planted in the cache must come out)."""
    from shifu_amd.config import environment
    from shifu_amd.steps.create import run_init
    from shifu_amd.steps.stats import read_correlation, run_stats
    from shifu_amd.utils.synthetic import make_model_set
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    a = make_model_set(str(tmp_path), "a", "NN", n_rows=700, n_num=4, n_cat=1)
    run_init(a)
    run_stats(a)
    run_stats(a, correlation=True)
    n1, c1 = read_correlation(os.path.join(a, "correlation.csv"))
    cache = os.path.join(a, "tmp", "CorrelationPath", "corr.npy")
    C = np.load(cache)
    C[0, 1] = C[1, 0] = 0.123456
    np.save(cache, C)
    run_stats(a, correlation=True)                      # reuse off: recomputed
    n2, c2 = read_correlation(os.path.join(a, "correlation.csv"))
    np.testing.assert_allclose(c2, c1, rtol=1e-12)
    np.save(cache, C)
    environment.set_property("shifu.stats.corr.reuse", "true")
    try:
        run_stats(a, correlation=True)
    finally:
        environment.set_property("shifu.stats.corr.reuse", "false")
    n3, c3 = read_correlation(os.path.join(a, "correlation.csv"))
    assert n3 == n1 and abs(c3[0, 1] - 0.123456) < 1e-12


def _rank_norm_rss(rank, world, port, root, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), SHIFU_FORCE_CPU="1")
    from shifu_amd.parallel import dist
    from shifu_amd.steps.norm import run_norm
    dist.init_from_env("gloo")

    def status(key):
        for line in open("/proc/self/status"):
            if line.startswith(key):
                return int(line.split()[1]) * 1024
    open("/proc/self/clear_refs", "w").write("5")
    base = status("VmRSS:")
    run_norm(root)
    with open(f"{out}.{rank}", "w") as f:
        f.write(str(status("VmHWM:") - base))
    dist.barrier()
    dist.shutdown()


def test_norm_per_rank_host_memory(tmp_path):
    """Data-parallel norm parses only each rank's byte range: per-rank peak host memory growth is
    about 1/R of the single-process growth plus a fixed ~65 MB of buffers (2 ranks: < 0.5x + 80 MB)."""
    from shifu_amd.config.model_config import ModelConfig
    from shifu_amd.steps.create import run_init
    from shifu_amd.steps.stats import run_stats
    from shifu_amd.utils.synthetic import make_model_set
    root = make_model_set(str(tmp_path), "m", "NN", n_rows=320_000, n_num=30, n_cat=2)
    run_init(root)
    os.environ["SHIFU_FORCE_CPU"] = "1"
    run_stats(root)
    out = str(tmp_path / "rss")
    mp.start_processes(_rank_norm_rss, args=(1, _port(), root, out + "1"), nprocs=1, join=True, start_method="spawn")
    mp.start_processes(_rank_norm_rss, args=(2, _port(), root, out + "2"), nprocs=2, join=True, start_method="spawn")
    single = int(open(out + "1.0").read())
    ranks = [int(open(f"{out}2.{r}").read()) for r in range(2)]
    print("norm rss growth MB: 1 rank %.1f, 2 ranks %s" % (single / 1e6, [round(r / 1e6, 1) for r in ranks]))
    assert max(ranks) < 0.5 * single + 80e6, (single, ranks)


def _rank_stats_one_empty(rank, world, port, root):
    """Rank 1's byte range yields no valid rows (all filtered / no line start); rank 0 streams all."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), SHIFU_FORCE_CPU="1")
    from shifu_amd.config import environment
    from shifu_amd.data import stream as DS
    from shifu_amd.parallel import dist
    from shifu_amd.steps.stats import run_stats
    orig = DS.iter_model_data

    def rows_of(mc, plan, chunk, r, w, *a, **k):
        return iter(()) if r == 1 else orig(mc, plan, chunk, 0, 1, *a, **k)
    DS.iter_model_data = rows_of
    environment.props()["shifu.stats.streaming"] = "true"
    environment.props()["shifu.stats.chunkMB"] = str(8 / 1024)
    dist.init_from_env("gloo")
    run_stats(root)
    dist.barrier()
    dist.shutdown()


def test_streamed_stats_rank_without_rows(tmp_path, monkeypatch):
    """a rank with no rows must still join every merge with same-sized partials."""
    monkeypatch.setenv("SHIFU_FORCE_CPU", "1")
    from shifu_amd.config import environment
    from shifu_amd.steps.create import run_init
    from shifu_amd.steps.stats import run_stats
    from shifu_amd.utils.synthetic import make_model_set
    a = make_model_set(str(tmp_path), "a", "NN", n_rows=1201, n_num=5, n_cat=2)
    run_init(a)
    b = str(tmp_path / "b")
    shutil.copytree(a, b)
    monkeypatch.setitem(environment.props(), "shifu.stats.streaming", "true")
    run_stats(a)
    mp.start_processes(_rank_stats_one_empty, args=(2, _port(), b), nprocs=2, join=True, start_method="spawn")
    ca = json.load(open(os.path.join(a, "ColumnConfig.json")))
    cb = json.load(open(os.path.join(b, "ColumnConfig.json")))
    for x, y in zip(ca, cb):
        assert x["columnBinning"].get("binBoundary") == y["columnBinning"].get("binBoundary"), x["columnName"]
        assert x["columnBinning"].get("binCountPos") == y["columnBinning"].get("binCountPos"), x["columnName"]
        for k in ("totalCount", "missingCount", "max", "min"):
            assert x["columnStats"].get(k) == y["columnStats"].get(k), (x["columnName"], k)
        if x["columnStats"].get("mean") is not None:
            np.testing.assert_allclose(x["columnStats"]["mean"], y["columnStats"]["mean"], rtol=1e-9)
