"""bench.py --gpus N launches N ranks itself (no torchrun): gloo on CPU, world size 2."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=600):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env["SHIFU_FORCE_CPU"] = "1"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       env=env, timeout=timeout, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_bench_gpus2_launches_two_ranks():
    out = _run(["--gpus", "2", "--rows", "4000", "--cols", "64", "--steps", "2", "--warmup", "1",
                "--gbdt-steps", "1", "--gbdt-warmup", "0", "--gbdt-rows", "500"])
    assert out["n_gpus"] == 2
    assert out["config"]["parallelism"] == "dp2"
    assert out["config"]["global_batch"] == 8000
    assert out["value"] > 0 and "gbdt_rounds_per_s" in out
    assert out["gbdt_config"]["parallelism"] == "dp2"
    assert out["rank_step_ms_max"] >= out["rank_step_ms_min"] > 0
    assert out["allreduce_ms_per_step"] >= 0


def test_bench_gpus1_single_process():
    out = _run(["--gpus", "1", "--rows", "2000", "--cols", "64", "--steps", "1", "--warmup", "0",
                "--gbdt-steps", "0"])
    assert out["n_gpus"] == 1 and out["config"]["parallelism"] == "dp1"


def test_bench_launcher_fails_fast_when_a_rank_dies():
    """one rank exits at init -> the launcher stops the others and returns non-zero
    promptly (not after the 1800 s process-group timeout)."""
    import time
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(SHIFU_FORCE_CPU="1", SHIFU_BENCH_FAIL_RANK="1")
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--rows", "4000", "--cols", "64",
                        "--steps", "2", "--warmup", "1", "--gbdt-steps", "0"], capture_output=True, text=True,
                       env=env, timeout=120, cwd=ROOT)
    dt = time.monotonic() - t0
    assert p.returncode != 0, p.stdout
    assert dt < 30, dt
    assert "a rank failed" in p.stderr
