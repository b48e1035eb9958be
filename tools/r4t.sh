#!/bin/bash
# r4t: persistent forward at the bench chunk shape -- bitwise test, per-kernel lab A/B, bench line.
set -o pipefail
out=gpurun_out/r4t
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_mlp_gpu.py > $out/gpu_tests.txt 2>&1 || { tail -40 $out/gpu_tests.txt; exit 1; }
tail -2 $out/gpu_tests.txt
timeout -k 10 300 python tools/mlp_lab.py --iters 5 --tune 10:0 10:1 > $out/mlp_lab_persist.jsonl 2> $out/mlp_lab.err || { tail -20 $out/mlp_lab.err; exit 1; }
cat $out/mlp_lab_persist.jsonl
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > $out/bench_default.json 2> $out/bench_default.err || { tail -30 $out/bench_default.err; exit 1; }
cut -c1-300 $out/bench_default.json
