#!/bin/bash
# r4b: new GPU tests (device-collective guard with 2 ranks on one GPU, signed-zero sort, GBT one-hot
# streamed norm), then the default bench line with both GBDT workloads + per-level tables, then a
# later window (rounds 51-55) of the balanced workload.
set -o pipefail
out=gpurun_out/r4b
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_dist_stats.py tests/test_sort_gpu.py tests/test_norm_stream.py tests/test_tensorflow_alg.py tests/test_svm.py tests/test_stats_kernels_gpu.py > $out/gpu_tests_new.txt 2>&1 || { tail -30 $out/gpu_tests_new.txt; exit 1; }
tail -3 $out/gpu_tests_new.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --gbdt-levels > $out/bench_default.json 2> $out/bench_default.err || { tail -20 $out/bench_default.err; exit 1; }
cat $out/bench_default.json | cut -c1-600
timeout -k 10 300 python bench.py --model gbdt --gbdt-data balanced --gbdt-late 50 --steps 5 --warmup 1 --gbdt-levels > $out/bench_gbdt_balanced_late50.json 2> $out/bench_gbdt_balanced_late50.err
# forward-GEMM ablations (dbg bits: 2 main loop only, 32 A rows from an L2-resident window, 64 no MFMA,
# 128 no activation in the epilogue)
timeout -k 10 300 python tools/mlp_lab.py --iters 5 --dbg 0 2 34 66 98 128 > $out/mlp_lab_fwd_ablation.jsonl 2> $out/mlp_lab.err
