#!/bin/bash
# r4b: new GPU tests (device-collective guard with 2 ranks on one GPU, signed-zero sort, GBT one-hot
# streamed norm, TF on the MLP engine, batched SMO, SE first layer), then the default bench line
# with both GBDT workloads + per-level tables, a later window of the balanced workload, and the
# forward-GEMM ablations.  Test failures (pytest rc 1) do not stop the benches; crashes/timeouts do.
set -o pipefail
out=gpurun_out/r4b
mkdir -p $out
(df -h /tmp . ; free -g; nproc) > $out/box_info.txt 2>&1
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_dist_stats.py tests/test_sort_gpu.py tests/test_norm_stream.py tests/test_tensorflow_alg.py \
  tests/test_svm.py tests/test_stats_kernels_gpu.py tests/test_stats_stream.py > $out/gpu_tests_new.txt 2>&1
rc=$?
tail -5 $out/gpu_tests_new.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --gbdt-levels > $out/bench_default.json 2> $out/bench_default.err || { tail -20 $out/bench_default.err; exit 1; }
cut -c1-400 $out/bench_default.json
timeout -k 10 300 python bench.py --model gbdt --gbdt-data balanced --gbdt-late 50 --steps 5 --warmup 1 --gbdt-levels > $out/bench_gbdt_balanced_late50.json 2> $out/bench_gbdt_balanced_late50.err || exit 1
# forward-GEMM ablations (dbg bits: 2 main loop only, 32 A rows from an L2-resident window, 64 no MFMA,
# 128 no activation in the epilogue)
timeout -k 10 300 python tools/mlp_lab.py --iters 5 --dbg 0 2 34 66 98 128 > $out/mlp_lab_fwd_ablation.jsonl 2> $out/mlp_lab.err
