# strip head: numerics tests, then the per-kernel chunk table with and without it
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u -m pytest tests/test_mlp_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "strip_head or fused_head or bench_configuration or two_chunk" > gpurun_out/r6/strip_head_tests_$1.log 2>&1 \
  || { tail -30 gpurun_out/r6/strip_head_tests_$1.log; exit 1; }
tail -3 gpurun_out/r6/strip_head_tests_$1.log
timeout -k 10 200 python -u tools/mlp_lab.py --iters 5 > gpurun_out/r6/mlp_lab_strip_head_$1.jsonl 2>&1 || exit 1
timeout -k 10 200 python -u tools/mlp_lab.py --iters 5 --env SHIFU_STRIP_HEAD=0 >> gpurun_out/r6/mlp_lab_strip_head_$1.jsonl 2>&1 || exit 1
cat gpurun_out/r6/mlp_lab_strip_head_$1.jsonl
