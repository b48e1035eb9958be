#!/bin/bash
# r4e: fp32 NN scoring on the own split-bf16 GEMM (tests + eval bench throughput vs vendor fp32),
# then the persistent-head A/B on the full MLP bench and the dgrad 8-phase (--big 3) lab variant.
set -o pipefail
out=gpurun_out/r4e
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gemm_ops.py tests/test_mlp_gpu.py tests/test_stats_kernels_gpu.py > $out/gpu_tests.txt 2>&1 || { tail -30 $out/gpu_tests.txt; exit 1; }
tail -3 $out/gpu_tests.txt
timeout -k 10 300 python bench.py --model eval --steps 3 --warmup 1 > $out/bench_eval.json 2> $out/bench_eval.err || { tail -20 $out/bench_eval.err; exit 1; }
python -c "import json; d=json.loads(open('$out/bench_eval.json').read().strip().splitlines()[-1]); print({k: v for k, v in d.items() if k.startswith('nn_')})"
for hp in 0 1; do
  SHIFU_HEAD_PERSIST=$hp timeout -k 10 300 python bench.py --steps 10 --warmup 3 --gbdt-steps 0 > $out/bench_mlp_headpersist$hp.json 2> $out/bench_mlp_headpersist$hp.err || exit 1
  cut -c1-200 $out/bench_mlp_headpersist$hp.json
done
timeout -k 10 300 python tools/mlp_lab.py --iters 5 --big 0 3 > $out/mlp_lab_big.jsonl 2> $out/mlp_lab_big.err || exit 1
cat $out/mlp_lab_big.jsonl
