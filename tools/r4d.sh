#!/bin/bash
# r4d: where the pipeline steps' time goes now (cProfile, 1M x 1600 on the GPU path), the
# persistent-head A/B on the full MLP bench (same box), and the dgrad 8-phase (--big 3) lab variant.
set -o pipefail
out=gpurun_out/r4d
mkdir -p $out
timeout -k 10 500 python tools/pipe_lab.py --rows 1000000 --cols 1600 --steps stats norm eval --top 30 > $out/pipe_lab_1Mx1600.txt 2>&1 || { tail -20 $out/pipe_lab_1Mx1600.txt; exit 1; }
grep "^====" $out/pipe_lab_1Mx1600.txt
for hp in 0 1; do
  SHIFU_HEAD_PERSIST=$hp timeout -k 10 300 python bench.py --steps 10 --warmup 3 --gbdt-steps 0 > $out/bench_mlp_headpersist$hp.json 2> $out/bench_mlp_headpersist$hp.err || exit 1
  cut -c1-200 $out/bench_mlp_headpersist$hp.json
done
timeout -k 10 300 python tools/mlp_lab.py --iters 5 --big 0 3 > $out/mlp_lab_big.jsonl 2> $out/mlp_lab_big.err || exit 1
cat $out/mlp_lab_big.jsonl
