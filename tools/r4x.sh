#!/bin/bash
# r4x: MLP chunk rows above 2M (per-chunk fixed costs amortised; HBM permitting).
set -o pipefail
out=gpurun_out/r4x
mkdir -p $out
for cr in 2097152 2621440 3145728; do
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 --gbdt-steps 0 --chunk-rows $cr > $out/bench_mlp_chunk$cr.json 2> $out/bench_mlp_chunk$cr.err || { tail -5 $out/bench_mlp_chunk$cr.err; echo "chunk $cr failed"; continue; }
  python -c "import json; d=json.loads(open('$out/bench_mlp_chunk$cr.json').read().strip().splitlines()[-1]); print($cr, d['value'], d['ms_per_step'], d.get('hbm_peak_gb'))"
done
