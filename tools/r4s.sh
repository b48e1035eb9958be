#!/bin/bash
# r4s: rocprofv3 kernel statistics of the default bench line (MLP + GBDT) on the final tree.
set -o pipefail
out=gpurun_out/r4s
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o bench -- python bench.py --steps 3 --warmup 1 --gbdt-steps 2 > $out/bench.json 2> $out/bench.err || { tail -30 $out/bench.err; exit 1; }
cut -c1-300 $out/bench.json
head -25 $(find $out/prof -name "*kernel_stats.csv" | head -1) | cut -c1-200
rm -f $(find $out/prof -name "*kernel_trace.csv")
