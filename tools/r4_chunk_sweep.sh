#!/bin/bash
# MLP bench at several chunk sizes (MALL residency of the per-chunk intermediates), then a
# kernel-trace profile of the 64K-row chunk variant.
set -o pipefail
out=gpurun_out/r4a
mkdir -p $out
for c in 2097152 262144 131072 65536; do
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --gbdt-steps 0 --chunk-rows $c > $out/bench_c$c.json 2> $out/bench_c$c.err || exit $?
  echo "chunk $c: $(cat $out/bench_c$c.json)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof64k -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --gbdt-steps 0 --chunk-rows 65536 --rows 16777216 > $GRAFT_REPO_ROOT/$out/prof64k.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof2m -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --gbdt-steps 0 --chunk-rows 2097152 --rows 16777216 > $GRAFT_REPO_ROOT/$out/prof2m.log 2>&1
