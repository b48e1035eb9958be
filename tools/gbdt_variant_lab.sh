#!/usr/bin/env bash
# GBDT histogram A/B: the bench's balanced GBDT half with per-level timings, one process per
# SHIFU_HIST_PF value (the kernel choice is read once per process).
#   gpurun -- bash tools/gbdt_variant_lab.sh TAG 1 3 4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH=$(pwd)
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
# each argument: PF[:ROOT_HU[:ITEMS]]
for spec in "$@"; do
  IFS=: read -r v rh it <<< "$spec"
  rh=${rh:-2}; it=${it:-2048}
  SHIFU_HIST_PF=$v SHIFU_HIST_ROOT_HU=$rh SHIFU_GBDT_ITEMS=$it timeout -k 10 300 python -u bench.py --model gbdt --gbdt-data balanced --steps 3 --warmup 1 \
    --gbdt-levels > $O/v$v-$rh-$it.json 2> $O/v$v-$rh-$it.log || { echo "variant $spec failed"; tail -3 $O/v$v-$rh-$it.log; exit 1; }
  python -c "
import json; d=json.loads(open('$O/v$v-$rh-$it.json').read().strip().splitlines()[-1])
print('$spec', round(d['ms_per_step'],1), [(l['level'], l['ms_per_round'], l['tb_per_s']) for l in d['levels']])"
done
