# GBDT GPU tests, then the GBDT bench (both label sets) over environment variants ("-" = none).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=. TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/r6/gbdtab_$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gbdt.py tests/test_gbdt_gpu_dist.py -m gpu \
  > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
i=0
for v in "$@"; do
  i=$((i + 1))
  for lab in balanced favourable; do
    envs=""; [ "$v" != "-" ] && envs="$v"
    env $envs timeout -k 10 300 python -u bench.py --model gbdt --steps 6 --warmup 2 --gbdt-data $lab --gbdt-levels \
      > "$OUT/b${i}_$lab.json" 2> "$OUT/b${i}_$lab.log" || { tail -20 "$OUT/b${i}_$lab.log"; exit 1; }
    python3 -c "
import json
d=json.loads(open('$OUT/b${i}_$lab.json').read().strip().splitlines()[-1])
print('[$v]', '$lab', round(d['value'],3), round(d['ms_per_step'],2), [(l['level'], l['ms_per_round']) for l in (d.get('levels') or [])])"
  done
done
