# Prefetch-depth A/B of the GBDT histogram kernels (root tile ROOT_PD, half-record H64_PD).
#   gpurun --timeout 1200 -- bash tools/r6/gbdt_pd.sh TAG "rootpd,h64pd" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=. TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/r6/gbdtpd_$TAG
mkdir -p "$OUT"
last=${@: -1}
SHIFU_GBDT_ROOT_PD=${last%,*} SHIFU_GBDT_H64_PD=${last#*,} timeout -k 10 300 python -u -m pytest -x -q --timeout 200 \
  --timeout-method thread tests/test_gbdt.py -m gpu > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for v in "$@"; do
  for lab in balanced favourable; do
    SHIFU_GBDT_ROOT_PD=${v%,*} SHIFU_GBDT_H64_PD=${v#*,} timeout -k 10 300 python -u bench.py --model gbdt --steps 6 \
      --warmup 1 --gbdt-data $lab --gbdt-levels > "$OUT/b_${v/,/_}_$lab.json" 2> "$OUT/b_${v/,/_}_$lab.log" \
      || { tail -20 "$OUT/b_${v/,/_}_$lab.log"; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open('$OUT/b_${v/,/_}_$lab.json').read().strip().splitlines()[-1])
print('$v', '$lab', round(d['value'],3), round(d['ms_per_step'],2), [(l['level'], l['ms_per_round'], l['tb_per_s']) for l in (d.get('levels') or [])])"
  done
done
