# MLP bench (no GBDT) A/B over bench arguments on one box ("-" = defaults; "=" stands for a space).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=. TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/r6/mlpargs_$TAG
mkdir -p "$OUT"
i=0
for v in "$@"; do
  i=$((i + 1))
  args=""; [ "$v" != "-" ] && args=${v//=/ }
  timeout -k 10 300 python -u bench.py --gbdt-steps 0 --steps 5 --warmup 2 $args > "$OUT/b$i.json" 2> "$OUT/b$i.log" \
    || { tail -20 "$OUT/b$i.log"; exit 1; }
  python3 -c "
import json
d=json.loads(open('$OUT/b$i.json').read().strip().splitlines()[-1])
print('[$v]', round(d['value']/1e6,2), 'M rows/s', round(d['ms_per_step'],2), 'ms/epoch')"
done
