# GBDT bench A/B over environment settings on one box.
#   gpurun --timeout 1200 -- bash tools/r6/gbdt_env_ab.sh TAG "ENV=1 ENV2=0" "ENV=0" ...   ("-" = no env)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=. TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/r6/gbdtenv_$TAG
mkdir -p "$OUT"
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
