# MLP bench (no GBDT) A/B over environment settings on one box, after the MLP GPU tests.
#   gpurun --timeout 1200 -- bash tools/r6/mlp_env_ab.sh TAG "ENV=1" "-" ...   ("-" = no env)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=. TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/r6/mlpenv_$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_mlp_gpu.py -m gpu \
  > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
i=0
for v in "$@"; do
  i=$((i + 1))
  envs=""; [ "$v" != "-" ] && envs="$v"
  env $envs timeout -k 10 300 python -u bench.py --gbdt-steps 0 --steps 5 --warmup 2 > "$OUT/b$i.json" 2> "$OUT/b$i.log" \
    || { tail -20 "$OUT/b$i.log"; exit 1; }
  python3 -c "
import json
d=json.loads(open('$OUT/b$i.json').read().strip().splitlines()[-1])
print('[$v]', round(d['value']/1e6,2), 'M rows/s', round(d['ms_per_step'],2), 'ms/epoch')"
done
