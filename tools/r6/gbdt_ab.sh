# GBDT: GPU tests, then the GBDT bench with device decisions (default) and with host decisions
# (SHIFU_GBDT_DEV_DECIDE=0) on the same box.
#   gpurun --timeout 1200 -- bash tools/r6/gbdt_ab.sh TAG [extra bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=. TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/r6/gbdt_$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gbdt.py -m gpu \
  > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
timeout -k 10 600 python -u bench.py --model gbdt --gbdt-steps 5 --gbdt-warmup 1 --gbdt-levels "$@" \
  > "$OUT/bench_dev.json" 2> "$OUT/bench_dev.log" || { tail -30 "$OUT/bench_dev.log"; exit 1; }
cat "$OUT/bench_dev.json" | cut -c1-400
SHIFU_GBDT_DEV_DECIDE=0 timeout -k 10 600 python -u bench.py --model gbdt --gbdt-steps 5 --gbdt-warmup 1 \
  --gbdt-levels "$@" > "$OUT/bench_host.json" 2> "$OUT/bench_host.log" || { tail -30 "$OUT/bench_host.log"; exit 1; }
cat "$OUT/bench_host.json" | cut -c1-400
