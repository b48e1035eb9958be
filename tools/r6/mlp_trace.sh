# Kernel trace of the MLP half of the default bench (no GBDT) for the per-chunk timeline.
#   gpurun --timeout 900 -- bash tools/r6/mlp_trace.sh TAG [extra bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=. TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/r6/mlptrace_$TAG
mkdir -p "$OUT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/t" -o run -- \
  python3 -u bench.py --gbdt-steps 0 --steps 3 --warmup 1 "$@" > "$OUT/bench.json" 2> "$OUT/bench.log" \
  || { tail -20 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.json" | cut -c1-300
