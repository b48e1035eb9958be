# Kernel traces of the GBDT bench (device decisions vs host decisions) for tools/kernel_gaps.py.
#   gpurun --timeout 1200 -- bash tools/r6/gbdt_prof.sh TAG LABELS
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=. TMPDIR=/tmp
TAG=$1; LAB=${2:-balanced}
OUT=gpurun_out/r6/gbdtprof_$TAG
mkdir -p "$OUT"
cd /tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/dev" -o run -- \
  python3 -u bench.py --model gbdt --steps 6 --warmup 1 --gbdt-data "$LAB" > "$OUT/dev.json" 2> "$OUT/dev.log" \
  || { tail -20 "$OUT/dev.log"; exit 1; }
python3 tools/kernel_gaps.py $(ls "$OUT"/dev/*/run_kernel_trace.csv "$OUT"/dev/run_kernel_trace.csv 2>/dev/null | head -1) \
  --json "$OUT/dev_gaps.json" | tail -2
SHIFU_GBDT_DEV_DECIDE=0 timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/host" -o run -- \
  python3 -u bench.py --model gbdt --steps 6 --warmup 1 --gbdt-data "$LAB" > "$OUT/host.json" 2> "$OUT/host.log" \
  || { tail -20 "$OUT/host.log"; exit 1; }
python3 tools/kernel_gaps.py $(ls "$OUT"/host/*/run_kernel_trace.csv "$OUT"/host/run_kernel_trace.csv 2>/dev/null | head -1) \
  --json "$OUT/host_gaps.json" | tail -2
