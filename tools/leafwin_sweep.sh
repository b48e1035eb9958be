#!/bin/bash
# Kernel time of the final-level GBT prediction update (gbdt_leaf_window_kernel) per window size
# W and blocks per window Y: rocprofv3 kernel trace of a short balanced GBDT bench per setting.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/leafwin
export TMPDIR=/tmp
# LEAFWIN_SET: "W:Y W:Y ..." settings to measure
for wy in ${LEAFWIN_SET:-65536:16 65536:32}; do
  set -- ${wy/:/ }
  SHIFU_GBDT_LEAF_W=$1 SHIFU_GBDT_LEAF_Y=$2 timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv \
    -d gpurun_out/leafwin/w$1_y$2 -o r -- python3 bench.py --model gbdt --gbdt-data balanced --steps 3 --warmup 1 \
    > gpurun_out/leafwin/w$1_y$2.json 2>/dev/null || exit 1
  python3 - "$1" "$2" <<'PY'
import csv, glob, sys
t = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for f in glob.glob(f"gpurun_out/leafwin/w{sys.argv[1]}_y{sys.argv[2]}/**/*kernel_trace.csv", recursive=True)
     for r in csv.DictReader(open(f)) if "leaf_window" in r["Kernel_Name"]]
print(f"W={sys.argv[1]} Y={sys.argv[2]} calls={len(t)} mean_ms={sum(t)/max(1,len(t))/1e6:.3f}", flush=True)
PY
done
