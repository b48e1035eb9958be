#!/bin/bash
# Same-box A/B of one kernel between two builds of the HIP library: rocprofv3 kernel traces of
# the same command with SHIFU_HIP_LIB unset (in-tree build) and set to $BASE_LIB, alternating
# RUNS times; prints the mean time of kernels whose name contains $KERNEL.
#   KERNEL=partition_scatter BASE_LIB=ab/libshifu_hip_base.so bash tools/kernel_ab.sh python3 bench.py ...
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/kernel_ab
mkdir -p $O
for i in $(seq 1 ${RUNS:-2}); do
  for v in base new; do
    if [ $v = base ]; then export SHIFU_HIP_LIB=$PWD/$BASE_LIB; else unset SHIFU_HIP_LIB; fi
    timeout -k 10 ${STEP_SECS:-200} rocprofv3 --kernel-trace --output-format csv -d $O/${v}_$i -o r -- "$@" \
      > $O/${v}_$i.out 2>/dev/null || exit 1
    python3 - "$O/${v}_$i" "$KERNEL" "$v" <<'PY'
import csv, glob, sys
t = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for f in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)
     for r in csv.DictReader(open(f)) if sys.argv[2] in r["Kernel_Name"]]
print(f"{sys.argv[3]:4s} {sys.argv[1]} {sys.argv[2]} calls={len(t)} mean_ms={sum(t)/max(1,len(t))/1e6:.4f}", flush=True)
PY
  done
done
