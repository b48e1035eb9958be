#!/bin/bash
# r4v: GIL switch interval vs the streamed text pipeline (3M x 1600 stats + norm).
set -o pipefail
out=gpurun_out/r4v
mkdir -p $out
for sw in 5 0.5 0.1; do
  SHIFU_GIL_SWITCH_MS=$sw timeout -k 10 300 python tools/pipe_lab.py --rows 3000000 --cols 1600 --steps stats norm --top 20 > $out/pipe_lab_3M_sw$sw.txt 2>&1 || { tail -30 $out/pipe_lab_3M_sw$sw.txt; exit 1; }
  echo "switch $sw ms"; grep "^====\|GPU parse" $out/pipe_lab_3M_sw$sw.txt | cut -c1-260
done
