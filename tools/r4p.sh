#!/bin/bash
# r4p: queue depth of the streamed text pipeline (read | H2D | parse | consumer) at 3M x 1600.
set -o pipefail
out=gpurun_out/r4p
mkdir -p $out
for d in 1 2 3; do
  SHIFU_READ_PREFETCH=$d timeout -k 10 300 python tools/pipe_lab.py --rows 3000000 --cols 1600 --steps stats norm --top 25 --props shifu.data.prefetch=$d > $out/pipe_lab_3M_depth$d.txt 2>&1 || { tail -30 $out/pipe_lab_3M_depth$d.txt; exit 1; }
  echo "depth $d"; grep "^====" $out/pipe_lab_3M_depth$d.txt
done
