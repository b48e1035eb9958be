#!/bin/bash
# r4u: HIP hardware queues per process vs the streamed text pipeline (3M x 1600 stats + norm).
set -o pipefail
out=gpurun_out/r4u
mkdir -p $out
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python tools/pipe_lab.py --rows 3000000 --cols 1600 --steps stats norm --top 20 > $out/pipe_lab_3M_q$q.txt 2>&1 || { tail -30 $out/pipe_lab_3M_q$q.txt; exit 1; }
  echo "queues $q"; grep "^====\|GPU parse" $out/pipe_lab_3M_q$q.txt | cut -c1-260
done
