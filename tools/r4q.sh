#!/bin/bash
# r4q: where the streamed text pipeline waits -- pass logs with read times (3M x 1600) and a HIP
# runtime + kernel trace of stats at 1M x 1600.
set -o pipefail
out=gpurun_out/r4q
mkdir -p $out
timeout -k 10 300 python tools/pipe_lab.py --rows 3000000 --cols 1600 --steps stats norm --top 25 > $out/pipe_lab_3M.txt 2>&1 || { tail -30 $out/pipe_lab_3M.txt; exit 1; }
grep "^====\|GPU parse" $out/pipe_lab_3M.txt | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --runtime-trace --kernel-trace --stats --output-format csv -d $out/prof -o trace -- python tools/pipe_lab.py --rows 1000000 --cols 1600 --steps stats --top 5 > $out/prof_run.txt 2>&1 || { tail -30 $out/prof_run.txt; exit 1; }
find $out/prof -name "*.csv" | head -20
