#!/bin/bash
# r4f: GPU text parsing (K0) -- bit-identity tests, then stats + norm at 1M x 1600 with the GPU
# parse off and on (same box, same generated data shape).
set -o pipefail
out=gpurun_out/r4f
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parse.py tests/test_norm_stream.py > $out/gpu_tests.txt 2>&1 || { tail -40 $out/gpu_tests.txt; exit 1; }
tail -3 $out/gpu_tests.txt
for gp in false true; do
  timeout -k 10 400 python tools/pipe_lab.py --rows 1000000 --cols 1600 --steps stats norm --top 40 --props shifu.data.gpuParse=$gp > $out/pipe_lab_gpuparse_$gp.txt 2>&1 || { tail -30 $out/pipe_lab_gpuparse_$gp.txt; exit 1; }
  grep "^====\|generated" $out/pipe_lab_gpuparse_$gp.txt
done
