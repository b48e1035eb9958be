#!/bin/bash
# r4k: the whole GPU test suite + smoke on the final tree (what the driver runs at round end).
set -o pipefail
out=gpurun_out/r4k
mkdir -p $out
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $out/gpu_tests_full.txt 2>&1; rc=$?
tail -5 $out/gpu_tests_full.txt
grep -E "FAILED|ERROR" $out/gpu_tests_full.txt | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || { tail -20 $out/smoke.txt; exit 1; }
tail -3 $out/smoke.txt
