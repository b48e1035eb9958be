#!/bin/bash
# Run GPU steps in order, each under its own time limit: "name|seconds|command" per argument.
# A step ending in 0 or 1 (test failures) lets the next one start; anything else (fault, abort,
# time limit, signal) ends the script there.
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  echo "[steps] $name (limit ${secs}s)"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[steps] $name rc=$rc"; tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[steps] stopping after $name"; exit $rc; fi
done
