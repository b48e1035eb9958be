#!/bin/bash
# r4l: the whole GPU suite + smoke (round-end check), then r4j's measurements.
set -o pipefail
out=gpurun_out/r4l
mkdir -p $out
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
hb=$!
trap "kill $hb" EXIT
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $out/gpu_tests_full.txt 2>&1; rc=$?
tail -3 $out/gpu_tests_full.txt
grep -E "FAILED|ERROR" $out/gpu_tests_full.txt | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || { tail -20 $out/smoke.txt; exit 1; }
tail -2 $out/smoke.txt
timeout -k 10 400 python tools/pipe_lab.py --rows 3000000 --cols 1600 --steps stats norm --top 30 > $out/pipe_lab_3M.txt 2>&1 || { tail -30 $out/pipe_lab_3M.txt; exit 1; }
grep "^====\|GPU parse:" $out/pipe_lab_3M.txt | cut -c1-250
timeout -k 10 400 python tools/pipe_lab.py --rows 3000000 --cols 1600 --steps stats norm --top 30 --props shifu.stats.chunkMB=1024 shifu.norm.chunkMB=1024 > $out/pipe_lab_3M_chunk1G.txt 2>&1 || { tail -30 $out/pipe_lab_3M_chunk1G.txt; exit 1; }
grep "^====\|GPU parse:" $out/pipe_lab_3M_chunk1G.txt | cut -c1-250
timeout -k 10 900 python bench.py --model pipeline --rows 20000000 --cols 1600 --pipeline-epochs 400 --pipeline-replicate 8 --pipeline-tmp /dev/shm --pipeline-eval-rows 20000000 > $out/bench_pipeline_20M.json 2> $out/bench_pipeline_20M.err || { tail -30 $out/bench_pipeline_20M.err; exit 1; }
python -c "import json; d=json.loads(open('$out/bench_pipeline_20M.json').read().strip().splitlines()[-1]); print(d['step_seconds'], d['value'], d.get('eval_auc'), d.get('se_recall_of_planted_columns'))"
grep "GPU parse:" $out/bench_pipeline_20M.err | cut -c1-250
