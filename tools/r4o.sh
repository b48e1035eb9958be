#!/bin/bash
# r4o: staged cache uploads on by default -> the 20M x 1600 pipeline (20M eval rows) again.
set -o pipefail
out=gpurun_out/r4o
mkdir -p $out
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
hb=$!
trap "kill $hb" EXIT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_norm_stream.py > $out/gpu_tests.txt 2>&1 || { tail -40 $out/gpu_tests.txt; exit 1; }
tail -2 $out/gpu_tests.txt
timeout -k 10 900 python bench.py --model pipeline --rows 20000000 --cols 1600 --pipeline-epochs 400 --pipeline-replicate 8 --pipeline-tmp /dev/shm --pipeline-eval-rows 20000000 > $out/bench_pipeline_20M.json 2> $out/bench_pipeline_20M.err || { tail -30 $out/bench_pipeline_20M.err; exit 1; }
python -c "import json; d=json.loads(open('$out/bench_pipeline_20M.json').read().strip().splitlines()[-1]); print(d['step_seconds'], d['value'], d.get('eval_auc'), d.get('se_recall_of_planted_columns'), d['varsel_phases_s (SE: rows load, NN training, sensitivity)'], d['train_setup_s'])"
