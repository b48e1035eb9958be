#!/bin/bash
# r4m: 1 GB GPU-path blocks by default; upload-rate lab (pinned staging vs pageable from /dev/shm);
# the 20M x 1600 pipeline with the 20M-row eval set again.
set -o pipefail
out=gpurun_out/r4m
mkdir -p $out
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
hb=$!
trap "kill $hb" EXIT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_stats_stream.py tests/test_gpu_parse.py tests/test_norm_stream.py tests/test_dist_stats.py > $out/gpu_tests.txt 2>&1 || { tail -40 $out/gpu_tests.txt; exit 1; }
tail -2 $out/gpu_tests.txt
timeout -k 10 300 python tools/upload_lab.py --rows 4000000 > $out/upload_lab.txt 2>&1 || { tail -20 $out/upload_lab.txt; exit 1; }
tail -1 $out/upload_lab.txt
timeout -k 10 900 python bench.py --model pipeline --rows 20000000 --cols 1600 --pipeline-epochs 400 --pipeline-replicate 8 --pipeline-tmp /dev/shm --pipeline-eval-rows 20000000 > $out/bench_pipeline_20M.json 2> $out/bench_pipeline_20M.err || { tail -30 $out/bench_pipeline_20M.err; exit 1; }
python -c "import json; d=json.loads(open('$out/bench_pipeline_20M.json').read().strip().splitlines()[-1]); print(d['step_seconds'], d['value'], d.get('eval_auc'), d.get('se_recall_of_planted_columns'), d['varsel_phases_s (SE: rows load, NN training, sensitivity)'], d['train_setup_s'])"
grep "GPU parse:" $out/bench_pipeline_20M.err | cut -c1-250
