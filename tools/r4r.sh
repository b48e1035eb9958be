#!/bin/bash
# r4r: pooled page-locked block buffers (no hipHostMalloc inside a pass) -- tests, 3M profile,
# and the 20M x 1600 pipeline once more.
set -o pipefail
out=gpurun_out/r4r
mkdir -p $out
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
hb=$!
trap "kill $hb" EXIT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_stats_stream.py tests/test_gpu_parse.py tests/test_norm_stream.py > $out/gpu_tests.txt 2>&1 || { tail -40 $out/gpu_tests.txt; exit 1; }
tail -2 $out/gpu_tests.txt
timeout -k 10 300 python tools/pipe_lab.py --rows 3000000 --cols 1600 --steps stats norm --top 25 > $out/pipe_lab_3M.txt 2>&1 || { tail -30 $out/pipe_lab_3M.txt; exit 1; }
grep "^====\|GPU parse" $out/pipe_lab_3M.txt | cut -c1-300
timeout -k 10 900 python bench.py --model pipeline --rows 20000000 --cols 1600 --pipeline-epochs 400 --pipeline-replicate 8 --pipeline-tmp /dev/shm --pipeline-eval-rows 20000000 > $out/bench_pipeline_20M.json 2> $out/bench_pipeline_20M.err || { tail -30 $out/bench_pipeline_20M.err; exit 1; }
python -c "import json; d=json.loads(open('$out/bench_pipeline_20M.json').read().strip().splitlines()[-1]); print(d['step_seconds'], d['value'], d.get('eval_auc'), d.get('se_recall_of_planted_columns'), d['varsel_phases_s (SE: rows load, NN training, sensitivity)'], d['train_setup_s'])"
grep "GPU parse" $out/bench_pipeline_20M.err | cut -c1-300
