#!/bin/bash
# r4n: staged-upload equality test, the 20M x 1600 pipeline (1 GB stats blocks, pageable cache
# uploads) and the default bench line on the final tree.
set -o pipefail
out=gpurun_out/r4n
mkdir -p $out
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
hb=$!
trap "kill $hb" EXIT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_norm_stream.py tests/test_gpu_parse.py > $out/gpu_tests.txt 2>&1 || { tail -40 $out/gpu_tests.txt; exit 1; }
tail -2 $out/gpu_tests.txt
timeout -k 10 300 python tools/upload_lab.py --rows 4000000 > $out/upload_lab.txt 2>&1 || { tail -20 $out/upload_lab.txt; exit 1; }
tail -1 $out/upload_lab.txt
timeout -k 10 900 python bench.py --model pipeline --rows 20000000 --cols 1600 --pipeline-epochs 400 --pipeline-replicate 8 --pipeline-tmp /dev/shm --pipeline-eval-rows 20000000 > $out/bench_pipeline_20M.json 2> $out/bench_pipeline_20M.err || { tail -30 $out/bench_pipeline_20M.err; exit 1; }
python -c "import json; d=json.loads(open('$out/bench_pipeline_20M.json').read().strip().splitlines()[-1]); print(d['step_seconds'], d['value'], d.get('eval_auc'), d.get('se_recall_of_planted_columns'), d['varsel_phases_s (SE: rows load, NN training, sensitivity)'], d['train_setup_s'])"
grep "GPU parse:" $out/bench_pipeline_20M.err | head -3 | cut -c1-250
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > $out/bench_default.json 2> $out/bench_default.err || { tail -30 $out/bench_default.err; exit 1; }
cut -c1-400 $out/bench_default.json
