#!/bin/bash
# r4g: GPU parse + one-hot kernel tests, stats/norm profile at 1M x 1600, and the 3M x 1600
# pipeline bench (400 epochs) to compare with r4c (host parse).
set -o pipefail
out=gpurun_out/r4g
mkdir -p $out
df -h / /dev/shm /tmp > $out/df.txt 2>&1
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parse.py tests/test_norm_stream.py tests/test_gemm_ops.py > $out/gpu_tests.txt 2>&1 || { tail -40 $out/gpu_tests.txt; exit 1; }
tail -2 $out/gpu_tests.txt
timeout -k 10 300 python tools/pipe_lab.py --rows 1000000 --cols 1600 --steps stats norm --top 30 > $out/pipe_lab_1M.txt 2>&1 || { tail -30 $out/pipe_lab_1M.txt; exit 1; }
grep "^====" $out/pipe_lab_1M.txt
timeout -k 10 500 python bench.py --model pipeline --rows 3000000 --cols 1600 --pipeline-epochs 400 > $out/bench_pipeline_3M.json 2> $out/bench_pipeline_3M.err || { tail -30 $out/bench_pipeline_3M.err; exit 1; }
python -c "import json; d=json.loads(open('$out/bench_pipeline_3M.json').read().strip().splitlines()[-1]); print(d['step_seconds'], d['value'], d.get('eval_auc'), d.get('se_recall_of_planted_columns'))"
