#!/bin/bash
# r4c: (0) MLP GPU tests incl. the persistent head (now default) + head A/B in the lab + the MLP bench;
# (1) the CLI pipeline at the largest reference-width shape the box's disk holds (3M training +
# 0.75M eval rows x 1600 columns, 400 epochs: varsel SE trains 200 epochs over all 1600 candidates);
# (2) a roctx marker trace of `shifu train` (GBT) with its range summary.
set -o pipefail
out=gpurun_out/r4c
mkdir -p $out
root=$(pwd)
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_mlp_gpu.py > $out/gpu_tests_mlp.txt 2>&1
rc=$?
tail -4 $out/gpu_tests_mlp.txt
if [ $rc -ne 0 ]; then echo "mlp tests rc $rc: stopping"; exit $rc; fi
timeout -k 10 300 python tools/mlp_lab.py --iters 5 --tune 11:0 11:1 > $out/mlp_lab_head_persist.jsonl 2> $out/mlp_lab.err || exit 1
cat $out/mlp_lab_head_persist.jsonl
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --gbdt-steps 0 > $out/bench_mlp.json 2> $out/bench_mlp.err || exit 1
cut -c1-300 $out/bench_mlp.json
timeout -k 10 900 python bench.py --model pipeline --rows 3000000 --pipeline-epochs 400 --workdir /tmp/shifu_pipe \
  > $out/bench_pipeline_3Mx1600.json 2> $out/bench_pipeline_3Mx1600.err || { tail -30 $out/bench_pipeline_3Mx1600.err; exit 1; }
cut -c1-600 $out/bench_pipeline_3Mx1600.json
rm -rf /tmp/shifu_pipe
timeout -k 10 300 python tools/gbt_model_set.py /tmp/gbtms --rows 1000000 --num 60 --trees 20 > $out/gbt_prep.log 2>&1 || { tail -20 $out/gbt_prep.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace -d $root/$out/gbt_trace -o run -- python3 $root/tools/run_in.py /tmp/gbtms/gbt train > $root/$out/gbt_trace.log 2>&1 || { tail -20 $root/$out/gbt_trace.log; exit 1; }
cd $root
db=$(ls $out/gbt_trace/*.db $out/gbt_trace/*/*.db 2>/dev/null | head -1)
python tools/marker_summary.py $db --top shifu.train --json $out/gbt_marker_summary.json
