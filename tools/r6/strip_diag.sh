mkdir -p gpurun_out/r6
timeout -k 10 200 python -u tools/r6/strip_diag.py > gpurun_out/r6/strip_diag_$1.jsonl 2> gpurun_out/r6/strip_diag_$1.err
