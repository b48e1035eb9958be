set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u tools/strip_lab.py --rounds 3 > gpurun_out/r6/strip_lab_$1.jsonl 2> gpurun_out/r6/strip_lab_$1.err
