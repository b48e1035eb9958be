set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u tools/strip_lab.py --rounds 3 > gpurun_out/r6/strip_lab_b.jsonl 2> gpurun_out/r6/strip_lab_b.err &&
timeout -k 10 900 python -u bench.py --model varsel --stream --rows 21000000 --cols 10000 --host-rows 2097152 --steps 2 --warmup 1 > gpurun_out/r6/varsel_stream_21Mx10k.json 2> gpurun_out/r6/varsel_stream_21Mx10k.err
