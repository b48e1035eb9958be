# Same-box A/B of the MLP bench half: ring forward (SHIFU_GEMM_TUNE=14=0) vs the strip engine
# (default), alternating, two rounds each.
set -o pipefail
mkdir -p gpurun_out/r6
for r in 1 2; do
  SHIFU_GEMM_TUNE=14=0 timeout -k 10 200 python -u bench.py --gbdt-steps 0 --steps 5 --warmup 2 \
    > gpurun_out/r6/ab_ring_$r.json 2> gpurun_out/r6/ab_ring_$r.err || exit 1
  timeout -k 10 200 python -u bench.py --gbdt-steps 0 --steps 5 --warmup 2 \
    > gpurun_out/r6/ab_strip_$r.json 2> gpurun_out/r6/ab_strip_$r.err || exit 1
done
