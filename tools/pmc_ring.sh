#!/bin/bash
# PMC passes over the ring-GEMM lab kernels (one counter group per run; rocprofv3 --pmc never
# combined with tracing domains).  Usage: tools/pmc_ring.sh <outdir> <case...>
set -e
out=$1; shift
mkdir -p "$out"
export PYTHONPATH=.
groups=(
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
  "GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU"
  "FETCH_SIZE TCC_HIT_sum TA_BUSY_avr"
)
for c in "$@"; do
  mkdir -p "$out/$c"
  for gi in "${!groups[@]}"; do
    timeout -s KILL 90 rocprofv3 --pmc ${groups[$gi]} --output-format csv -d "$out/$c/g$gi" -o run -- \
      python3 tools/ring_lab.py --no-check --rounds 1 --only "$c" > "$out/$c/g$gi.log" 2>&1
  done
done
