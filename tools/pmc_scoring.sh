#!/usr/bin/env bash
# PMC counters of every kernel of the K13 tree-inference and GBDT root-u32 kernels (bench.py treeinfer 1M rows, gbdt 4M rows; no
# per-dispatch counter saturates at 2^31).  One counter group per rocprofv3 run, --pmc never combined
# with tracing.  Summary: python tools/pmc_kernels.py gpurun_out/pmc_scoring
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
R=$(pwd)
export PYTHONPATH=$R
O=$R/gpurun_out/pmc_scoring
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
groups=(
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY"
  "FETCH_SIZE GRBM_GUI_ACTIVE"
  "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
  "SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
)
for gi in "${!groups[@]}"; do
  timeout -s KILL 120 rocprofv3 --pmc ${groups[$gi]} --output-format csv -d $O/g$gi -o run -- \
    python3 $R/bench.py --model treeinfer --rows 1048576 --steps 1 --warmup 0 > $O/g$gi.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc ${groups[$gi]} --output-format csv -d $O/gh$gi -o run -- \
    python3 $R/bench.py --model gbdt --rows 4000000 --steps 2 --warmup 1 > $O/gh$gi.log 2>&1
  echo "group $gi done"
done
