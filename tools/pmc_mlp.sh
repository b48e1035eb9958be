#!/usr/bin/env bash
# PMC counters of every kernel of the MLP training step (bench.py, 1M rows in 256K-row chunks so no
# per-dispatch counter saturates at 2^31).  One counter group per rocprofv3 run, --pmc never combined
# with tracing.  Summary: python tools/pmc_kernels.py gpurun_out/pmc_mlp
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
R=$(pwd)
export PYTHONPATH=$R
O=$R/gpurun_out/pmc_mlp
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
    python3 $R/bench.py --rows 1048576 --chunk-rows 262144 --steps 1 --warmup 0 --gbdt-steps 0 > $O/g$gi.log 2>&1
  echo "group $gi done"
done
