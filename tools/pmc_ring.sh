#!/usr/bin/env bash
# PMC counters of the forward GEMM kernels (tools/ring_lab.py --no-lab: 8-phase + ring variants at
# the bench's 2M x 1024 -> 512 chunk), one counter group per rocprofv3 run (--pmc never combined with
# tracing).  Summary: python tools/pmc_summary.py gpurun_out/pmc_ring ring0=ring_nt_kernel ...
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
R=$(pwd)
export PYTHONPATH=$R
O=$R/gpurun_out/pmc_ring/${1:-fwd}
shift || true
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
groups=(
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS"
  "FETCH_SIZE GRBM_GUI_ACTIVE"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
)
for gi in "${!groups[@]}"; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc ${groups[$gi]} --output-format csv -d $O/g$gi -o run -- \
    python3 $R/tools/ring_lab.py --no-lab --rounds 1 --iters 3 "$@" > $O/g$gi.log 2>&1
  echo "group $gi done"
done
