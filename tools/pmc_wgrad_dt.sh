#!/usr/bin/env bash
# PMC A/B: wgrad1 (both operands via ds_read_b64_tr_b16) vs wgrad1_dt (D via ds_read_b128).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
R=$(pwd); export PYTHONPATH=$R; O=$R/gpurun_out/pmc_wgrad_dt; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for k in wgrad1 wgrad1_dt; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_LDS \
    --output-format csv -d $O/sq_$k -o r -- python3 $R/tools/bench_gemm.py --big 0 --iters 3 --only dgrad1_t $k > $O/sq_$k.json
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $O/tcc_$k -o r \
    -- python3 $R/tools/bench_gemm.py --big 0 --iters 3 --only dgrad1_t $k > $O/tcc_$k.json
done
