#!/usr/bin/env bash
# PMC A/B of the wgrad kernels (128x128 register-staged vs 256x256 8-phase) at the forward-1
# shape (1M rows, 512 x 1024 output).  One counter pass per run, no traces.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
R=$(pwd)
export PYTHONPATH=$R
O=$R/gpurun_out/pmc_wgrad
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for big in 0 3; do
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --output-format csv -d $O/tcc$big -o r \
    -- python3 $R/tools/bench_gemm.py --big $big --iters 3 --only wgrad1 > $O/tcc$big.json
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_LDS \
    --output-format csv -d $O/sq$big -o r -- python3 $R/tools/bench_gemm.py --big $big --iters 3 --only wgrad1 > $O/sq$big.json
  timeout -s KILL 90 rocprofv3 --pmc TCC_MISS_sum TCC_EA0_ATOMIC_sum GRBM_GUI_ACTIVE --output-format csv -d $O/tcm$big -o r \
    -- python3 $R/tools/bench_gemm.py --big $big --iters 3 --only wgrad1 > $O/tcm$big.json
done
