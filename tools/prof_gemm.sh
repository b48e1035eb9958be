#!/usr/bin/env bash
# PMC profile of the MLP kernels (two counter passes; never combined with sys/runtime traces).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out/prof_gemm
export PYTHONPATH=$(pwd)
timeout -k 10 300 python3 tools/bench_gemm.py --iters 10 > gpurun_out/prof_gemm/bench_gemm.json
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES \
  --output-format csv -d $R/gpurun_out/prof_gemm/sq -o sq -- python3 $R/tools/bench_gemm.py --iters 3
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT \
  --output-format csv -d $R/gpurun_out/prof_gemm/tcc -o tcc -- python3 $R/tools/bench_gemm.py --iters 3
