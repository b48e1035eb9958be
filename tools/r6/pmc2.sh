# Two PMC passes over a bench.py run, summarised per kernel family (raw CSVs stay on the box).
#   gpurun -- bash tools/r6/pmc2.sh TAG <bench args...>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=.
TAG=$1; shift
OUT=gpurun_out/r6/pmc_$TAG
mkdir -p "$OUT"
i=0
for ctrs in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES" \
            "FETCH_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE"; do
  i=$((i + 1))
  timeout -s KILL 300 rocprofv3 --pmc $ctrs --output-format csv -d /tmp/pmc$i -o run -- \
    python3 -u bench.py "$@" > "$OUT/p$i.log" 2>&1 || { tail -20 "$OUT/p$i.log"; exit 1; }
  python3 tools/r6/pmc_summary.py $(ls /tmp/pmc$i/*counter_collection.csv /tmp/pmc$i/*/*counter_collection.csv 2>/dev/null | head -1) > "$OUT/p$i.json" || exit 1
done
echo done
