# Two PMC passes over the GBDT bench, summarised per kernel family (the raw CSVs stay on the box).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=.
OUT=gpurun_out/r6/gbdtpmc
mkdir -p "$OUT"
LAB=${1:-favourable}
i=0
for ctrs in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" \
            "FETCH_SIZE TA_BUSY_avr GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU"; do
  i=$((i + 1))
  timeout -s KILL 300 rocprofv3 --pmc $ctrs --output-format csv -d /tmp/pmc$i -o run -- \
    python3 -u bench.py --model gbdt --steps 2 --warmup 1 --gbdt-data $LAB > "$OUT/p$i.log" 2>&1 || { tail -20 "$OUT/p$i.log"; exit 1; }
  python3 tools/r6/pmc_summary.py $(ls /tmp/pmc$i/*counter_collection.csv /tmp/pmc$i/*/*counter_collection.csv 2>/dev/null | head -1) > "$OUT/p$i.json" || exit 1
done
cat "$OUT"/p1.json | head -50
