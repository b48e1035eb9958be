#!/usr/bin/env bash
# PMC passes over the GBDT histogram kernel (bench.py --model gbdt, 20M rows x 1000 cols).
# One counter group per run, no traces; summary of gbdt_hist_kernel dispatches to stdout.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
R=$(pwd)
export PYTHONPATH=$R
O=$R/gpurun_out/pmc_gbdt
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS="--model gbdt --rows 20000000 --steps 2 --warmup 1"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --output-format csv -d $O/tcc -o r \
  -- python3 $R/bench.py $ARGS > $O/tcc.json
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_LDS \
  --output-format csv -d $O/sq -o r -- python3 $R/bench.py $ARGS > $O/sq.json
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE \
  --output-format csv -d $O/sq2 -o r -- python3 $R/bench.py $ARGS > $O/sq2.json
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o r \
  -- python3 $R/bench.py $ARGS > $O/kt.json
python3 - "$O" <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
for grp in ("tcc", "sq", "sq2"):
    tot = collections.defaultdict(float)
    n = collections.Counter()
    for f in glob.glob(f"{O}/{grp}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if "gbdt_hist_kernel" not in row["Kernel_Name"]:
                continue
            tot[row["Counter_Name"]] += float(row["Counter_Value"])
            n[row["Counter_Name"]] += 1
    for k in sorted(tot):
        print(f"{grp:4s} {k:28s} total {tot[k]:.4e} over {n[k]} dispatch-records")
ms = 0.0
for f in glob.glob(f"{O}/kt/**/*kernel_trace.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "gbdt_hist_kernel" in row["Kernel_Name"]:
            ms += (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6
print(f"gbdt_hist_kernel total kernel time {ms:.2f} ms (kernel-trace run)")
PY
