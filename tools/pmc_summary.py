"""Summarise rocprofv3 --pmc counter CSVs (layout <dir>/<case>/g*/...csv, one counter group per g* run):
per case, the mean per-dispatch value of every counter of the kernels whose name contains the
case's kernel pattern, plus derived ratios.

    python tools/pmc_summary.py <dir> [case=pattern ...]
"""
import collections
import csv
import glob
import os
import sys

DEFAULT = {"fwd1": "gemm_nt_8ph", "wgrad0_ring": "ring_tn_kernel",
           "wgrad0_old": "wgrad_tn_kernel", "wgrad1_ring": "ring_tn_kernel"}


def case_counters(d, pat):
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "g*", "*counter_collection.csv")):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (_, c), v in per.items():
            vals[c].append(v)
    return {c: sum(v) / len(v) for c, v in vals.items()}


def main(d, pairs):
    cases = dict(DEFAULT)
    cases.update(dict(p.split("=", 1) for p in pairs))
    for case in sorted(os.listdir(d)):
        if not os.path.isdir(os.path.join(d, case)):
            continue
        c = case_counters(os.path.join(d, case), cases.get(case, case))
        if not c:
            continue
        print(f"== {case}")
        for k in sorted(c):
            print(f"   {k:32s} {c[k]:.4g}")
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if k in c:
                    print(f"   {k + ' / WAVE_CYCLES':32s} {c[k] / wc:.3f}")
        g = c.get("GRBM_GUI_ACTIVE")
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            print(f"   {'MFMA busy / (GRBM/8 * 1024 SIMDs)':32s} {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (g / 8 * 1024):.3f}")
        if "SQ_LDS_BANK_CONFLICT" in c and "SQ_LDS_IDX_ACTIVE" in c:
            print(f"   {'LDS bank conflict / IDX_ACTIVE':32s} {c['SQ_LDS_BANK_CONFLICT'] / max(1, c['SQ_LDS_IDX_ACTIVE']):.3f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
