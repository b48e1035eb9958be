"""Per-kernel-name mean counters from rocprofv3 --pmc CSVs (<dir>/g*/...counter_collection.csv),
kernels whose name contains one of the given substrings, with MFMA busy and wait ratios.

    python tools/pmc_by_kernel.py <dir> [substring ...]
"""
import collections
import csv
import glob
import os
import sys


def main(d, pats):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "g*", "**", "*counter_collection.csv"), recursive=True):
        per = collections.defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if pats and not any(p in k for p in pats):
                continue
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = k
        for (di, c), v in per.items():
            vals[names[di]][c].append(v)
    for k, cs in sorted(vals.items()):
        c = {n: sum(v) / len(v) for n, v in cs.items()}
        print(f"== {k[:110]}  (dispatches {max(len(v) for v in cs.values())})")
        for n in sorted(c):
            print(f"   {n:28s} {c[n]:.4g}")
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if n in c:
                    print(f"   {n + ' / WAVE_CYCLES':40s} {c[n] / wc:.3f}")
        if "SQ_BUSY_CYCLES" in c and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            # SQ_BUSY_CYCLES sums quad-cycles over the SEs; MFMA busy counts cycles per SIMD
            print(f"   {'MFMA busy / (SQ_BUSY_CYCLES * 4 / 32 SE * 1024 SIMD)':40s} "
                  f"{c['SQ_VALU_MFMA_BUSY_CYCLES'] / (c['SQ_BUSY_CYCLES'] * 4 / 32 * 1024):.3f}")
        if "SQ_LDS_BANK_CONFLICT" in c and "SQ_LDS_IDX_ACTIVE" in c:
            print(f"   {'LDS bank conflict / IDX_ACTIVE':40s} {c['SQ_LDS_BANK_CONFLICT'] / max(1, c['SQ_LDS_IDX_ACTIVE']):.3f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
