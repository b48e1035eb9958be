"""Per-kernel summary of rocprofv3 --pmc CSVs (layout <dir>/g*/.../*counter_collection.csv, one
counter group per g* run, e.g. tools/pmc_mlp.sh): per kernel name, the mean per-dispatch value of
every counter plus derived ratios (MFMA busy share, LDS conflict rate, HBM bytes per dispatch).

    python tools/pmc_kernels.py <dir> [--min-calls N]
"""
import collections
import csv
import glob
import os
import re
import sys


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)            # drop the argument list
    return re.sub(r"^void ", "", name)[:60]


def collect(d):
    per_kernel = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "g*", "**", "*counter_collection.csv"), recursive=True):
        disp = collections.defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            key = (r["Dispatch_Id"], r["Counter_Name"])
            disp[key] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = short(r["Kernel_Name"])
        for (did, c), v in disp.items():
            per_kernel[names[did]][c].append(v)
    return per_kernel


def main(d, min_calls=1):
    pk = collect(d)
    for k in sorted(pk):
        c = {n: sum(v) / len(v) for n, v in pk[k].items()}
        calls = max(len(v) for v in pk[k].values())
        if calls < min_calls:
            continue
        print(f"== {k}  ({calls} dispatch samples)")
        for n in sorted(c):
            print(f"   {n:28s} {c[n]:.4g}")
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if n in c:
                    print(f"   {n + ' / WAVE_CYCLES':28s} {c[n] / wc:.3f}")
        if "SQ_BUSY_CYCLES" in c and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            # MFMA busy is summed over the SIMDs (4 per CU, 256 CUs); SQ_BUSY_CYCLES over the 32 SEs
            print(f"   {'MFMA busy / (BUSY/32*1024)':28s} "
                  f"{c['SQ_VALU_MFMA_BUSY_CYCLES'] / (c['SQ_BUSY_CYCLES'] / 32 * 1024):.3f}")
        if "SQ_LDS_BANK_CONFLICT" in c and "SQ_LDS_IDX_ACTIVE" in c:
            print(f"   {'LDS conflict / IDX_ACTIVE':28s} {c['SQ_LDS_BANK_CONFLICT'] / max(1, c['SQ_LDS_IDX_ACTIVE']):.3f}")
        if "FETCH_SIZE" in c:
            print(f"   {'HBM fetch MB':28s} {c['FETCH_SIZE'] / 1024:.1f}")
        if "WRITE_SIZE" in c:
            print(f"   {'HBM write MB':28s} {c['WRITE_SIZE'] / 1024:.1f}")


if __name__ == "__main__":
    args = sys.argv[1:]
    mc = 1
    if "--min-calls" in args:
        i = args.index("--min-calls")
        mc = int(args[i + 1])
        del args[i:i + 2]
    main(args[0], mc)
