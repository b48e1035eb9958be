"""Summarise a rocprofv3 kernel trace: per (kernel, grid) count / mean / min / max ms.

    python tools/prof_summary.py <kernel_trace.csv | results.db>

Accepts the csv written by ``--output-format csv`` and the rocpd SQLite database that
rocprofv3 (ROCm 7.x) writes by default.
"""
import collections
import csv
import sqlite3
import sys


def rows_from_csv(path):
    for x in csv.DictReader(open(path)):
        blocks = int(x['Grid_Size_X']) // max(1, int(x['Workgroup_Size_X']))
        yield (x['Kernel_Name'], blocks, x['VGPR_Count'], x['Accum_VGPR_Count'], x['SGPR_Count'],
               (int(x['End_Timestamp']) - int(x['Start_Timestamp'])) / 1e6)


def rows_from_db(path):
    c = sqlite3.connect(path)
    q = ("select name, grid_x, workgroup_x, vgpr_count, accum_vgpr_count, sgpr_count, duration "
         "from kernels")
    for name, gx, wx, v, a, s, d in c.execute(q):
        yield (name, int(gx) // max(1, int(wx)), str(v), str(a), str(s), d / 1e6)


def main(path):
    src = rows_from_db(path) if path.endswith(".db") else rows_from_csv(path)
    d = collections.defaultdict(list)
    for name, blocks, v, a, s, ms in src:
        d[(name[:60], blocks, v, a, s)].append(ms)
    tot = sum(sum(v) for v in d.values())
    print(f"{'kernel':60s} {'blocks':>8s} vgpr agpr sgpr {'n':>4s} {'mean_ms':>8s} {'min':>7s} {'max':>7s} {'%':>5s}")
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        if sum(v) / tot < 0.001:
            continue
        print(f"{k[0]:60s} {k[1]:8d} {k[2]:>4s} {k[3]:>4s} {k[4]:>4s} {len(v):4d} {sum(v)/len(v):8.3f} "
              f"{min(v):7.3f} {max(v):7.3f} {100*sum(v)/tot:5.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
