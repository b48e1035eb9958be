"""H2D / kernel overlap from a rocprofv3 --kernel-trace --memory-copy-trace database.

    python tools/overlap_summary.py gpurun_out/<dir>/<name>_results.db

Reports total host-to-device copy time, total kernel busy time, the wall span, and the time during
which a copy and a kernel were active together (interval intersection of the two unions)."""
import sqlite3
import sys


def union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def inter(u, v):
    i = j = 0
    tot = 0
    while i < len(u) and j < len(v):
        a, b = max(u[i][0], v[j][0]), min(u[i][1], v[j][1])
        if a < b:
            tot += b - a
        if u[i][1] < v[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main(db):
    con = sqlite3.connect(db)
    cols = [r[1] for r in con.execute("pragma table_info(rocpd_memory_copy)")]
    kind = "name" if "name" in cols else None
    rows = con.execute("select start, end, size" + (", name" if kind else "") + " from rocpd_memory_copy").fetchall()
    h2d = [(r[0], r[1]) for r in rows if not kind or "HOST_TO_DEVICE" in str(r[3]).upper()]
    nbytes = sum(r[2] for r in rows if not kind or "HOST_TO_DEVICE" in str(r[3]).upper())
    ks = [(r[0], r[1]) for r in con.execute("select start, end from rocpd_kernel_dispatch")]
    uc, uk = union(h2d), union(ks)
    span = (max([b for _, b in uc + uk]) - min([a for a, _ in uc + uk])) / 1e9
    tc, tk = sum(b - a for a, b in uc) / 1e9, sum(b - a for a, b in uk) / 1e9
    ov = inter(uc, uk) / 1e9
    print(f"h2d copies: {len(h2d)}  {nbytes / 1e9:.1f} GB  busy {tc:.3f} s  ({nbytes / 1e9 / max(tc, 1e-9):.1f} GB/s)")
    print(f"kernels:    {len(ks)}  busy {tk:.3f} s")
    print(f"wall span:  {span:.3f} s   copy/kernel overlap {ov:.3f} s = {100 * ov / max(tc, 1e-9):.0f}% of copy time")


if __name__ == "__main__":
    main(sys.argv[1])
