"""Summarise a ``rocprofv3 --marker-trace`` database: the roctx ranges of one top-level range
(default ``shifu.train``), time per range family (digits stripped: gbdt.level3.partition ->
gbdt.levelN.partition) and the fraction of the top range's wall time covered by named child ranges.

    python tools/marker_summary.py <results.db> [--top shifu.train] [--json out.json]
"""
import argparse
import json
import re
import sqlite3
from collections import defaultdict


def union_len(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", default="shifu.train")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    rows = []
    for name, s, e, cat, ext in con.execute("select name, start, end, category, extdata from regions"):
        # roctx ranges: the region is the API call (roctxThreadRangeA), the range text its message
        try:
            msg = json.loads(ext or "{}").get("message")
        except ValueError:
            msg = None
        rows.append((msg or name, s, e, cat))
    tops = [(s, e) for n, s, e, _ in rows if n == a.top]
    if not tops:
        names = sorted({n for n, *_ in rows})
        raise SystemExit(f"no range named {a.top}; ranges seen: {names[:40]}")
    t0, t1 = min(s for s, _ in tops), max(e for _, e in tops)
    wall = t1 - t0
    fam = defaultdict(lambda: [0, 0])
    child = []
    for n, s, e, _ in rows:
        if n == a.top or e <= t0 or s >= t1 or not (n.startswith("gbdt.") or n.startswith("nn.") or
                                                   n.startswith("train.") or n.startswith("stats.") or
                                                   n.startswith("eval.") or n.startswith("varsel.")):
            continue
        k = re.sub(r"\d+", "N", n)
        fam[k][0] += e - s
        fam[k][1] += 1
        child.append((max(s, t0), min(e, t1)))
    # leaf families (a tree range contains its level ranges): coverage of the union of all children
    cov = union_len(child) / wall if wall else 0.0
    leaf = [(max(s, t0), min(e, t1)) for n, s, e, _ in rows
            if re.match(r"gbdt\.level\d+\.|gbdt\.hist_allreduce|gbdt\.apply_residual|train\.|nn\.|stats\.|eval\.|varsel\.", n)
            and e > t0 and s < t1]
    leaf_cov = union_len(leaf) / wall if wall else 0.0
    out = {"top_range": a.top, "wall_ms": wall / 1e6, "covered_by_child_ranges": round(cov, 4),
           "covered_by_leaf_phase_ranges": round(leaf_cov, 4),
           "families_ms": {k: {"ms": round(v[0] / 1e6, 3), "calls": v[1]}
                           for k, v in sorted(fam.items(), key=lambda kv: -kv[1][0])}}
    print(json.dumps(out, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
