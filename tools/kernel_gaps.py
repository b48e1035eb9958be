"""Per-tree GPU timeline from a rocprofv3 kernel trace of the GBDT bench: for every boosting
round (the interval between two gbdt_residual_kernel launches) the wall span, the busy time (union
of kernel intervals), the idle gaps between kernels ("host gaps": the GPU waiting on the host) and
the time per kernel family.

    python tools/kernel_gaps.py <run_kernel_trace.csv> [--skip 1] [--json out.json]
"""
import argparse
import csv
import json
import re
from collections import defaultdict


def family(name: str) -> str:
    m = re.search(r"(gbdt_\w+?_kernel|strip_\w+?_kernel|\w+_kernel)", name)
    if m:
        return m.group(1)
    return name.split("(")[0][-60:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="gbdt_residual_kernel", help="kernel that ends a round")
    ap.add_argument("--skip", type=int, default=1, help="rounds to drop at the start (warm-up)")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    ks = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), family(r["Kernel_Name"])))
    ks.sort()
    ends = [i for i, k in enumerate(ks) if k[2] == a.marker]
    rounds = []
    for j in range(1, len(ends)):
        seg = ks[ends[j - 1] + 1: ends[j] + 1]
        if not seg:
            continue
        t0, t1 = ks[ends[j - 1]][1], seg[-1][1]
        busy, cur_s, cur_e = 0, None, None
        gaps = []
        fam = defaultdict(float)
        for s, e, nm in seg:
            fam[nm] += (e - s) / 1e6
            if cur_e is None:
                gaps.append(max(0, s - t0))
                cur_s, cur_e = s, e
            elif s > cur_e:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        span = t1 - t0
        big = sorted(gaps, reverse=True)[:8]
        rounds.append({"round": j, "span_ms": span / 1e6, "busy_ms": busy / 1e6, "gap_ms": (span - busy) / 1e6,
                       "n_kernels": len(seg), "largest_gaps_us": [round(g / 1e3, 1) for g in big],
                       "kernels_ms": {k: round(v, 3) for k, v in sorted(fam.items(), key=lambda x: -x[1])}})
    rounds = rounds[a.skip:]
    for r in rounds:
        print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items() if k != "kernels_ms"}))
    if rounds:
        agg = defaultdict(float)
        for r in rounds:
            for k, v in r["kernels_ms"].items():
                agg[k] += v / len(rounds)
        mean = {"rounds": len(rounds), "span_ms": sum(r["span_ms"] for r in rounds) / len(rounds),
                "busy_ms": sum(r["busy_ms"] for r in rounds) / len(rounds),
                "gap_ms": sum(r["gap_ms"] for r in rounds) / len(rounds),
                "kernels_ms": {k: round(v, 3) for k, v in sorted(agg.items(), key=lambda x: -x[1])}}
        print(json.dumps({"mean": mean}))
        if a.json:
            with open(a.json, "w") as f:
                json.dump({"rounds": rounds, "mean": mean}, f, indent=1)


if __name__ == "__main__":
    main()
