"""Summarise a rocprofv3 --pmc counter_collection.csv per kernel family (sums over dispatches)."""
import csv
import json
import re
import sys
from collections import defaultdict

path = sys.argv[1]
agg = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(set)
with open(path) as f:
    for r in csv.DictReader(f):
        name = r.get("Kernel_Name", "")
        m = re.search(r"(gbdt_\w+?_kernel(?:<[^>]*>)?|strip_\w+?_kernel(?:<[^>]*>)?|ring_\w+?_kernel(?:<[^>]*>)?)", name)
        fam = m.group(1) if m else "other"
        agg[fam][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[fam].add(r.get("Dispatch_Id", ""))
out = {k: {"dispatches": len(cnt[k]), **{c: v for c, v in sorted(d.items())}} for k, d in agg.items() if k != "other"}
print(json.dumps(out, indent=1))
