"""Summarise a rocprofv3 kernel_trace csv: per (kernel, grid) count / mean / min / max ms."""
import collections, csv, sys
r = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for x in r:
    k = (x['Kernel_Name'][:60], int(x['Grid_Size_X']) // max(1, int(x['Workgroup_Size_X'])), x['VGPR_Count'], x['Accum_VGPR_Count'], x['SGPR_Count'])
    d[k].append((int(x['End_Timestamp']) - int(x['Start_Timestamp'])) / 1e6)
tot = sum(sum(v) for v in d.values())
print(f"{'kernel':60s} {'blocks':>8s} vgpr agpr sgpr {'n':>4s} {'mean_ms':>8s} {'min':>7s} {'max':>7s} {'%':>5s}")
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    if sum(v) / tot < 0.001: continue
    print(f"{k[0]:60s} {k[1]:8d} {k[2]:>4s} {k[3]:>4s} {k[4]:>4s} {len(v):4d} {sum(v)/len(v):8.3f} {min(v):7.3f} {max(v):7.3f} {100*sum(v)/tot:5.1f}")
