"""One-launch BatchNorm kernel durations of a rocprofv3 kernel trace, by direction and grid (row chunks x channel
groups x groups): median us over the last third of the trace.

    python scripts/bn_grid_table.py kernel_trace.csv"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows[len(rows) * 2 // 3:]:
    for tag in ("k_bn_fwd_fused", "k_bn_bwd_fused"):
        if tag in r["Kernel_Name"]:
            key = (tag, int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
            d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
print("| kernel | grid (row chunks, channel groups, groups) | launches | median us | sum us |")
print("|---|---|---|---|---|")
for k, v in sorted(d.items()):
    v.sort()
    print(f"| `{k[0]}` | {k[1]} x {k[2]} x {k[3]} | {len(v)} | {v[len(v) // 2]:.2f} | {sum(v):.0f} |")
