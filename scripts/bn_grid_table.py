"""BatchNorm kernels of a rocprofv3 kernel trace grouped by (kernel, grid): calls per step and average time
(last third of the trace).  python scripts/bn_grid_table.py kernel_trace.csv [--steps-per-third N]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[len(rows) * 2 // 3:]
steps = max(1, sum(1 for r in rows if "k_optim" in r["Kernel_Name"]))
d = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    if "k_bn" in n:
        blocks = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
        key = (n.split("(")[0].replace("void ", "").replace("pde::(anonymous namespace)::", ""), blocks,
               int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
        d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
tot = 0.0
print("| kernel | grid (x, y, z) | calls/step | avg us | us/step |\n|---|---|---|---|---|")
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    tot += sum(v) / steps
    print(f"| `{k[0]}` | {k[1]} x {k[2]} x {k[3]} | {len(v) / steps:.1f} | {sum(v) / len(v):.2f} | {sum(v) / steps:.1f} |")
print(f"\nBatchNorm total {tot:.0f} us/step over {steps} steps")
