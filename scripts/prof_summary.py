#!/usr/bin/env python3
"""Summarise a rocprofv3 ``*_kernel_stats.csv``: top kernels by total time, per-step figures.

    python scripts/prof_summary.py <kernel_stats.csv> [steps_traced] [--md]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else None
    md = "--md" in sys.argv
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    if md:
        print("| kernel | calls | avg us | total ms | % |")
        print("|---|---|---|---|---|")
    for r in rows[:30]:
        name = r["Name"].replace("pde::(anonymous namespace)::", "").replace("|", "/")
        name = name[:100]
        t = float(r["TotalDurationNs"]) / 1e6
        if md:
            print(f"| `{name}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | {t:.2f} | {float(r['Percentage']):.1f} |")
        else:
            print(f"{t:9.2f}ms {r['Calls']:>6} {float(r['AverageNs']) / 1e3:8.1f}us {float(r['Percentage']):5.1f}% {name}")
    msg = f"total GPU kernel time {tot / 1e6:.2f} ms"
    if steps:
        msg += f" over ~{steps} steps = {tot / 1e6 / steps:.3f} ms/step"
    print(msg)


if __name__ == "__main__":
    main()
