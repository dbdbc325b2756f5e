#!/usr/bin/env python3
"""Per-step kernel table of a hipGraph bench trace (rocprofv3 ``--kernel-trace`` csv): kernels per step,
average duration, us per step and share -- over the last third of the trace, with the step count taken from
the optimizer kernel (one ``k_optim`` launch per training step).

    python scripts/graph_kernel_table.py <kernel_trace.csv> [--title T] [--step-kernel k_optim]
"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--title", default="")
    ap.add_argument("--step-kernel", default="k_optim")
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    ks = ks[-len(ks) // 3:]
    steps = sum(1 for _, _, n in ks if args.step_kernel in n) or 1
    span = ks[-1][1] - ks[0][0]
    agg = defaultdict(lambda: [0, 0])
    for s, e, n in ks:
        agg[n][0] += 1
        agg[n][1] += e - s
    busy = sum(v[1] for v in agg.values())
    print(f"# {args.title}\n")
    print(f"last third of the trace: {len(ks)} kernels, {steps} optimizer steps -> {len(ks) / steps:.0f} kernels per "
          f"step; span {span / 1e3:.0f} us -> {span / 1e3 / steps:.0f} us per step (kernel busy "
          f"{busy / 1e3 / steps:.0f} us)\n")
    print("| kernel | calls/step | avg us | us/step | % |")
    print("|---|---|---|---|---|")
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:30]:
        name = n.replace("pde::(anonymous namespace)::", "").replace("|", "/")[:100]
        print(f"| `{name}` | {c / steps:.1f} | {t / c / 1e3:.2f} | {t / steps / 1e3:.1f} | {100 * t / busy:.1f} |")


if __name__ == "__main__":
    main()
