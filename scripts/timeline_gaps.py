#!/usr/bin/env python3
"""Busy time vs wall span of the GPU timeline from a rocprofv3 ``*_kernel_trace.csv``.

    python scripts/timeline_gaps.py <kernel_trace.csv> [--last N] [--seq M]

Looks at the last N kernels (default: all), reports the span first-start -> last-end, the summed
kernel time and the idle fraction, the idle gap distribution, and (``--seq M``) the last M kernels
in launch order with their durations and the gap before each -- the per-step kernel sequence of a
hipGraph replay.
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=0)
    ap.add_argument("--seq", type=int, default=0)
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    if args.last:
        ks = ks[-args.last:]
    span = ks[-1][1] - ks[0][0]
    busy = 0
    gaps = []
    cur_end = ks[0][0]
    for s, e, _ in ks:
        if s > cur_end:
            gaps.append(s - cur_end)
        busy += max(0, e - max(s, cur_end))
        cur_end = max(cur_end, e)
    gaps.sort()
    print(f"kernels {len(ks)}  span {span / 1e3:.1f} us  busy {busy / 1e3:.1f} us  idle {100 * (1 - busy / span):.1f}%")
    if gaps:
        n = len(gaps)
        print(f"gaps: n={n} median {gaps[n // 2] / 1e3:.2f} us  p90 {gaps[int(n * 0.9)] / 1e3:.2f} us  "
              f"max {gaps[-1] / 1e3:.2f} us  total {sum(gaps) / 1e3:.1f} us")
    if args.seq:
        prev = None
        for s, e, name in ks[-args.seq:]:
            gap = (s - prev) / 1e3 if prev is not None else 0.0
            print(f"  +{gap:6.2f} us  {(e - s) / 1e3:7.2f} us  {name.replace('pde::(anonymous namespace)::', '')[:90]}")
            prev = e


if __name__ == "__main__":
    main()
