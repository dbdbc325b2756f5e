"""Join a PDE_GEMM_LOG=1 stderr log with a rocprofv3 kernel trace of the same eager run: per GEMM launch its
shape (M, N, K, operand kinds, tile, split) and measured duration -> a table of the GEMMs of one step sorted by
time, with achieved TFLOP/s.

    python scripts/gemm_shape_table.py gemm.log kernel_trace.csv --steps 3 --title "resnet50 b32"
"""
import argparse
import collections
import csv
import re

LINE = re.compile(r"\[gemm\] (\S+) M=(\d+) N=(\d+) K=(\d+) akind=(\d+) bkind=(\d+) tile=(\d+)x(\d+) tiles=(\d+) "
                  r"split=(\d+) gflop=([\d.]+)")


def launches(log_path):
    """One entry per kernel launch: a list of (what, M, N, K, ak, bk, tile, tiles, split, gflop) problems."""
    out, pending = [], None
    for ln in open(log_path):
        m = LINE.search(ln)
        if not m:
            continue
        what = m.group(1)
        prob = (what, int(m.group(2)), int(m.group(3)), int(m.group(4)), int(m.group(5)), int(m.group(6)),
                f"{m.group(7)}x{m.group(8)}", int(m.group(9)), int(m.group(10)), float(m.group(11)))
        if what.endswith(".0"):
            pending = [prob]
        elif what.endswith(".1"):
            out.append((pending or []) + [prob])
            pending = None
        else:
            out.append([prob])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("log")
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=1, help="steps in the run (the table shows the last one)")
    ap.add_argument("--title", default="GEMM launches")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    kern = [r for r in rows if ("gemm" in r["Kernel_Name"] and "reduce" not in r["Kernel_Name"])]
    lau = launches(a.log)
    n = min(len(kern), len(lau))
    if len(kern) != len(lau):
        print(f"<!-- warning: {len(kern)} GEMM kernels in the trace, {len(lau)} logged launches; joined the last {n} -->")
    kern, lau = kern[-n:], lau[-n:]
    per_step = n // max(1, a.steps)
    kern, lau = kern[-per_step:], lau[-per_step:]
    agg = collections.OrderedDict()
    tot_us = tot_gf = 0.0
    for r, probs in zip(kern, lau):
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
        gf = sum(p[9] for p in probs)
        key = " + ".join(f"{p[0]} {p[1]}x{p[2]}x{p[3]} k{p[4]}{p[5]} {p[6]} t{p[7]} s{p[8]}" for p in probs)
        e = agg.setdefault(key, [0, 0.0, 0.0])
        e[0] += 1
        e[1] += us
        e[2] += gf
        tot_us += us
        tot_gf += gf
    print(f"# {a.title}\n")
    print(f"{per_step} GEMM launches per step, {tot_us:.0f} us traced, {tot_gf:.1f} GFLOP -> "
          f"{tot_gf / max(tot_us, 1e-9) * 1e3:.1f} TFLOP/s over the GEMM time\n")
    print("| launch (problem: MxNxK, operand kinds, tile, tiles, split) | n | us/step | avg us | TFLOP/s |")
    print("|---|---|---|---|---|")
    for key, (cnt, us, gf) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"| `{key}` | {cnt} | {us:.1f} | {us / cnt:.2f} | {gf / us * 1e3:.1f} |")


if __name__ == "__main__":
    main()
