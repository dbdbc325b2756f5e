"""Join a PDE_GEMM_LOG=1 stderr log with a rocprofv3 --pmc counter_collection.csv of the same eager run: per GEMM
problem shape (M, N, K, operand kinds, tile, split), the SQ counters summed over its dispatches of the last step,
plus the resources rocprofv3 records per dispatch (VGPRs, AGPRs, scratch bytes per lane, LDS).

    python scripts/gemm_pmc_table.py gemm.log counter_collection.csv [more.csv ...] --steps 3 --top 5

Several csv files (one per counter pass of the SAME command) are merged by dispatch order."""
import argparse
import collections
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_shape_table import launches  # noqa: E402


def dispatches(path):
    """[(kernel name, {counter: value}, resources)] of the GEMM dispatches in dispatch order."""
    by = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name", "")
        if "gemm" not in name or "reduce" in name:
            continue
        key = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)
        d = by.setdefault(key, [name, {}, {k: r.get(k) for k in ("VGPR_Count", "Accum_VGPR_Count", "Scratch_Size",
                                                                  "LDS_Block_Size", "Grid_Size", "Workgroup_Size")}])
        d[1][r["Counter_Name"]] = d[1].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [by[k] for k in sorted(by)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("log")
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--top", type=int, default=5)
    ap.add_argument("--title", default="GEMM SQ counters")
    a = ap.parse_args()
    passes = [dispatches(p) for p in a.csv]
    n = min(len(p) for p in passes)
    merged = []
    for i in range(n):
        name, ctr, res = passes[0][len(passes[0]) - n + i]
        c = dict(ctr)
        for p in passes[1:]:
            c.update(p[len(p) - n + i][1])
        merged.append((name, c, res))
    lau = launches(a.log)
    m = min(n, len(lau))
    merged, lau = merged[-m:], lau[-m:]
    per_step = m // max(1, a.steps)
    merged, lau = merged[-per_step:], lau[-per_step:]
    agg = collections.OrderedDict()
    for (name, c, res), probs in zip(merged, lau):
        key = " + ".join(f"{p[0]} {p[1]}x{p[2]}x{p[3]} k{p[4]}{p[5]} {p[6]} t{p[7]} s{p[8]}" for p in probs)
        e = agg.setdefault(key, {"n": 0, "ctr": collections.Counter(), "res": res, "kernel": name})
        e["n"] += 1
        e["ctr"].update(c)
    order = sorted(agg.items(), key=lambda kv: -kv[1]["ctr"].get("SQ_WAVE_CYCLES", kv[1]["ctr"].get("SQ_BUSY_CYCLES", 0)))
    print(f"# {a.title}\n")
    print(f"{per_step} GEMM dispatches in the last step; top {a.top} problems by SQ_WAVE_CYCLES.  Ratios: "
          "mfma/busy = SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CYCLES; wait_any / active_inst = share of wave-cycles waiting "
          "on anything / issuing; lds_wait = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES; conflict = SQ_LDS_BANK_CONFLICT / "
          "SQ_LDS_IDX_ACTIVE.  Resources as rocprofv3 records them per dispatch (arch VGPRs, AGPRs, scratch B/lane, "
          "LDS B).\n")
    print("| problem | n | kernel | vgpr/agpr | scratch B | lds B | mfma/busy | wait_any | active_inst | lds_wait | "
          "conflict | counters per dispatch |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    for key, e in order[:a.top]:
        c, k = e["ctr"], e["n"]
        wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0

        def r(x, y):
            return f"{c.get(x, 0.0) / y:.3f}" if y else "-"
        res = e["res"]
        per = ", ".join(f"{nm}={v / k:.3g}" for nm, v in sorted(c.items()))
        print(f"| `{key}` | {k} | `{e['kernel'][:40]}` | {res.get('VGPR_Count')}/{res.get('Accum_VGPR_Count')} | "
              f"{res.get('Scratch_Size')} | {res.get('LDS_Block_Size')} | {r('SQ_VALU_MFMA_BUSY_CYCLES', c.get('SQ_BUSY_CYCLES', 0))} | "
              f"{r('SQ_WAIT_ANY', wc)} | {r('SQ_ACTIVE_INST_ANY', wc)} | {r('SQ_WAIT_INST_LDS', wc)} | "
              f"{r('SQ_LDS_BANK_CONFLICT', c.get('SQ_LDS_IDX_ACTIVE', 0))} | {per} |")


if __name__ == "__main__":
    main()
