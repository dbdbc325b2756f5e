"""Summarise a rocprofv3 --pmc counter_collection.csv: per kernel, the sum of each counter over its
dispatches, plus the derived SQ fractions (wait / issue-stall / active of SQ_WAVE_CYCLES) and the LDS
bank-conflict share of LDS cycles."""
import collections
import csv
import sys


def main(path, top=12):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    calls = collections.Counter()
    with open(path) as f:
        for row in csv.DictReader(f):
            k = row.get("Kernel_Name", "?")
            tot[k][row["Counter_Name"]] += float(row["Counter_Value"])
            calls[(k, row["Counter_Name"])] += 1
    order = sorted(tot, key=lambda k: -tot[k].get("SQ_WAVE_CYCLES", 0.0))
    for k in order[:top]:
        c = tot[k]
        n = max(v for (kk, _), v in calls.items() if kk == k)
        wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        parts = [f"{k[:60]:60s} dispatches={n}"]
        for name in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if name in c:
                parts.append(f"{name[3:].lower()}={c[name] / wc:.2f}")
        if "SQ_LDS_IDX_ACTIVE" in c and c["SQ_LDS_IDX_ACTIVE"]:
            parts.append(f"lds_conflict/lds_active={c.get('SQ_LDS_BANK_CONFLICT', 0.0) / c['SQ_LDS_IDX_ACTIVE']:.2f}")
        for name, v in sorted(c.items()):
            if name not in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                parts.append(f"{name}={v / n:.4g}/disp")
        print("  ".join(parts))


def phases(path, kernel="k_cnn_train"):
    """Per-phase counters from scripts/cnn_phase_pmc.py: dispatches of `kernel` in launch order are the
    warm-up, then prefixes ending after phases 1..11, then the full kernel; consecutive differences."""
    rows = collections.defaultdict(dict)
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel in row.get("Kernel_Name", ""):
                rows[int(row["Dispatch_Id"])][row["Counter_Name"]] = rows[int(row["Dispatch_Id"])].get(
                    row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    ids = sorted(rows)[-13:]  # warm-up + 11 prefixes + full
    names = ["P0 load", "P1 conv1", "P2 conv2", "P3 fc1", "P4a fc2", "P4b loss", "P5 fc2bwd", "P6 fc1bwd",
             "P7a c2wgrad", "P7b c2dgrad", "P9 conv1wgrad", "rest"]
    prev = {}
    for i, d in enumerate(ids[1:]):
        c = rows[d]
        diff = {k: v - prev.get(k, 0.0) for k, v in c.items()}
        prev = c
        print(f"{names[i]:14s} " + "  ".join(f"{k[3:] if k.startswith('SQ_') else k}={v:.3g}" for k, v in sorted(diff.items())))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "--phases":
        phases(sys.argv[1])
    else:
        main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 12)
