"""Per-kernel register / scratch / occupancy table from hipcc -Rpass-analysis=kernel-resource-usage output.

    hipcc ... -Rpass-analysis=kernel-resource-usage 2> ra.txt; python scripts/kernel_regs.py ra.txt [filter]
"""
import re
import subprocess
import sys


def parse(path):
    rows, d = [], {}
    for line in open(path):
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            if d:
                rows.append(d)
            d = {"name": m.group(1)}
            continue
        for k, pat in [("vgpr", r"VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("sgpr", r"SGPRs: (\d+)"),
                       ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"), ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"),
                       ("lds", r"LDS Size \[bytes/block\]: (\d+)")]:
            m = re.search(pat, line)
            if m:
                d[k] = int(m.group(1))
    if d:
        rows.append(d)
    names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                           text=True).stdout.splitlines()
    for r, n in zip(rows, names):
        r["demangled"] = n.replace("pde::(anonymous namespace)::", "").split("(pde::")[0].split("(unsigned")[0]
    return rows


if __name__ == "__main__":
    rows = parse(sys.argv[1])
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    print("| kernel | VGPR | AGPR | SGPR | scratch B/lane | waves/SIMD | LDS B |")
    print("|---|---|---|---|---|---|---|")
    for r in rows:
        if flt in r["demangled"]:
            print(f"| `{r['demangled']}` | {r.get('vgpr')} | {r.get('agpr')} | {r.get('sgpr')} | {r.get('scratch')} | "
                  f"{r.get('occ')} | {r.get('lds')} |")
