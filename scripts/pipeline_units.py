#!/usr/bin/env python3
"""Predicted 2-GPU pipeline step of the ResNet-50 split (BASELINE configs 3/4) per pipeline-unit size, from the
measured single-stage times (bench.py --model resnet50_stage --batch 8g --mb-group g).

A batch of 32 images in micro-batches of m = 8 (the reference's split size) is U = 4 / g units of g micro-batches.
With stage times t1(g), t2(g) per unit (forward + backward + SGD of the unit, P2P excluded), a GPipe or 1F1B
schedule over 2 stages costs about (U + 1) * max(t1, t2) per step (fill + drain = one extra unit slot); the
2-GPU throughput is 32 / that step.  1F1B has the same bubble as GPipe at 2 stages (it only bounds the number of
activations in flight), so both predictions are equal here.

    python scripts/pipeline_units.py r4g_stages.jsonl
"""
import json
import sys


def main():
    recs = [json.loads(ln) for ln in open(sys.argv[1]) if ln.strip()]
    t = {}
    for r in recs:
        c = r["config"]
        t[(c["stage"], c["mb_per_unit"])] = r["ms_per_step"]
    print("| micro-batches per unit g | units per step U | stage 1 ms/unit | stage 2 ms/unit | predicted GPipe / 1F1B "
          "2-GPU step ms | img/s (2 GPUs) |")
    print("|---|---|---|---|---|---|")
    best = None
    for g in sorted({k[1] for k in t}):
        if (1, g) not in t or (2, g) not in t:
            continue
        U = 4 // g
        step = (U + 1) * max(t[(1, g)], t[(2, g)])
        ips = 32 / step * 1e3
        best = max(best or (0, 0), (ips, g))
        print(f"| {g} | {U} | {t[(1, g)]:.3f} | {t[(2, g)]:.3f} | {step:.3f} | {ips:.0f} |")
    if best:
        print(f"\nbest unit: g = {best[1]} ({best[0]:.0f} img/s predicted on 2 GPUs)")


if __name__ == "__main__":
    main()
