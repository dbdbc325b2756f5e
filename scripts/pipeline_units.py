#!/usr/bin/env python3
"""Predicted 2-GPU pipeline step of the ResNet-50 split (BASELINE configs 3/4) per pipeline-unit size, from the
measured single-stage times (bench.py --model resnet50_stage --batch 8g --mb-group g) and the measured whole-model
1-GPU step (bench.py --model resnet50), side by side.

A batch of 32 images in micro-batches of m = 8 (the reference's split size) is U = 4 / g units of g micro-batches.
With stage times t1(g), t2(g) per unit (forward + backward + SGD of the unit) and p = the P2P time of one unit's
activation (or gradient) over xGMI, a 2-stage GPipe / 1F1B step is

    step(U) = t1 + t2 + (U - 1) * max(t1, t2) + 2 p

(the first unit crosses both stages serially -- for U = 1 there is no overlap at all -- and every further unit
adds one slot of the slower stage; the activation and the gradient of the last unit are on the critical path).
1F1B has the same bubble as GPipe at 2 stages.  p = bytes / bw with the unit's bf16 activation
(g * 8 images x 512 x 16 x 16) and bw = --p2p-gbs (default 50 GB/s, one xGMI link as the P2P ring measured it).

    python scripts/pipeline_units.py stages.jsonl [--one-gpu bench.jsonl] [--p2p-gbs 50]
"""
import argparse
import json


def predict(t1: float, t2: float, units: int, p_ms: float) -> float:
    """Predicted 2-stage pipeline step (ms) for `units` units with per-unit stage times t1, t2 (ms)."""
    return t1 + t2 + (units - 1) * max(t1, t2) + 2 * p_ms


def table(recs, one_gpu_img_s=None, p2p_gbs=50.0, batch=32, split=8):
    t = {}
    for r in recs:
        c = r["config"]
        if "stage" in c and "mb_per_unit" in c:
            t[(c["stage"], c["mb_per_unit"])] = r["ms_per_step"]
    rows, best = [], None
    for g in sorted({k[1] for k in t}):
        if (1, g) not in t or (2, g) not in t:
            continue
        units = batch // (split * g)
        p_ms = g * split * 512 * 16 * 16 * 2 / (p2p_gbs * 1e9) * 1e3
        step = predict(t[(1, g)], t[(2, g)], units, p_ms)
        ips = batch / step * 1e3
        rows.append({"mb_per_unit": g, "units": units, "t1_ms": t[(1, g)], "t2_ms": t[(2, g)], "p2p_ms": round(p_ms, 4),
                     "step_ms": round(step, 4), "predicted_2gpu_img_s": round(ips, 1)})
        if best is None or ips > best["predicted_2gpu_img_s"]:
            best = rows[-1]
    return {"rows": rows, "best": best, "one_gpu_img_s": one_gpu_img_s}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stages")
    ap.add_argument("--one-gpu", help="a bench.py --model resnet50 JSON line (file) for the 1-GPU whole-model rate")
    ap.add_argument("--p2p-gbs", type=float, default=50.0)
    a = ap.parse_args()
    recs = [json.loads(ln) for ln in open(a.stages) if ln.strip().startswith("{")]
    one = None
    if a.one_gpu:
        for ln in open(a.one_gpu):
            if ln.strip().startswith("{"):
                r = json.loads(ln)
                if r["config"]["model"].startswith("resnet50") and "stage" not in r["config"]:
                    one = r["value"]
    res = table(recs, one, a.p2p_gbs)
    print("| micro-batches per unit g | units U | stage 1 ms/unit | stage 2 ms/unit | P2P ms | predicted 2-GPU step ms "
          "| predicted img/s (2 GPUs) |")
    print("|---|---|---|---|---|---|---|")
    for r in res["rows"]:
        print(f"| {r['mb_per_unit']} | {r['units']} | {r['t1_ms']:.3f} | {r['t2_ms']:.3f} | {r['p2p_ms']:.3f} | "
              f"{r['step_ms']:.3f} | {r['predicted_2gpu_img_s']:.0f} |")
    if res["best"]:
        print(f"\nbest unit: g = {res['best']['mb_per_unit']} ({res['best']['predicted_2gpu_img_s']:.0f} img/s predicted "
              f"on 2 GPUs)" + (f"; 1 GPU whole model: {one:.0f} img/s" if one else ""))


if __name__ == "__main__":
    main()
