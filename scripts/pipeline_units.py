#!/usr/bin/env python3
"""Predicted 2-GPU pipeline step of the ResNet-50 split (BASELINE configs 3/4) per pipeline-unit size, from the
measured single-stage times (bench.py --model resnet50_stage --stage s --batch 8g --mb-group g) and the measured
whole-model 1-GPU step (bench.py --model resnet50), side by side.

A batch of 32 images in micro-batches of m = 8 (the reference's split size) is U = 4 / g units of g micro-batches.
Each stage record carries its captured step's phases (fwd / bwd / opt device ms).  With c_s = fwd + bwd of one
unit on stage s, o_1 = stage 1's optimiser step and p = the P2P time of one unit's activation (or gradient) over
xGMI, a 2-stage GPipe / 1F1B step is

    step(U) = c1 + c2 + (U - 1) * max(c1, c2) + o1 + 2 p

The first unit crosses both stages serially -- for U = 1 there is no overlap at all, step = c1 + c2 + o1 + 2p --
and every further unit adds one slot of the slower stage.  The activation and the gradient of the last unit are on
the critical path, and so is stage 1's optimiser step (its last backward is the last of the step; stage 2's update
overlaps it).  1F1B has the same bubble as GPipe at 2 stages.  p = bytes / bw with the unit's bf16 activation
(g * 8 images x 512 x 16 x 16) and bw = --p2p-gbs (default 50 GB/s, one xGMI link as the P2P ring measured it).
A record without phases falls back to its whole ms_per_step as c_s and o_1 = 0.

    python scripts/pipeline_units.py stages.jsonl [--one-gpu bench.jsonl] [--p2p-gbs 50] [--json out.json]

``--json`` writes the table the bench reads (bench/harness.py: the resnet50_pp record's default unit size,
``predicted_2gpu_img_s`` and ``one_gpu_img_s`` come from it).
"""
import argparse
import json


def predict(c1: float, c2: float, units: int, p_ms: float, o1: float = 0.0) -> float:
    """Predicted 2-stage pipeline step (ms) for `units` units with per-unit stage compute c1, c2 (ms)."""
    return c1 + c2 + (units - 1) * max(c1, c2) + o1 + 2 * p_ms


def _split(rec):
    """(per-unit fwd+bwd ms, optimiser ms) of a stage record."""
    ph = ((rec["config"].get("phases") or {}).get("rank0_ms")) or {}
    if "fwd" in ph and "bwd" in ph:
        c = ph["fwd"] + ph["bwd"] + ph.get("other", 0.0) + ph.get("comm", 0.0)
        # the captured copy's phases sum to its span; scale to the timed step (graph launch gaps included)
        span = ph.get("span") or (c + ph.get("opt", 0.0))
        k = rec["ms_per_step"] / span if span else 1.0
        return c * k, ph.get("opt", 0.0) * k
    return rec["ms_per_step"], 0.0


def table(recs, one_gpu_img_s=None, p2p_gbs=50.0, batch=32, split=8):
    t = {}
    for r in recs:
        c = r["config"]
        if "stage" in c and "mb_per_unit" in c:
            t[(c["stage"], c["mb_per_unit"])] = r
    rows, best = [], None
    for g in sorted({k[1] for k in t}):
        if (1, g) not in t or (2, g) not in t:
            continue
        units = batch // (split * g)
        p_ms = g * split * 512 * 16 * 16 * 2 / (p2p_gbs * 1e9) * 1e3
        (c1, o1), (c2, _) = _split(t[(1, g)]), _split(t[(2, g)])
        step = predict(c1, c2, units, p_ms, o1)
        ips = batch / step * 1e3
        rows.append({"mb_per_unit": g, "units": units, "t1_ms": t[(1, g)]["ms_per_step"],
                     "t2_ms": t[(2, g)]["ms_per_step"], "c1_ms": round(c1, 4), "c2_ms": round(c2, 4),
                     "opt1_ms": round(o1, 4), "p2p_ms": round(p_ms, 4), "step_ms": round(step, 4),
                     "predicted_2gpu_img_s": round(ips, 1)})
        if best is None or ips > best["predicted_2gpu_img_s"]:
            best = rows[-1]
    return {"formula": "c1 + c2 + (U-1)*max(c1,c2) + opt1 + 2*p2p", "p2p_gbs": p2p_gbs, "rows": rows,
            "best": best, "one_gpu_img_s": one_gpu_img_s}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stages")
    ap.add_argument("--one-gpu", help="a bench.py --model resnet50 JSON line (file) for the 1-GPU whole-model rate")
    ap.add_argument("--p2p-gbs", type=float, default=50.0)
    ap.add_argument("--json", help="also write the table as JSON (read by the bench)")
    a = ap.parse_args()
    recs = [json.loads(ln) for ln in open(a.stages) if ln.strip().startswith("{")]
    one = None
    for ln in (open(a.one_gpu) if a.one_gpu else []):
        if ln.strip().startswith("{"):
            r = json.loads(ln)
            if r["config"]["model"] == "resnet50_128px":
                one = r["value"]
    res = table(recs, one, a.p2p_gbs)
    res["source"] = a.stages
    print("| micro-batches per unit g | units U | stage 1 ms/unit (fwd+bwd / opt) | stage 2 ms/unit (fwd+bwd) "
          "| P2P ms | predicted 2-GPU step ms | predicted img/s (2 GPUs) |")
    print("|---|---|---|---|---|---|---|")
    for r in res["rows"]:
        print(f"| {r['mb_per_unit']} | {r['units']} | {r['t1_ms']:.3f} ({r['c1_ms']:.3f} / {r['opt1_ms']:.3f}) | "
              f"{r['t2_ms']:.3f} ({r['c2_ms']:.3f}) | {r['p2p_ms']:.3f} | {r['step_ms']:.3f} | "
              f"{r['predicted_2gpu_img_s']:.0f} |")
    if res["best"]:
        print(f"\nbest unit: g = {res['best']['mb_per_unit']} ({res['best']['predicted_2gpu_img_s']:.0f} img/s predicted "
              f"on 2 GPUs)" + (f"; 1 GPU whole model: {one:.0f} img/s" if one else ""))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
