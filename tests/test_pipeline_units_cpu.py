"""The 2-GPU pipeline predictor behind the resnet50_pp default unit size (scripts/pipeline_units.py) and the
bench's reading of its measured table (bench/harness.py ``_unit_table``)."""
import importlib.util
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _mod():
    spec = importlib.util.spec_from_file_location("pipeline_units", os.path.join(REPO, "scripts", "pipeline_units.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _rec(stage, g, ms, fwd, bwd, opt):
    return {"ms_per_step": ms, "value": 8 * g / ms * 1e3,
            "config": {"model": f"resnet50_128px_stage{stage}", "stage": stage, "mb_per_unit": g,
                       "phases": {"rank0_ms": {"fwd": fwd, "bwd": bwd, "opt": opt, "span": fwd + bwd + opt}}}}


def test_one_unit_has_no_overlap():
    m = _mod()
    # U = 1: the two stages run one after the other, plus stage 1's update and both transfers
    assert m.predict(1.0, 2.0, 1, 0.1, 0.05) == 1.0 + 2.0 + 0.05 + 0.2
    # every further unit adds one slot of the slower stage
    assert m.predict(1.0, 2.0, 4, 0.1, 0.0) == 1.0 + 2.0 + 3 * 2.0 + 0.2


def test_table_best_unit_and_json(tmp_path):
    m = _mod()
    recs = [_rec(1, 1, 1.0, 0.45, 0.5, 0.05), _rec(2, 1, 1.5, 0.7, 0.75, 0.05),
            _rec(1, 4, 1.6, 0.75, 0.8, 0.05), _rec(2, 4, 1.9, 0.9, 0.95, 0.05)]
    res = m.table(recs, one_gpu_img_s=9900.0)
    rows = {r["mb_per_unit"]: r for r in res["rows"]}
    assert set(rows) == {1, 4} and rows[4]["units"] == 1 and rows[1]["units"] == 4
    # U = 1 at g = 4: c1 + c2 + opt1 + 2 p (phases scaled to the timed step)
    r4 = rows[4]
    assert abs(r4["step_ms"] - (r4["c1_ms"] + r4["c2_ms"] + r4["opt1_ms"] + 2 * r4["p2p_ms"])) < 1e-3
    assert res["best"]["mb_per_unit"] == max(rows, key=lambda g: rows[g]["predicted_2gpu_img_s"])
    stages = tmp_path / "stages.jsonl"
    stages.write_text("\n".join(json.dumps(r) for r in recs) + "\n")
    one = tmp_path / "one.jsonl"
    one.write_text(json.dumps({"value": 9900.0, "config": {"model": "resnet50_128px"}}) + "\n")
    out = tmp_path / "units.json"
    import subprocess
    import sys

    subprocess.run([sys.executable, os.path.join(REPO, "scripts", "pipeline_units.py"), str(stages), "--one-gpu",
                    str(one), "--json", str(out)], check=True, capture_output=True)
    tab = json.loads(out.read_text())
    assert tab["one_gpu_img_s"] == 9900.0 and tab["best"]["mb_per_unit"] in (1, 4)

    # the bench reads the table it is pointed at
    from pytorch_distributed_examples_amd.bench import harness

    old = os.environ.get("PDE_PIPE_UNIT_TABLE")
    os.environ["PDE_PIPE_UNIT_TABLE"] = str(out)
    try:
        assert harness._unit_table()["best"] == tab["best"]
    finally:
        if old is None:
            os.environ.pop("PDE_PIPE_UNIT_TABLE")
        else:
            os.environ["PDE_PIPE_UNIT_TABLE"] = old


def test_committed_table_is_readable():
    from pytorch_distributed_examples_amd.bench import harness

    tab = harness._unit_table()
    assert tab is not None, "bench/pipeline_units.json (= profiles/r5_pipeline_units.json) is the measured table"
    assert tab["best"]["mb_per_unit"] in {r["mb_per_unit"] for r in tab["rows"]}
    assert tab["one_gpu_img_s"] and all("predicted_2gpu_img_s" in r for r in tab["rows"])
