"""bench.py's stdout line stays parseable: the round-5 line (22.9 KB, every secondary record with its
notes) came back ``parsed: null`` from the driver.  The line builder runs here on the committed full
record of that run (profiles/r05z17/bench.json) and on a synthetic worst case."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

CONTRACT = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config")


def _canned():
    return json.load(open(os.path.join(ROOT, "profiles", "r05z17", "bench.json")))


def test_line_compact_and_round_trips():
    full = _canned()
    assert len(json.dumps(full)) > 20000
    txt = bench.result_line(full)
    assert "\n" not in txt
    assert len(txt) < bench.LINE_MAX
    back = json.loads(txt)
    for k in CONTRACT:
        assert k in back, k
    assert back["value"] == full["value"]
    rf = back["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in rf, k
    cb = back["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cb, k
    assert set(back["secondary"]) == set(full["secondary"])
    for name, s in back["secondary"].items():
        assert s["value"] == bench._sig(full["secondary"][name]["value"])
        assert "frac" in s["roofline"]


def test_line_falls_back_under_the_limit():
    full = _canned()
    # a pathological record: many secondary lines with long kernel names
    for i in range(60):
        full["secondary"][f"extra{i}"] = dict(full["secondary"]["curn_red"],
                                              roofline={"kernel": "k" * 200, "frac": 0.5})
    txt = bench.result_line(full)
    assert len(txt) < bench.LINE_MAX
    assert json.loads(txt)["value"] == full["value"]


def test_detail_file_written(tmp_path):
    full = _canned()
    p = tmp_path / "d" / "bench_detail.json"
    bench.write_detail(full, str(p))
    assert json.load(open(p))["secondary"].keys() == full["secondary"].keys()
