"""The CPU baseline legs of bench.py (oracle/cpu_baseline.py: test/measurement infrastructure)
and the committed reference-vs-port calibration (tools/calibrate_cpu_baseline.py)."""
import json
import os

import numpy as np

from oracle import cpu_baseline as CB

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rate_and_ess_per_sweep_single():
    it, el, what = CB.rate("single", 0.3)
    assert it > 0 and el >= 0.3 and "pulsar_gibbs.py" in what
    e = CB.ess_per_sweep("single", 20, 300)
    assert 0 < e["ess_per_sweep"] <= 1 and e["sweeps"] == 300


def test_every_kind_builds_a_step():
    for kind in ("indep", "curn", "curn_red", "ecorr"):
        step, get_x, what = CB.KINDS[kind]()
        step()
        x = np.asarray(get_x())
        assert x.ndim == 1 and np.all(np.isfinite(x)), kind


def test_calibration_within_bounds():
    """the restatement's speed is checked against the reference in the build container;
    the committed ratios are the ones bench.py scales the host rate by."""
    cal = json.load(open(os.path.join(ROOT, "profiles", "cpu_calibration.json")))
    for kind in ("single", "curn", "curn_red"):
        r = cal["ratios"][kind]
        assert r["reference_it_s"] > 0 and r["port_it_s"] > 0
        assert abs(r["ref_over_port"] - r["reference_it_s"] / r["port_it_s"]) < 1e-12
        assert 0.5 < r["ref_over_port"] < 2.0, (kind, r)
