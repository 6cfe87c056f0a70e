"""The CPU baseline legs of bench.py (oracle/cpu_baseline.py: test/measurement infrastructure)
and the committed reference-vs-port calibration (tools/calibrate_cpu_baseline.py)."""
import json
import os

import numpy as np

from oracle import cpu_baseline as CB

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rate_and_ess_per_sweep_single(tmp_path):
    it, el, what = CB.rate("single", 0.3)
    assert it > 0 and el >= 0.3 and "pulsar_gibbs.py" in what
    from pulsar_timing_gibbsspec_amd.diagnostics import ESS_RUN
    pool = CB.EssPool(4, str(tmp_path))
    pool.submit("single", chains=3)
    e = pool.collect("single", timeout=600)
    assert "error" not in e, e
    assert e["chains"] == 3 and (e["burn_in"], e["sweeps"]) == ESS_RUN["single"]
    assert 0 < e["ess_per_sweep"] <= 1 and 0 < e["se"] < e["ess_per_sweep"]
    assert len(e["per_bin"]) == 30 and e["ess_per_sweep"] == min(e["per_bin"])
    # the analytic-rho chain mixes in a few tens of sweeps (GPU: 1/0.04 ~ 25, profiles/r05z17)
    assert 0.01 < e["ess_per_sweep"] < 0.2
    assert not list(tmp_path.glob("*.npy"))


def test_fast_draws_match_the_reference_law():
    """The ESS runs' equal-law shortcuts: the Cholesky b draw has the SVD draw's mean and covariance,
    and the log-space CURN / vectorised red grid draws return the oracle's grid indices."""
    from oracle import gibbs_oracle as O
    from pulsar_timing_gibbsspec_amd import synthetic
    pta = synthetic.single_pulsar_pta("J1713+0747", seed=0)
    T, N, r = pta.get_basis()[0], pta.get_ndiag({})[0], pta.get_residuals()[0]
    TNT, d = O.tnt(T, N, r)
    ph = O.phiinv_single(np.random.default_rng(0).uniform(-9, -4, 30), T.shape[1] - 60)
    m = T.shape[1]
    mean_svd = O.bdraw_svd(TNT, d, ph, np.zeros(m))
    mean_chol = CB._bdraw_fast(TNT, d, ph, np.zeros(m))
    assert np.max(np.abs(mean_chol - mean_svd)) <= 1e-7 * np.max(np.abs(mean_svd))
    E = np.eye(m)
    A = np.stack([CB._bdraw_fast(TNT, d, ph, E[i]) - mean_chol for i in range(m)], axis=1)
    B = np.stack([O.bdraw_svd(TNT, d, ph, E[i]) - mean_svd for i in range(m)], axis=1)
    cov_a, cov_b = A @ A.T, B @ B.T
    assert np.max(np.abs(cov_a - cov_b)) <= 1e-7 * np.max(np.abs(cov_b))
    rng = np.random.default_rng(1)
    for _ in range(20):
        taus = 10 ** rng.uniform(-17, -9, (45, 30))
        irn = 10 ** rng.uniform(-19, -9, (45, 30))
        U = rng.random(30)
        assert np.array_equal(CB._curn_fast(taus, irn, U)[1], O.rho_grid_cdf_curn(taus, irn, U, 1e-18, 1e-8)[1])
        gw = 10 ** rng.uniform(-19, -9, 30)
        Ur = rng.random((45, 30))
        Ur[0, 0] = 0.0                               # u < cdf[0]: index -1 wraps to the top point
        ra, ia = O.rho_grid_cdf_red(taus, gw, Ur, 1e-20, 1e-8)
        rb, ib = CB._red_fast(taus, gw, Ur)
        assert np.array_equal(ra, rb) and np.array_equal(ia % 1000, ib)


def test_every_fast_kind_builds_a_step():
    for kind in ("indep", "curn", "curn_red", "curn_plred", "ecorr", "config5"):
        step, get_x, what = CB.KINDS[kind](fast=True)
        step()
        x = np.asarray(get_x())
        assert x.ndim == 1 and np.all(np.isfinite(x)), kind


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
