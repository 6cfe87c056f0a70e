"""Calibrate bench.py's CPU baseline (the oracle's restatement, ``oracle/cpu_baseline.py``)
against the REFERENCE itself -- build container only (the reference cannot travel to the GPU
box).  BASELINE.md asks for the restatement's speed to be checked against the reference here.

Both run single-threaded (OPENBLAS_NUM_THREADS=1) in this one process, alternately, on the same
synthetic inputs: the reference's own ``PulsarBlockGibbs.sample`` (J1713, configs[0]/[1]) and
``PTABlockGibbs.sample`` (45-pulsar CURN, CURN + red, configs[3]), the reference-default
redsample='mh' model (``curn_plred``, its own methods in sample()'s order) and configs[2]'s 45
independent ``PulsarBlockGibbs.sample`` runs (``indep``), the ECORR samplers (``ecorr``,
``ecorr_white``: the notebook's order over the reference's own blocks) and one configs[4] pulsar
through the reference's white-noise loop (``config5``), imported read-only through
tests/golden/make_golden.py's loader and driven by the enterprise-shaped facade, against the
port's loops of the same names.  Writes profiles/cpu_calibration.json with
ref_over_port = reference rate / port rate per kind (median of the repeats); bench.py reports
``cpu_baseline.reference_equivalent`` = the port's host rate x that ratio.

    PYTHONDONTWRITEBYTECODE=1 python tools/calibrate_cpu_baseline.py [/root/reference]
"""
import os
import sys

for _v in ("OPENBLAS_NUM_THREADS", "OMP_NUM_THREADS", "MKL_NUM_THREADS"):
    os.environ[_v] = "1"

import json  # noqa: E402
import platform  # noqa: E402
import tempfile  # noqa: E402
import time  # noqa: E402

import numpy as np  # noqa: E402

sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

from make_golden import _quiet, load_reference  # noqa: E402
from oracle import cpu_baseline as CB  # noqa: E402
from pulsar_timing_gibbsspec_amd import synthetic  # noqa: E402


def ref_single(ref, niter):
    pta = synthetic.single_pulsar_pta("J1713+0747", seed=0)
    np.random.seed(1)
    g = _quiet(ref["pulsar_gibbs"].PulsarBlockGibbs, pta)
    x0 = np.concatenate([p.sample().flatten() for p in g.params])
    with tempfile.TemporaryDirectory() as d:
        t0 = time.perf_counter()
        _quiet(g.sample, x0, outdir=d, niter=niter)
        return niter / (time.perf_counter() - t0)


def ref_pta(ref, kind, niter):
    pta = synthetic.array_pta(kind=kind, seed=0)
    np.random.seed(5)
    g = _quiet(ref["pta_gibbs"].PTABlockGibbs, pta, hypersample="conditional",
               redsample="conditional" if kind == "curn_red" else "mh")
    x0 = np.concatenate([p.sample().flatten() for p in g.params])
    with tempfile.TemporaryDirectory() as d:
        t0 = time.perf_counter()
        _quiet(g.sample, x0, outdir=d, niter=niter)
        return niter / (time.perf_counter() - t0)


def ref_plred(ref, niter, acl=20, n_psr=None):
    """The reference's DEFAULT PTA model (redsample='mh', power-law red noise, 45 pulsars) driven
    with its own methods in sample()'s order (pta_gibbs.py:664-712: record, TNT reset, red MH block
    of aclength_hyper steps, CURN draw, gated b, chain.txt every 100 sweeps).  sample() itself cannot
    pass sweep 0 on this path (its iters=100 warm-up ends in an SVD of an empty covariance, pta_hyper),
    so every sweep runs the steady-state branch with aclength_hyper = acl -- the patch
    make_golden.py's pta_hyper_mh pins draw for draw.  Sweep 0's b draw is outside the timing."""
    pta = synthetic.array_pta(kind="curn_plred", seed=0, n_psr=n_psr)
    np.random.seed(5)
    g = _quiet(ref["pta_gibbs"].PTABlockGibbs, pta, hypersample="conditional", redsample="mh")
    x0 = np.concatenate([p.sample().flatten() for p in g.params])
    g.aclength_hyper = acl
    g._b = _quiet(g.update_b, x0)
    chain = np.zeros((niter, x0.size))
    xnew = x0
    with tempfile.TemporaryDirectory() as d:
        t0 = time.perf_counter()
        for ii in range(niter):
            chain[ii] = xnew
            g.TNT, g.d = [], []
            xnew = g.update_hyper_params(xnew, iters=None)
            xnew = g.update_rho_params(xnew)
            if np.all(xnew != chain[ii][-1]):
                g._b = g.update_b(xnew)
            if ii % 100 == 0 and ii > 0:
                np.savetxt(f"{d}/chain.txt", chain[:ii + 1])
        return niter / (time.perf_counter() - t0)


def ref_indep(ref, niter):
    """configs[2]: the reference's PulsarBlockGibbs.sample over each of the 45 independent pulsars
    (pulsar_gibbs.py:620-710), as a user would loop over them; array sweeps per second = niter /
    the summed time of the 45 runs."""
    ptas = synthetic.pulsar_ptas(synthetic.array_pta(kind="indep", seed=0))
    np.random.seed(3)
    tot = 0.0
    for pta in ptas:
        g = _quiet(ref["pulsar_gibbs"].PulsarBlockGibbs, pta)
        x0 = np.concatenate([p.sample().flatten() for p in g.params])
        with tempfile.TemporaryDirectory() as d:
            t0 = time.perf_counter()
            _quiet(g.sample, x0, outdir=d, niter=niter)
            tot += time.perf_counter() - t0
    return niter / tot


def _pulsar_loop(g, x0, niter, blocks):
    """The reference's PulsarBlockGibbs.sample body (pulsar_gibbs.py:656-710) with the Metropolis
    blocks given (each in its steady-state branch: the iters=1000 warm-ups need the absent acor),
    timed from sweep 1: record, TNT reset, blocks, rho|b, gated b, chain/bchain .npy every 100."""
    g._b = g.update_b(x0)
    chain = np.zeros((niter, x0.size))
    bchain = np.zeros((niter, g._b.size))
    xnew = x0.copy()
    with tempfile.TemporaryDirectory() as d:
        t0 = time.perf_counter()
        for ii in range(niter):
            chain[ii], bchain[ii] = xnew, g._b
            g.TNT = g.d = None
            for blk in blocks:
                xnew = blk(xnew, iters=None)
            xnew = g.update_gwrho_params(xnew)
            if np.all(xnew != chain[ii][-1]):
                g._b = g.update_b(xnew)
            if ii % 100 == 0 and ii > 0:
                np.save(f"{d}/chain.npy", chain[:ii + 1])
                np.save(f"{d}/bchain.npy", bchain[:ii + 1])
        return niter / (time.perf_counter() - t0)


def ref_ecorr(ref, niter, white, acl=10):
    """SURVEY 8f-4 (the port's ``ecorr`` / ``ecorr_white``): the reference's update_ecorr_params
    (pulsar_gibbs.py:409-486, its get_lnlikelihood bound to get_lnlikelihood_fullmarg, :569-610, as
    the notebook sampler does) [after update_white_params, :332-406], rho|b and the gated b draw, on
    the synthetic J1713 ECORR pulsar; aclength = acl for every block (as the port)."""
    pta = synthetic.ecorr_pulsar_pta("J1713+0747", seed=0, white_vary=white)
    np.random.seed(41)
    g = _quiet(ref["pulsar_gibbs"].PulsarBlockGibbs, pta)
    g.get_lnlikelihood = g.get_lnlikelihood_fullmarg
    x0 = np.concatenate([p.sample().flatten() for p in g.params])
    wind = g.get_efacequad_indices()
    if white:
        x0[wind] = [1.0 if "efac" in n else -7.0 for n in np.array(g.param_names)[wind]]
    g.aclength_white = g.aclength_ecorr = acl
    blocks = ([g.update_white_params] if white else []) + [g.update_ecorr_params]
    return _pulsar_loop(g, x0, niter, blocks)


def ref_config5(ref, niter, acl=20):
    """configs[4] (the port's ``config5``): one 10^4-TOA, m = 216 pulsar through the reference's own
    PulsarBlockGibbs loop with the white MH block (20 steps, pulsar_gibbs.py:373-404; TNT recomputed
    every sweep, :495-502), per 200-pulsar array sweep (x 1/200, as the port)."""
    pta = synthetic.config5_pulsar_pta(seed=1)
    np.random.seed(51)
    g = _quiet(ref["pulsar_gibbs"].PulsarBlockGibbs, pta)
    x0 = np.concatenate([p.sample().flatten() for p in g.params])
    g.aclength_white = acl
    return _pulsar_loop(g, x0, niter, [g.update_white_params]) * CB.PER_SWEEP["config5"]


def port(kind, seconds):
    it, el, _ = CB.rate(kind, seconds)
    return it / el


def main(root):
    ref = load_reference(root)
    plan = {"single": (lambda: ref_single(ref, 3000), 3.0),
            "curn": (lambda: ref_pta(ref, "curn", 150), 5.0),
            "curn_red": (lambda: ref_pta(ref, "curn_red", 120), 5.0),
            "curn_plred": (lambda: ref_plred(ref, 12), 5.0),
            "indep": (lambda: ref_indep(ref, 60), 5.0),
            "ecorr": (lambda: ref_ecorr(ref, 60, False), 5.0),
            "ecorr_white": (lambda: ref_ecorr(ref, 50, True), 5.0),
            "config5": (lambda: ref_config5(ref, 12), 5.0)}
    only = [a[len("--only="):].split(",") for a in sys.argv if a.startswith("--only=")]
    if only:
        plan = {k: v for k, v in plan.items() if k in only[0]}
    out = {"ratios": {}, "host": platform.processor() or CB.cpu_model(), "cpu": CB.cpu_model(),
           "threads": 1, "repeats": 3,
           "note": "single-threaded rates in the build container; reference = the reference's own sample() loop "
                   "(index-finder scans, TNT reset and recompute, SVD draws, chain bookkeeping and periodic saves "
                   "included) on the facade PTA; port = oracle/cpu_baseline.py's loop"}
    for kind, (fref, secs) in plan.items():
        r, p = [], []
        for _ in range(3):
            r.append(fref())
            p.append(port(kind, secs))
        rr, pp = float(np.median(r)), float(np.median(p))
        out["ratios"][kind] = {"reference_it_s": rr, "port_it_s": pp, "ref_over_port": rr / pp,
                               "reference_runs": r, "port_runs": p}
        print(kind, f"reference {rr:.1f} it/s, port {pp:.1f} it/s, ratio {rr / pp:.3f}", flush=True)
    path = os.path.join(ROOT, "profiles", "cpu_calibration.json")
    if only and os.path.exists(path):            # merge into the existing record
        old = json.load(open(path))
        old["ratios"].update(out["ratios"])
        out = old
    with open(path, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    main(args[0] if args else "/root/reference")
