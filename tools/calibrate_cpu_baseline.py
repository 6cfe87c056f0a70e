"""Calibrate bench.py's CPU baseline (the oracle's restatement, ``oracle/cpu_baseline.py``)
against the REFERENCE itself -- build container only (the reference cannot travel to the GPU
box).  BASELINE.md asks for the restatement's speed to be checked against the reference here.

Both run single-threaded (OPENBLAS_NUM_THREADS=1) in this one process, alternately, on the same
synthetic inputs: the reference's own ``PulsarBlockGibbs.sample`` (J1713, configs[0]/[1]) and
``PTABlockGibbs.sample`` (45-pulsar CURN, CURN + red, configs[3]), imported read-only through
tests/golden/make_golden.py's loader and driven by the enterprise-shaped facade, against the
port's loops ``single`` / ``curn`` / ``curn_red``.  Writes profiles/cpu_calibration.json with
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


def port(kind, seconds):
    it, el, _ = CB.rate(kind, seconds)
    return it / el


def main(root):
    ref = load_reference(root)
    plan = {"single": (lambda: ref_single(ref, 3000), 3.0),
            "curn": (lambda: ref_pta(ref, "curn", 150), 5.0),
            "curn_red": (lambda: ref_pta(ref, "curn_red", 120), 5.0)}
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
    with open(os.path.join(ROOT, "profiles", "cpu_calibration.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    main(args[0] if args else "/root/reference")
