"""Standalone driver of the ECORR likelihood kernel (k_ecorr_prefix, likelihood mode, shared
operands) on bench.py's synthetic J1713-like pulsar, for rocprofv3 counter passes without the rest
of the bench: builds the model as bench.bench_ecorr does and runs `reps` all-chain evaluations.
    python tools/ecorr_probe.py [chains] [reps]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(C=4096, reps=20):
    from pulsar_timing_gibbsspec_amd import _lib, synthetic
    from pulsar_timing_gibbsspec_amd.ecorr import EcorrFreeSpectrumChains, EcorrModel
    pta = synthetic.ecorr_pulsar_pta("J1713+0747", seed=0)
    names = pta.param_names
    ebk = pta.signals["J1713+0747_basis_ecorr"].epoch_backend
    ne = ebk.size
    eind = [i for i, n in enumerate(names) if "ecorr" in n]
    gw = [i for i, n in enumerate(names) if "rho" in n]
    T = pta.get_basis()[0]
    gwid = ne + np.arange(2 * len(gw))
    ctx = _lib.Context(0, seed=20251017)
    em = EcorrModel(ctx, T, pta.get_ndiag()[0], pta.get_residuals()[0], np.arange(ne), ebk, gwid, eind,
                    [-8.5] * len(eind), [-5.0] * len(eind), len(names), C)
    rng = np.random.default_rng(0)
    x0 = np.concatenate([np.full((C, len(eind)), -6.3), rng.uniform(-9, -4, (C, len(gw)))], axis=1)
    eng = EcorrFreeSpectrumChains(em, gw, gwid, 1e-18, 1e-8, x0, aclength=10)
    eng.sweep()
    eng._phiinv(False)
    torch.cuda.synchronize()
    for _ in range(reps):
        em._eval(eng.x, eng.phiinv_F)
    torch.cuda.synchronize()
    print("ok", C, reps, float(em.lnl[:4].sum()))


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
