"""ECORR sweep time against the number of backends (the incremental Metropolis step re-weights one
backend's epochs): bench.py's ecorr construction on ecorr_pulsar_pta(n_backends=k), C chains, K timed
sweeps after a 60 ms warm-up.  Run once with GS_ECORR_INC=1 (default) and once with 0.
    python tools/ecorr_backends_ab.py [chains] [sweeps]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(nbk, C, K):
    from pulsar_timing_gibbsspec_amd import _lib, synthetic
    from pulsar_timing_gibbsspec_amd.ecorr import EcorrFreeSpectrumChains, EcorrModel
    pta = synthetic.ecorr_pulsar_pta("J1713+0747", seed=0, n_backends=nbk)
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
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.06:
        eng.sweep()
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        eng.sweep()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / K * 1e3
    print(f"inc={os.environ.get('GS_ECORR_INC', '1')} backends={nbk} epochs={ne} ms/sweep={ms:.4f} "
          f"chain-it/s={C / ms * 1e3:.4e}", flush=True)


if __name__ == "__main__":
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    for nbk in (2, 4, 8):
        run(nbk, C, K)
