"""Diagnose the rocprofv3 --pmc SIGSEGV on the ECORR lines: run the ECORR
sweep (bench_ecorr's model, few chains, two sweeps) after writing /proc/self/maps, so the crash's
unsymbolised frames can be mapped to (library, offset) and symbolised with llvm-symbolizer in the
build container (same image).  Under rocprofv3:

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/x -o run -- python3 tools/ecorr_pmc_probe.py OUTDIR [C]

GS_PROBE_PHASE: 'factor' (the full ECORR likelihood launch only) or 'sweep' (default: two sweeps).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out = sys.argv[1]
    C = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    os.makedirs(out, exist_ok=True)
    import torch
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
    x0 = np.concatenate([np.full((C, len(eind)), -6.3), np.random.default_rng(0).uniform(-9, -4, (C, len(gw)))],
                        axis=1)
    eng = EcorrFreeSpectrumChains(em, gw, gwid, 1e-18, 1e-8, x0, aclength=4)
    torch.cuda.synchronize()
    with open(os.path.join(out, "maps.txt"), "w") as f:
        f.write(open("/proc/self/maps").read())
    print("[probe] maps written; first ECORR launch next", flush=True)
    if os.environ.get("GS_PROBE_PHASE", "sweep") == "factor":
        em.factor(eng.x)
    else:
        for _ in range(2):
            eng.sweep()
    torch.cuda.synchronize()
    print("[probe] done", flush=True)


if __name__ == "__main__":
    main()
