"""How much of the red-noise grid is negligible in practice (CURN + red, configs[3])?

Runs the PTA engine for a burn-in on the 45 simulated pulsars, then for the red conditional
(pta_gibbs.py:252-276) counts, per (pulsar, frequency, chain) row, the grid points whose
pdf term h e^-h (h = tau / (2 (gw + rho_g))) is below 1e-20 of the row's largest term.
Prints one JSON line.  Needs a GPU.
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from pulsar_timing_gibbsspec_amd import _lib, synthetic
    from pulsar_timing_gibbsspec_amd.engine import DeviceModel, PTAChains
    C, burn = 64, 200
    pta = synthetic.array_pta(kind="curn_red", seed=0)
    T, N, R = pta.get_basis(), pta.get_ndiag({}), pta.get_residuals()
    names = pta.param_names
    rind = [i for i, n in enumerate(names) if "rho" in n and "gw" in n]
    hind = np.array([i for i, n in enumerate(names) if "red" in n and "rho" in n])
    ctx = _lib.Context(0, seed=3)
    model = DeviceModel(ctx, T, N, R, [np.arange(t.shape[1] - 60, t.shape[1]) for t in T],
                        [np.full(t.shape[1] - 60, 1e-40) for t in T])
    x0 = np.random.default_rng(0).uniform(-9, -4, (C, len(names)))
    eng = PTAChains(model, len(names), rind, hind.reshape(len(T), -1), (1e-18, 1e-8), (1e-20, 1e-8), C, x0)
    for _ in range(burn):
        eng.sweep()
    torch.cuda.synchronize()
    tau = eng.tau.cpu().numpy()            # [P, n_f, C] (tau of the last sweep)
    x = eng.x.cpu().numpy()
    gw = 10.0 ** (2.0 * x[:, rind])        # [C, n_f]
    g = eng.grid_red[:eng.ngrid].cpu().numpy()
    th = 0.5 * tau                           # [P, n_f, C]
    h = th[..., None] / (gw.T[None, :, :, None] + g[None, None, None, :])
    lp = np.log(h) - h
    rel = lp - lp.max(axis=-1, keepdims=True)
    neg = rel < np.log(1e-20)
    left = np.cumprod(neg, axis=-1).sum(axis=-1)          # negligible prefix length per row
    out = {"rows": int(neg.shape[0] * neg.shape[1] * neg.shape[2]), "ngrid": int(g.size),
           "negligible_frac": float(neg.mean()), "negligible_prefix_frac": float(left.mean() / g.size),
           "prefix_frac_quantiles": [float(q) for q in np.quantile(left / g.size, [0.1, 0.5, 0.9])],
           "wave_min_prefix_frac": float(np.mean(left.reshape(-1, 64).min(axis=1)) / g.size)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
