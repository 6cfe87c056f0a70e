"""A/B of the red free-spectrum grid draw (configs[3] CURN + red, 45 pulsars x 30 bins x C chains):
GS_OPT_GRID_EXACT 0 (k_rho_red_cert16, default), 3 (k_rho_red_cert, round 3), 2 (f64 wave kernel),
HIP-event time per launch on the context stream, the f64-redo (fallback) row fraction, and whether
the indices agree with mode 2.  python tools/ab_red_grid.py [chains] [reps]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pulsar_timing_gibbsspec_amd import _lib, synthetic  # noqa: E402
from pulsar_timing_gibbsspec_amd.engine import DeviceModel, PTAChains  # noqa: E402


def main(C=2048, reps=10):
    ctx = _lib.Context(0, seed=5)
    pta = synthetic.array_pta(kind="curn_red", seed=0)
    T, N, R = pta.get_basis(), pta.get_ndiag({}), pta.get_residuals()
    names = pta.param_names
    rind = [i for i, n in enumerate(names) if "rho" in n and "gw" in n]
    hind = np.array([i for i, n in enumerate(names) if "red" in n and "rho" in n])
    gwid = [np.arange(t.shape[1] - 60, t.shape[1]) for t in T]
    fixed = [np.full(t.shape[1] - 60, 1e-40) for t in T]
    model = DeviceModel(ctx, T, N, R, gwid, fixed)
    x0 = np.random.default_rng(0).uniform(-9, -4, (C, len(names)))
    eng = PTAChains(model, len(names), rind, hind.reshape(len(T), -1), (1e-18, 1e-8), (1e-20, 1e-8), C, x0)
    for _ in range(20):                      # near the posterior
        eng.sweep()
    lib, h = ctx.lib, ctx.handle
    _lib.check(lib.gs_tau(h, eng.P, C, model.NF, model.ldb, _lib.ptr(model.fidx), _lib.ptr(eng.b), 0,
                          _lib.ptr(eng.tau)), "gs_tau")
    _lib.check(lib.gs_phi_from_x(h, C, eng.n_f, _lib.ptr(eng.x), eng.n_param, _lib.ptr(eng.gw_col),
                                 _lib.ptr(eng.gwphi)), "phi")
    fb = torch.zeros(1, dtype=torch.int32, device="cuda")
    out = {}
    idx = {}
    nrow = eng.P * eng.n_f * C
    for mode in (2, 3, 0):
        ctx.set_option(_lib.OPT_GRID_EXACT, mode)
        ix = torch.zeros(nrow, dtype=torch.int32, device="cuda")
        x = eng.x.clone()

        def go():
            _lib.check(lib.gs_rho_red(h, eng.P, C, eng.n_f, _lib.ptr(eng.tau), _lib.ptr(eng.gwphi), 1000,
                                      _lib.ptr(eng.grid_red), None, 7, 0, _lib.ptr(x), eng.n_param,
                                      _lib.ptr(eng.red_col), _lib.ptr(ix)), "gs_rho_red")
        go()
        torch.cuda.synchronize()
        fb.zero_()
        _lib.check(lib.gs_ctx_set_grid_fallback_counter(h, _lib.ptr(fb)), "fb")
        go()
        torch.cuda.synchronize()
        _lib.check(lib.gs_ctx_set_grid_fallback_counter(h, None), "fb")
        nfb = int(fb.item())
        st = ctx.stream
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            go()
        e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        idx[mode] = ix.cpu().numpy()
        out[mode] = dict(ms=ms, fallback_rows=nfb, fallback_frac=nfb / nrow,
                         points_per_s=nrow * 1000 / (ms * 1e-3))
    ctx.set_option(_lib.OPT_GRID_EXACT, 0)
    for m in (3, 0):
        out[m]["index_mismatch_vs_f64"] = int(np.sum(idx[m] != idx[2]))
    print(json.dumps({"chains": C, "rows": nrow, "modes": out}))


if __name__ == "__main__":
    a = [int(v) for v in sys.argv[1:]]
    main(*a)
