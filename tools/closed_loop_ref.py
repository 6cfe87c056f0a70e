"""CPU: how far does an error-free b|rho, fed the reference's own draws, drift from the reference's
fed-back chain?  Also the reference's open-loop (per-draw) distance from the exact draw.
Usage: python tools/closed_loop_ref.py [j1713] [indep]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import gibbs_oracle as O  # noqa: E402
from tests.conftest import golden  # noqa: E402
from tests.parity_data import (INDEP_ZC_FILE, ZC_FILE, exact_chol_draw_pre, exact_sweep_single, exact_tnt,  # noqa: E402
                               indep_pick, normwise_rel, single_replay)


def one(name, f, zc_file, key, n=None):
    R = single_replay(f, zc_file=zc_file, key=key)
    n = int(f["chain"].shape[0]) if n is None else n
    tl = exact_tnt(f["T"], f["Nvec"], f["r"])
    gw, order = R["gwid"], R["order"]
    phi = lambda x: O.phiinv_single(x, R["n_tm"])  # noqa: E731
    ch, bc, _ = exact_sweep_single(tl, gw, f["x0"], R["rhomin"], R["rhomax"], R["zc"], f["U"], n, phi, order)
    cx, cb, _ = O.sweep_single(R["TNT"], R["d"], gw, f["x0"], R["rhomin"], R["rhomax"], R["zc"], f["U"], n, phi,
                               draw="chol", order=order)
    ol = max(normwise_rel(f["bchain"][j], exact_chol_draw_pre(tl, phi(f["chain"][j]), R["zc"][j], order))
             for j in range(1, n))
    print(f"{name} n={n}: exact-loop vs ref x {normwise_rel(ch, f['chain'][:n]):.3g} "
          f"b {normwise_rel(bc[1:], f['bchain'][1:n]):.3g} | fp64-chol-loop vs ref x "
          f"{normwise_rel(cx, f['chain'][:n]):.3g} b {normwise_rel(cb[1:], f['bchain'][1:n]):.3g} | "
          f"ref per draw vs exact {ol:.3g}")


if __name__ == "__main__":
    what = sys.argv[1:] or ["j1713", "indep"]
    if "j1713" in what:
        one("J1713", golden("single_j1713.npz"), ZC_FILE, "zc")
    if "indep" in what:
        ga = golden("indep_array.npz")
        for k in range(3):
            one(f"configs[2] pulsar {int(ga['picks'][k])}", indep_pick(ga, k), INDEP_ZC_FILE, f"zc{k}")
