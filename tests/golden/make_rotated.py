"""Freeze the rotated normals of the single-pulsar golden run (tests/golden/single_j1713_zc.npz).

The reference draws b = mn + U S^-1/2 z (pulsar_gibbs.py:508-518); the device draws
b = mn + L^-T z'.  Exact-draw parity feeds the device z' = L^T U S^-1/2 z computed
along the reference trajectory (tests/parity_data.py).  That rotation takes an SVD of
Sigma (cond ~1e6..1e9), and its last bits depend on the host's BLAS: thread count and
the OpenBLAS kernel picked for the CPU move z' by ~5e-10, which a 1e-9 parity check
cannot absorb.  So z' is computed ONCE here (single-threaded OpenBLAS, this container)
and committed (tests/golden/single_j1713_zc.npz, indep_array_zc.npz); tests and smoke() read it instead of recomputing it on whatever host
they run on.

Inputs: tests/golden/single_j1713.npz and indep_array.npz only (no reference import).  Run from the repo
root:  python tests/golden/make_rotated.py
"""
import os
import sys

os.environ["OPENBLAS_NUM_THREADS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
from threadpoolctl import threadpool_limits  # noqa: E402

from tests.parity_data import INDEP_ZC_FILE, ZC_FILE, indep_pick, single_replay_compute  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")


def main():
    g = np.load(os.path.join(GOLDEN, "single_j1713.npz"), allow_pickle=False)
    with threadpool_limits(limits=1):
        zc = single_replay_compute(g)["zc"]
    np.savez_compressed(ZC_FILE, zc=zc)
    print(f"wrote {ZC_FILE}: zc {zc.shape}")
    # configs[2]: the three reference-run pulsars of tests/golden/indep_array.npz
    g = np.load(os.path.join(GOLDEN, "indep_array.npz"), allow_pickle=False)
    out = {}
    with threadpool_limits(limits=1):
        for k in range(len(g["picks"])):
            out[f"zc{k}"] = single_replay_compute(indep_pick(g, k))["zc"]
    np.savez_compressed(INDEP_ZC_FILE, **out)
    print(f"wrote {INDEP_ZC_FILE}: {[v.shape for v in out.values()]}")


if __name__ == "__main__":
    main()
