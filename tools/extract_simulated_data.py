"""Extract the 45-pulsar simulated array into a compact data file.

Run ONCE in the build container (the reference tree does not exist on the GPU
box).  It reads only DATA from the reference: the TOA epochs/errors of each
``simulated_data/<PSR>.tim`` and, from ``<PSR>.par``, the number of fitted
timing parameters and the binary period.  Nothing else is copied.

    python tools/extract_simulated_data.py /root/reference/simulated_data

Output: ``pulsar_timing_gibbsspec_amd/data/simulated_array.npz`` with
``names`` (45,), ``offsets`` (46,) into the flat ``mjd`` / ``err_us`` arrays,
``nfit`` (45,), ``pb_days`` (45,, 0 for isolated pulsars).
"""
import glob
import os
import sys

import numpy as np


def read_tim(path):
    mjd, err = [], []
    with open(path) as fh:
        for line in fh:
            tok = line.split()
            if len(tok) < 4 or tok[0] in ("FORMAT", "MODE", "C", "#"):
                continue
            mjd.append(float(tok[2]))
            err.append(float(tok[3]))
    return np.array(mjd), np.array(err)


def read_par(path):
    nfit, pb = 0, 0.0
    with open(path) as fh:
        for line in fh:
            tok = line.split()
            if len(tok) >= 3 and tok[2] == "1":
                nfit += 1
            if tok and tok[0] == "PB":
                pb = float(tok[1].replace("D", "E"))
    return nfit, pb


def main(src):
    tims = sorted(glob.glob(os.path.join(src, "*.tim")))
    names, mjds, errs, nfits, pbs = [], [], [], [], []
    for t in tims:
        name = os.path.basename(t)[:-4]
        m, e = read_tim(t)
        nfit, pb = read_par(os.path.join(src, name + ".par"))
        names.append(name)
        mjds.append(m)
        errs.append(e)
        nfits.append(nfit)
        pbs.append(pb)
    offsets = np.concatenate([[0], np.cumsum([len(m) for m in mjds])])
    out = os.path.join(os.path.dirname(__file__), "..", "pulsar_timing_gibbsspec_amd",
                       "data", "simulated_array.npz")
    np.savez_compressed(out, names=np.array(names), offsets=offsets,
                        mjd=np.concatenate(mjds), err_us=np.concatenate(errs),
                        nfit=np.array(nfits), pb_days=np.array(pbs))
    print(f"wrote {out}: {len(names)} pulsars, {offsets[-1]} TOAs")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/simulated_data")
