"""gs_bdraw_tiled one chain per wave (GS_OPT_SWEEP_SCHED = 2) against two chains per wave (3) on the
PTA curn engine: HIP-event time per launch with every chain drawing, on the 45-pulsar array (two of
whose pulsars have nM = 17 and take the row-major fixed block) and on its first 3 pulsars (all nM <= 16)
at a chain count that fills the chip the same way.

    python tools/bdraw_pair_ab.py [out.json]
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from pulsar_timing_gibbsspec_amd import PTABlockGibbs, _lib, synthetic
    res = {}
    for n_psr, C in ((45, 2048), (3, 30720)):
        pta = synthetic.array_pta(kind="curn", n_psr=n_psr, seed=5)
        gb = PTABlockGibbs(pta, nchains=C, seed=13)
        x0 = np.concatenate([np.atleast_1d(p.sample()).ravel() for p in gb.params])
        eng = gb._new_engine(x0)
        eng.sweep()
        st = eng.ctx.stream
        for rep in range(2):
            for sched in (2, 3):
                eng.ctx.set_option(_lib.OPT_SWEEP_SCHED, sched)
                for _ in range(3):
                    eng._bdraw(None, _lib.EV_B, None)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                with torch.cuda.stream(st):
                    e0.record(st)
                    for _ in range(20):
                        eng._bdraw(None, _lib.EV_B, None)
                    e1.record(st)
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / 20
                shape = eng.ctx.get_option(_lib.OPT_LAST_SWEEP_SHAPE)
                key = f"psr{n_psr}_c{C}_sched{sched}"
                res.setdefault(key, []).append(ms)
                print(key, "shape", shape, "ms %.4f" % ms, flush=True)
        eng.ctx.set_option(_lib.OPT_SWEEP_SCHED, 0)
        del eng, gb
        torch.cuda.empty_cache()
    if len(sys.argv) > 1:
        json.dump(res, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
