"""Time the per-sweep TNT refresh of BASELINE configs[4] (gs_white_tnt + gs_prefix_sys) kernel by
kernel with HIP events: python tools/prefix_probe.py [n_psr] [chains] [reps]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pulsar_timing_gibbsspec_amd import _lib, synthetic  # noqa: E402
from pulsar_timing_gibbsspec_amd._lib import check, ptr  # noqa: E402
from pulsar_timing_gibbsspec_amd.white import WhiteNoiseModel  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 200
C = int(sys.argv[2]) if len(sys.argv) > 2 else 16
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
d = synthetic.config5_array(n_psr=P, n_toa=10_000, n_f=100, seed=0)
ctx = _lib.Context(0, seed=1)
ctx.set_option(_lib.OPT_X_PER_SYS, 1)
wm = WhiteNoiseModel(ctx, d["T"], d["r"], d["sigma"], d["backend"], [d["fidx"]] * P, [d["phiinv_fixed"]] * P,
                     [d["white"]] * P, C)
x = torch.as_tensor(np.repeat(d["x0"], C, axis=0), device=ctx.device)
wm.refresh(x, d["n_param"])
torch.cuda.synchronize()
lib, h, st = ctx.lib, ctx.handle, ctx.stream


def ev(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


t_tnt = ev(lambda: wm.tnt(x, d["n_param"]))
t_pre = ev(lambda: check(lib.gs_prefix_sys(h, wm.P, wm.C, wm.NF, wm.NMX, ptr(wm.pdesc), wm.tnt_cstride, wm.d_cstride,
                                           ptr(wm.TNT), ptr(wm.d), ptr(wm.fidx), ptr(wm.midx), ptr(wm.phfix),
                                           ptr(wm.model), ptr(wm.pinfo)), "prefix"))
print(f"systems {P * C}: gs_white_tnt {t_tnt:.3f} ms, gs_prefix_sys {t_pre:.3f} ms (NF {wm.NF}, NMX {wm.NMX})")
