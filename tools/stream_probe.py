"""Chain-history streaming probe (MI355X): how fast can the headline's recorded x rows reach
pinned host memory while the next block of sweeps runs?

Prints one JSON line with, per 100-sweep block of the configs[1] headline (4096 chains):
  kernel_ms      the fused sweep alone (rows into HBM)
  copy_ms        D2H of one block's x rows (98 MB) alone, torch copy_ to pinned memory
  streamed_ms    HistoryStreamer (as sample()): copy of block i overlapped with block i+1
  zero_copy_ms   the kernel writes x rows straight into pinned host memory (no copy)
Run under different runtime copy settings to compare (e.g. GPU_BLIT_ENGINE_TYPE).
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from pulsar_timing_gibbsspec_amd import _lib, synthetic
    from pulsar_timing_gibbsspec_amd.engine import DeviceModel, FreeSpectrumChains, HistoryStreamer

    C, S, NB = 4096, 100, 6
    pta = synthetic.single_pulsar_pta("J1713+0747", seed=0)
    T, N, r = pta.get_basis()[0], pta.get_ndiag({})[0], pta.get_residuals()[0]
    ctx = _lib.Context(0, seed=1)
    model = DeviceModel(ctx, [T], [N], [r], [np.arange(60)], [np.full(T.shape[1] - 60, 1e-40)])
    x0 = np.random.default_rng(0).uniform(-9, -4, (C, 30))
    run = FreeSpectrumChains(model, 1e-18, 1e-8, C, x0)
    dev = torch.device("cuda", 0)
    xr = torch.empty(S, C, 30, dtype=torch.float64, device=dev)
    run.run(S, x_rec=xr, record_b=False)
    torch.cuda.synchronize()
    out = {"env": {k: os.environ.get(k) for k in ("GPU_BLIT_ENGINE_TYPE", "HSA_ENABLE_SDMA",
                                                  "GPU_FORCE_BLIT_COPY_SIZE")}}

    def timed(fn, n=NB):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn(n)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    out["kernel_ms"] = timed(lambda n: [run.run(S, x_rec=xr, record_b=False) for _ in range(n)])
    hx = torch.empty(S, C, 30, dtype=torch.float64, pin_memory=True)
    out["copy_ms"] = timed(lambda n: [hx.copy_(xr, non_blocking=True) for _ in range(n)])
    out["copy_GBps"] = xr.numel() * 8 / out["copy_ms"] / 1e6

    # the same copy split over K streams (chunks of sweeps): several copy engines at once?
    sides = [torch.cuda.Stream(device=dev) for _ in range(4)]

    def split_copy(n, K):
        step = S // K
        for _ in range(n):
            for i in range(K):
                with torch.cuda.stream(sides[i]):
                    hx[i * step:(i + 1) * step].copy_(xr[i * step:(i + 1) * step], non_blocking=True)
    for K in (2, 4):
        out[f"copy_split{K}_ms"] = timed(lambda n: split_copy(n, K))

    streamer = HistoryStreamer(ctx, [(S, C, 30)])

    def streamed(n):
        slot, pending = 0, None
        for _ in range(n):
            (buf,) = streamer.buffers(slot, S)
            run.run(S, x_rec=buf, record_b=False)
            streamer.submit(slot, S)
            if pending is not None:
                streamer.fetch(pending)
            pending, slot = slot, slot ^ 1
        streamer.fetch(pending)
    out["streamed_ms"] = timed(streamed)

    hz = [torch.empty(S, C, 30, dtype=torch.float64, pin_memory=True) for _ in range(2)]
    out["zero_copy_ms"] = timed(lambda n: [run.run(S, x_rec=hz[i & 1], record_b=False) for i in range(n)])
    # the zero-copy rows equal the HBM rows of the same sweeps?
    run2 = FreeSpectrumChains(model, 1e-18, 1e-8, C, x0)
    run3 = FreeSpectrumChains(model, 1e-18, 1e-8, C, x0)
    a = run2.run(S, record_b=False)[0]
    run3.run(S, x_rec=hz[0], record_b=False)
    torch.cuda.synchronize()
    out["zero_copy_equal"] = bool(torch.equal(a.cpu(), hz[0]))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
