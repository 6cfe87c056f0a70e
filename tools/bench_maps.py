"""bench.py with /proc/self/maps written just before the first ECORR model is built (GS_MAPS_OUT), so
a crash inside a profiler's launch hook can be mapped to (library, offset) -- the round-5 PMC SIGSEGV
 came from bench.py's ECORR line, not from a standalone ECORR run."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from pulsar_timing_gibbsspec_amd import ecorr  # noqa: E402

_init = ecorr.EcorrModel.__init__


def _init_maps(self, *a, **k):
    with open(os.environ.get("GS_MAPS_OUT", "/tmp/maps.txt"), "w") as f:
        f.write(open("/proc/self/maps").read())
    print("[maps] written before the first ECORR model", file=sys.stderr, flush=True)
    _init(self, *a, **k)


ecorr.EcorrModel.__init__ = _init_maps

import bench  # noqa: E402

if __name__ == "__main__":
    sys.argv[0] = os.path.join(ROOT, "bench.py")
    bench.main()
