"""Test configuration.

* Single-threaded BLAS BEFORE numpy loads: the reference's SVD draw is only
  bit-reproducible with the same BLAS blocking, and the golden fixtures were
  generated with OPENBLAS_NUM_THREADS=1 (tests/golden/make_golden.py).
* Marker ``gpu``: needs an MI355X; everything else runs on CPU.
"""
import os
import sys

os.environ["OPENBLAS_NUM_THREADS"] = "1"
os.environ["OMP_NUM_THREADS"] = os.environ.get("OMP_NUM_THREADS", "1")
os.environ.setdefault("MKL_NUM_THREADS", "1")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import pytest  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP path)")


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="session")
def single():
    return golden("single_j1713.npz")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
