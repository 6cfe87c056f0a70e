"""The C-ABI library loads and exports every entry point include/*.h declares
(CPU-only: no compute call is made without a GPU)."""
import ctypes
import glob
import os
import re
import subprocess

import pytest

from tests.conftest import ROOT, gpu_available

LIB = os.path.join(ROOT, "pulsar_timing_gibbsspec_amd", "libpulsar_gibbs.so")


def declared_functions():
    names = []
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names += re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(gs_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", os.path.join(ROOT, "pulsar_timing_gibbsspec_amd", "csrc"), "-j4"],
                       check=True, capture_output=True)
    import torch  # noqa: F401  (share torch's HIP runtime, as _lib does)
    return ctypes.CDLL(LIB)


def test_header_declares_entry_points():
    names = declared_functions()
    for must in ("gs_ctx_create", "gs_tnt", "gs_prefix", "gs_bdraw", "gs_rho_analytic",
                 "gs_sweep_freespec", "gs_philox"):
        assert must in names


def test_library_exports_every_declared_symbol(lib):
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_table_matches_header(lib):
    from pulsar_timing_gibbsspec_amd import _lib
    assert set(_lib.SIGNATURES) == set(declared_functions())


def test_host_only_calls(lib):
    lib.gs_version.restype = ctypes.c_int
    assert lib.gs_version() == 1
    lib.gs_model_stride.restype = ctypes.c_int64
    lib.gs_model_stride.argtypes = [ctypes.c_int, ctypes.c_int]
    s = lib.gs_model_stride(60, 16)
    base = 60 * 61 + 60 + 16 * 61 + 16 + 256 + 2          # S0 | dF | G | h | R | aux[2]
    assert s == base + (base & 1)
    assert s % 2 == 0


def test_argument_validation_without_gpu(lib):
    """A NULL context is rejected before any HIP call; the index names the argument."""
    from pulsar_timing_gibbsspec_amd import _lib
    L = _lib.load()
    rc = L.gs_sweep_freespec(None, 1, 1, 60, 16, 76, None, None, None, None, 1e-18, 1e-8, 0,
                             None, None, 0, 1, None, None, None, None, None, None)
    assert rc == 1
    assert b"ctx" in L.gs_last_error()


@pytest.mark.skipif(gpu_available(), reason="CPU-only behaviour")
def test_no_cpu_fallback():
    from pulsar_timing_gibbsspec_amd import _lib
    with pytest.raises(_lib.GibbsLibError):
        _lib.Context(0)


def test_option_constants_match_header():
    """_lib's OPT_* constants are the header's GS_OPT_* enum values (GS_OPT_SWEEP_SCHED's 0..3 and the
    read-only GS_OPT_LAST_SWEEP_SHAPE included)."""
    from pulsar_timing_gibbsspec_amd import _lib
    src = open(os.path.join(ROOT, "include", "pulsar_gibbs.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    enum = {k: int(v) for k, v in re.findall(r"\bGS_OPT_(\w+)\s*=\s*(\d+)", src)}
    assert {"SWEEP_SCHED", "LAST_SWEEP_SHAPE"} <= set(enum)
    for name, val in enum.items():
        assert getattr(_lib, "OPT_" + name) == val, name
