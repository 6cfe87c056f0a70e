"""ctypes binding of the C-ABI in ``include/pulsar_gibbs.h``.

The library is built in-tree (``libpulsar_gibbs.so`` next to this file, see
``csrc/Makefile``).  ``torch`` is imported first so that the HIP runtime torch
bundles (soname ``libamdhip64.so.7``) is the one the library binds to: device
pointers and stream handles are then shared with torch.

There is no CPU fallback: if the library is missing or no GPU is visible, every
entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  (must precede the CDLL load; see module docstring)

LIB_PATH = os.environ.get("GS_LIB_PATH") or \
    os.path.join(os.path.dirname(os.path.abspath(__file__)), "libpulsar_gibbs.so")

OPT_BCAST = 1
OPT_PSR_BASE = 2
OPT_X_PER_SYS = 3
OPT_GRID_EXACT = 4
OPT_BREC_CHAINS = 5
OPT_PHI_PER_CHAIN = 6
OPT_SWEEP_SCHED = 7
OPT_DEBUG_HANDOFF = 8
OPT_LAST_SWEEP_SHAPE = 9
EV_B0, EV_RHO, EV_B, EV_RED, EV_CURN, EV_GUMBEL, EV_WHITE, EV_REDMH, EV_USER = 1, 2, 3, 4, 5, 6, 7, 8, 16
EV_ECORR, EV_ECORR_B, EV_ECORR_B0, EV_HYPER = 9, 10, 11, 12

_P = C.c_void_p
_I = C.c_int
_I64 = C.c_int64
_D = C.c_double

# name -> (restype, argtypes)
SIGNATURES = {
    "gs_version": (_I, []),
    "gs_build_info": (C.c_char_p, []),
    "gs_last_error": (C.c_char_p, []),
    "gs_ctx_create": (_I, [_I, C.c_uint64, _P, C.POINTER(_P)]),
    "gs_ctx_destroy": (_I, [_P]),
    "gs_ctx_set_stream": (_I, [_P, _P]),
    "gs_ctx_set_seed": (_I, [_P, C.c_uint64]),
    "gs_ctx_set_option": (_I, [_P, _I, _I]),
    "gs_ctx_get_option": (_I, [_P, _I]),
    "gs_model_stride": (_I64, [_I, _I]),
    "gs_sweep_lds_bytes": (_I, [_I, _I]),
    "gs_tnt": (_I, [_P, _I, _I, _P, _P, _P, _P, _P, _P]),
    "gs_prefix": (_I, [_P, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P]),
    "gs_bdraw": (_I, [_P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _I64, _I, _I64, _P, _P, _P]),
    "gs_model_tiled_stride": (_I64, [_I, _I]),
    "gs_model_tile": (_I, [_P, _I, _I, _I, _P, _P, _P]),
    "gs_bdraw_tiled": (_I, [_P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _I64, _I, _I64, _P, _P, _P]),
    "gs_rho_analytic": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _I64, _I64, _D, _D, _P, _I]),
    "gs_sweep_freespec": (_I, [_P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _D, _D, _I64, _P, _P,
                               _I64, _I, _P, _P, _P, _P, _P, _P]),
    "gs_philox": (_I, [_P, _I64, _P, _P]),
    "gs_tau": (_I, [_P, _I, _I, _I, _I, _P, _P, _I, _P]),
    "gs_rho_curn": (_I, [_P, _I, _I, _I, _P, _P, _I, _P, _P, _I64, _I64, _P, _I, _P, _P]),
    "gs_rho_red": (_I, [_P, _I, _I, _I, _P, _P, _I, _P, _P, _I64, _I64, _P, _I, _P, _P]),
    "gs_tau_sum": (_I, [_P, _I, _I, _I, _P, _P]),
    "gs_tau_sum_fx": (_I, [_P, _I, _I, _I, _P, _I, _P, _P]),
    "gs_tau_sum_fx_b": (_I, [_P, _I, _I, _I, _I, _P, _P, _I, _P, _P]),
    "gs_fx_to_double": (_I, [_P, _I64, _I, _P, _P]),
    "gs_ctx_set_sweep_counter": (_I, [_P, _P]),
    "gs_counter_add": (_I, [_P, _P, _I64]),
    "gs_ctx_set_fail_counts": (_I, [_P, _P]),
    "gs_ctx_set_grid_fallback_counter": (_I, [_P, _P]),
    "gs_ctx_set_bdraw_lnl": (_I, [_P, _P, _P]),
    "gs_lnlike_marg": (_I, [_P, _I, _I, _I, _I, _P, _I, _P, _P, _P, _P]),
    "gs_lnlike_marg_gated": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P]),
    "gs_rho_curn_sum": (_I, [_P, _I, _I, _I, _P, _I, _P, _P, _I64, _I64, _P, _I, _P, _P]),
    "gs_rho_gumbel": (_I, [_P, _I, _I, _P, _P, _I, _P, _P, _I64, _I64, _P, _I, _P, _P]),
    "gs_phi_from_x": (_I, [_P, _I, _I, _P, _I, _P, _P]),
    "gs_pta_record": (_I, [_P, _I, _I, _P, _P, _P]),
    "gs_pta_gate_phiinv": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P]),
    "gs_pta_gate_phiinv_irn": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P]),
    "gs_phi_powerlaw": (_I, [_P, _I, _I, _I, _P, _I, _P, _P, _P]),
    "gs_hyper_mh": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _I, _P, _I, _P, _P, _P, _P, _I, _P, _P, _P, _P, _I,
                         _I64, _I64, _P, _P, _P]),
    "gs_prefix_sys": (_I, [_P, _I, _I, _I, _I, _P, _I64, _I64, _P, _P, _P, _P, _P, _P, _P]),
    "gs_tnt_dd": (_I, [_P, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P]),
    "gs_prefix_dd": (_I, [_P, _I, _I, _I, _I, _P, _I64, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "gs_bdraw_sys": (_I, [_P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _I64, _I, _I64, _P, _P, _P]),
    "gs_white_resid": (_I, [_P, _I, _I, _I64, _I, _P, _P, _P, _P, _I64, _P]),
    "gs_white_mh": (_I, [_P, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _P, _I, _I, _P, _I64, _I64,
                         _P, _P, _P]),
    "gs_red_mh": (_I, [_P, _I, _I, _I, _I, _P, _I, _P, _P, _P, _P, _P, _P, _I, _I64, _I64, _P, _P, _P]),
    "gs_gate_phiinv_irn": (_I, [_P, _I, _I, _I, _P, _P, _P, _P, _P, _P]),
    "gs_white_tnt": (_I, [_P, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I64, _I64, _P, _P]),
    "gs_ecorr_schur": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _I, _P, _P, _I, _P, _P, _P, _P, _P]),
    "gs_ecorr_prefix": (_I, [_P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _I, _P, _P, _I, _P, _P, _P, _P, _P, _P,
                             _I64, _I64, _I64]),
    "gs_ecorr_lnl_state": (_I, [_P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _I, _P, _P, _P, _P, _P, _I, _P, _P, _P,
                                _P, _P, _P, _P, _I64, _I64, _I64]),
    "gs_ecorr_epoch_sums": (_I, [_P, _I, _P, _P, _P, _P, _P, _I, _P, _I, _P, _P, _P, _I, _I, _I, _P, _P, _P, _P,
                                 _P, _P]),
    "gs_ecorr_gather": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _I64, _P, _I64, _P, _P, _P]),
    "gs_ecorr_propose": (_I, [_P, _I, _I, _P, _P, _P, _P, _I, _I, _P, _I, _I64, _I64, _P, _P]),
    "gs_ecorr_accept": (_I, [_P, _I, _I, _P, _I, _P, _P, _P, _P, _P, _P, _P, _I, _P, _P, _P]),
    "gs_ecorr_accept_propose": (_I, [_P, _I, _I, _P, _I, _P, _P, _P, _P, _P, _P, _P, _I, _P, _P, _P,
                                     _P, _P, _I, _I, _I64, _I64, _P]),
    "gs_ecorr_accept_propose2": (_I, [_P, _I, _I, _P, _I, _P, _P, _P, _P, _P, _P, _P, _I, _P, _P, _P,
                                      _P, _P, _I, _I, _I64, _I64, _P, _P]),
    "gs_ecorr_bdraw_e": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _I, _P, _I, _P, _P, _I, _P, _I64, _I,
                              _I64, _P, _P, _I, _I64, _I64, _I, _P]),
}

_lib = None


class GibbsLibError(RuntimeError):
    pass


def load():
    """Load (once) and return the CDLL with typed signatures."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise GibbsLibError(
            f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc, gfx950). There is no CPU fallback.")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc, what):
    if rc != 0:
        msg = load().gs_last_error().decode(errors="replace")
        raise GibbsLibError(f"{what} failed ({rc}): {msg}")


def ptr(t):
    """Device-accessible pointer of a tensor (or None -> NULL): device memory, or pinned
    (page-locked, device-mapped) host memory, which kernels read and write over PCIe."""
    if t is None:
        return None
    if not t.is_cuda and not t.is_pinned():
        raise GibbsLibError("expected a device tensor (or pinned host memory)")
    if not t.is_contiguous():
        raise GibbsLibError("expected a contiguous tensor")
    return C.c_void_p(t.data_ptr())


class Context:
    """A ``gs_ctx``: device, Philox seed and the stream every call runs on."""

    def __init__(self, device=0, seed=0, stream=None):
        if not torch.cuda.is_available():
            raise GibbsLibError("no GPU visible: the HIP path has no CPU fallback")
        self.lib = load()
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        self.seed = int(seed)
        with torch.cuda.device(self.device):
            s = stream if stream is not None else torch.cuda.current_stream(self.device)
        self.stream = s
        h = C.c_void_p()
        check(self.lib.gs_ctx_create(self.device.index or 0, C.c_uint64(self.seed),
                                     C.c_void_p(s.cuda_stream), C.byref(h)), "gs_ctx_create")
        self.handle = h

    def set_seed(self, seed):
        self.seed = int(seed)
        check(self.lib.gs_ctx_set_seed(self.handle, C.c_uint64(self.seed)), "gs_ctx_set_seed")

    def set_option(self, option, value):
        check(self.lib.gs_ctx_set_option(self.handle, int(option), int(value)), "gs_ctx_set_option")

    def get_option(self, option):
        return int(self.lib.gs_ctx_get_option(self.handle, int(option)))

    def set_stream(self, stream):
        self.stream = stream
        check(self.lib.gs_ctx_set_stream(self.handle, C.c_void_p(stream.cuda_stream)), "gs_ctx_set_stream")

    def close(self):
        if getattr(self, "handle", None) is not None:
            self.lib.gs_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
