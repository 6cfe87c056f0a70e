"""MI355X-native free-spectrum Gibbs sampler for pulsar-timing arrays.

Drop-in for the hot path of astrolamb/pulsar_timing_gibbsspec: the
``PulsarBlockGibbs`` / ``PTABlockGibbs`` surface (plus ``PulsarArrayGibbs`` for an
array of independent pulsars) over hand-written gfx950 HIP kernels reached through
the C-ABI in ``include/pulsar_gibbs.h``.

The sampler classes are imported on first access (PEP 562), so that the host-only
modules (``synthetic``, ``plumbing``) load without torch or the HIP library.
"""
__version__ = "0.2.0"

_LAZY = {"PulsarBlockGibbs": "pulsar_gibbs", "PTABlockGibbs": "pta_gibbs", "PulsarArrayGibbs": "array_gibbs"}


def __getattr__(name):
    if name in _LAZY:
        import importlib
        return getattr(importlib.import_module(f".{_LAZY[name]}", __name__), name)
    raise AttributeError(f"module {__name__!r} has no attribute {name!r}")


__all__ = sorted(_LAZY)
