"""Parameter / basis bookkeeping shared by the Gibbs classes.

The reference repeats this bookkeeping inline in each sampler
(``pulsar_gibbs.py:42-196``, ``pta_gibbs.py:42-178``).  Here it is one set of small
functions with the same observable results -- parameter names and order, the
vector <-> dict map, prior bounds read from ``str(param)``, and the column indices of
the gw (and ECORR) Fourier blocks inside T -- used by ``PulsarBlockGibbs``,
``PTABlockGibbs`` and ``PulsarArrayGibbs``.
"""
from __future__ import annotations

import re

import numpy as np

_BOUNDS = re.compile(r"\(\s*pmin\s*=\s*([^,]+?)\s*,\s*pmax\s*=\s*([^)]+?)\s*\)")


def expand_names(params):
    """Flat parameter names: ``name`` for a scalar, ``name_0 .. name_{n-1}`` for a vector
    parameter of size n, in the PTA's parameter order (pulsar_gibbs.py:146-155)."""
    out = []
    for p in params:
        out.extend([f"{p.name}_{i}" for i in range(p.size)] if p.size else [p.name])
    return out


def vector_to_dict(params, xs):
    """Parameter vector -> {name: value}: a slice for vector parameters of size > 1, a
    float otherwise (pulsar_gibbs.py:157-164)."""
    widths = [p.size or 1 for p in params]
    starts = np.concatenate([[0], np.cumsum(widths)])
    return {p.name: (xs[s:s + w] if w > 1 else float(xs[s]))
            for p, s, w in zip(params, starts, widths)}


def matching_indices(names, pred):
    """Positions of the names for which ``pred`` holds (the get_*_indices helpers,
    pulsar_gibbs.py:167-196, pta_gibbs.py:149-178)."""
    return np.array([i for i, n in enumerate(names) if pred(n)])


def last_match(names, pred):
    """Position of the LAST name for which ``pred`` holds, or None (the reference's
    ``for ...: if ...: ind = ct`` scans keep the last hit)."""
    hits = [i for i, n in enumerate(names) if pred(n)]
    return hits[-1] if hits else None


def uniform_bounds(param):
    """(pmin, pmax) parsed from ``str(param)`` = ``'name:Uniform(pmin=a, pmax=b)[n]'`` --
    the reference reads prior bounds from the string form (pulsar_gibbs.py:84-87)."""
    m = _BOUNDS.search(str(param))
    if m is None:
        raise ValueError(f"no Uniform(pmin=..., pmax=...) bounds in {str(param)!r}")
    return float(m.group(1)), float(m.group(2))


def power_bounds(param):
    """Free-spectrum power bounds rho = 10**(2 log10_rho) at the prior edges."""
    lo, hi = uniform_bounds(param)
    return 10 ** (2 * lo), 10 ** (2 * hi)


def basis_layout(signals, keys=None):
    """Walk the PTA's signals in order and place each basis block in T
    (pulsar_gibbs.py:89-105, pta_gibbs.py:96-109): blocks of signals without a basis
    take no columns, and signals keyed with 'red' share the gw Fourier columns (they
    take none of their own).  Returns (gwid, ecid, b_param_names, n_columns); gwid /
    ecid are the columns of the last signal whose NAME contains 'gw' / 'ecorr'."""
    keys = list(signals) if keys is None else list(keys)
    gwid = ecid = None
    names = []
    col = 0
    for key in keys:
        sig = signals[key]
        F = sig.get_basis()
        width = 0 if F is None else F.shape[1]
        here = col + np.arange(width)
        if "gw" in sig.name:
            gwid = here
        if "ecorr" in sig.name:
            ecid = here
        if F is not None and "red" not in key:
            names.extend(f"{key}_{i}" for i in range(width))
            col += width
    return gwid, ecid, names, col
