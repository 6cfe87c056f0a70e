"""``PulsarArrayGibbs`` -- BASELINE configs[2]: every pulsar of an array, each with its own
intrinsic free spectrum, sampled at once.

The reference has no array sampler for independent pulsars: a user builds one
``PulsarBlockGibbs`` per pulsar (``pulsar_gibbs.py:42-136``) and calls its ``sample``
(``:620-710``) pulsar after pulsar.  This class keeps exactly that per-pulsar surface
(``.samplers[p]`` IS the pulsar's ``PulsarBlockGibbs``: params, param_names, gwid,
rhomin/rhomax, chain, bchain, _b) and that per-pulsar output (``outdir/<pulsar>/``:
pars_chain.txt, pars_bchain.txt, chain.npy, bchain.npy), but runs the sweeps of all
pulsars and all chains in ONE persistent fused launch (``gs_sweep_freespec`` over the
ragged (pulsar, chain) systems, m = 68..77 for the simulated array).

Multi-GPU: pulsars are independent, so ranks split them (``shard_pulsars``: contiguous
blocks balanced by m^3, the b|rho cost) with no collective.  Each pulsar's Philox
stream is keyed by its GLOBAL index (``psr_base``), so a sharded run reproduces the
unsharded chains bit for bit.
"""
from __future__ import annotations

import os

import numpy as np

from . import _lib
from .engine import DeviceModel
from .pulsar_gibbs import PulsarBlockGibbs, resolve_seed, sample_free_spectrum


def balanced_blocks(weights, world):
    """Contiguous [lo, hi) blocks, one per rank, with ~equal sums of ``weights`` (every
    rank keeps at least one item)."""
    w = np.asarray(weights, float)
    cw = np.concatenate([[0.0], np.cumsum(w)])
    cuts = [int(np.searchsorted(cw, cw[-1] * r / world)) for r in range(world + 1)]
    cuts[0], cuts[-1] = 0, len(w)
    for r in range(1, world):
        cuts[r] = min(max(cuts[r], cuts[r - 1] + 1), len(w) - (world - r))
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def shard_pulsars(ptas, rank, world):
    """(lo, hi): this rank's contiguous block of the single-pulsar PTAs, balanced by m^3."""
    if world > len(ptas):
        raise ValueError(f"{world} ranks for {len(ptas)} pulsars")
    m = [p.get_basis()[0].shape[1] for p in ptas]
    return balanced_blocks(np.asarray(m, float) ** 3, world)[rank]


class PulsarArrayGibbs(object):
    """PulsarBlockGibbs on every pulsar of an array, all (pulsar, chain) systems batched.

    ptas: one single-pulsar PTA per pulsar (e.g. ``synthetic.pulsar_ptas(pta)``);
    psr_base: global index of ptas[0] (pulsar-sharded runs: the rank's block start).
    Keyword extensions as PulsarBlockGibbs: nchains (per pulsar), device, seed."""

    def __init__(self, ptas, hypersample="conditional", *, nchains=1, device=0, seed=None, psr_base=0):
        self.seed, self._key = resolve_seed(seed)
        self._device = device
        self._ctx = None
        self.nchains = int(nchains)
        self.psr_base = int(psr_base)
        self.samplers = [PulsarBlockGibbs(p, hypersample, nchains=nchains, device=device, seed=self.seed)
                         for p in ptas]
        self.pulsars = [s.pulsar_name for s in self.samplers]
        s0 = self.samplers[0]
        for s in self.samplers:
            if (s.rhomin, s.rhomax) != (s0.rhomin, s0.rhomax):
                raise NotImplementedError("pulsars with different free-spectrum priors")
            if len(s.gwid) != len(s0.gwid):
                raise NotImplementedError("pulsars with different numbers of free-spectrum bins")
            # one fused free-spectrum sweep for all pulsars: every pulsar must be free-spectrum
            # only (no red / ECORR / white Metropolis block, every parameter a gw rho)
            if (s._red_loop() or s._ecorr_loop() or s._white_loop() or s.red_sig is not None
                    or s.hypersample != "conditional" or len(s.param_names) != len(s.gwid) // 2):
                raise NotImplementedError(
                    f"{s.pulsar_name}: PulsarArrayGibbs runs free-spectrum-only pulsars (analytic rho|b); "
                    "sample pulsars with red-noise, ECORR or white-noise blocks with PulsarBlockGibbs")

    @property
    def ctx(self):
        if self._ctx is None:
            self._ctx = _lib.Context(self._device, seed=self._key)
            for s in self.samplers:
                s._ctx = self._ctx
        return self._ctx

    def _model(self, xs_list):
        T, N, R, fixed = [], [], [], []
        for s, xs in zip(self.samplers, xs_list):
            s._check_device_loop(xs)
            params = s.map_params(xs)
            T.append(s.pta.get_basis(params)[0])
            N.append(s.pta.get_ndiag(params)[0])
            R.append(s._residuals)
            ph = s.pta.get_phiinv(params, logdet=False)[0]
            mask = np.ones(ph.size, bool)
            mask[s.gwid] = False
            fixed.append(ph[mask])
        return DeviceModel(self.ctx, T, N, R, [s.gwid for s in self.samplers], fixed)

    def sample(self, xs_list, outdir="./", niter=10000, resume=False, save_every=100, record_bchains=None):
        """Every pulsar's PulsarBlockGibbs.sample (pulsar_gibbs.py:620-710) at once.
        xs_list[p]: pulsar p's initial parameter vector.  Pulsar p writes to
        ``outdir/<pulsar name>/``.  Returns the list of chain-0 chains."""
        if len(xs_list) != len(self.samplers):
            raise ValueError(f"{len(xs_list)} initial vectors for {len(self.samplers)} pulsars")
        outdirs = [os.path.join(outdir, n) for n in self.pulsars]
        for s, o in zip(self.samplers, outdirs):
            print(f"Creating chain directory: {o}")
            os.makedirs(o, exist_ok=True)
            np.savetxt(f"{o}/pars_chain.txt", s.param_names, fmt="%s")
            np.savetxt(f"{o}/pars_bchain.txt", s.b_param_names, fmt="%s")
        model = self._model(xs_list)
        self._runner = sample_free_spectrum(self.samplers, model, xs_list, outdirs, niter, resume, save_every,
                                            psr_base=self.psr_base, record_bchains=record_bchains)
        return [s.chain for s in self.samplers]
