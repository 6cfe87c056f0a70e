"""Minimal enterprise-compatible PTA facade + synthetic pulsar-timing arrays.

The Gibbs samplers consume an enterprise ``PTA`` duck-typed (SURVEY.md §8b,
"PTA contract consumed").  enterprise/tempo2 are not installed here or on the
GPU box, so this module restates the parts of that contract the sampler
touches:

* ``Uniform`` parameters whose ``str()`` is ``"name:Uniform(pmin=a, pmax=b)[n]"``
  -- the reference parses prior bounds out of that string
  (``pulsar_gibbs.py:84-87``, ``pta_gibbs.py:83-94``);
* Fourier GP signals (sin at even, cos at odd columns, f_k = k/Tspan), with a
  free-spectrum PSD ``phi = repeat(10**(2*log10_rho), 2)`` or a power-law PSD;
  GP signals on the same frequencies share basis columns and their phi add
  (the reference assumes this: ``pulsar_gibbs.py:101-103``);
* a timing-model GP with phi = 1e40 (phiinv = 1e-40) on an orthonormalised
  (``use_svd``) or column-normalised design matrix;
* white noise ``N = efac^2 sigma^2 + 10**(2 log10_tnequad)``;
* the PTA getters ``get_residuals/get_basis/get_ndiag/get_phiinv`` (lists,
  one entry per pulsar), ``params`` sorted by name, ordered ``signals``.

The enterprise behaviours restated here are *[upstream, not vendored]*; the
reference consumes them only through T, N, phiinv and r, which
is where parity is pinned.
"""
from __future__ import annotations

import os
from collections import OrderedDict

import numpy as np

FYR = 1.0 / (365.25 * 86400.0)
DAY = 86400.0
_DATA = os.path.join(os.path.dirname(__file__), "data", "simulated_array.npz")


# --------------------------------------------------------------------------- params
class Uniform:
    """Uniform prior parameter (scalar or vector of ``size``)."""

    def __init__(self, name, pmin, pmax, size=None, rng=None):
        self.name = name
        self.pmin = pmin
        self.pmax = pmax
        self.size = size
        self._rng = rng if rng is not None else np.random.default_rng(12345)

    @property
    def params(self):
        return [self]

    def sample(self):
        v = self._rng.uniform(self.pmin, self.pmax, size=self.size)
        return v if self.size else np.float64(v)

    def get_logpdf(self, value=None, params=None):
        if params is not None:
            value = params[self.name]
        v = np.atleast_1d(np.asarray(value, dtype=float))
        inside = np.all((v >= self.pmin) & (v <= self.pmax))
        return float(-v.size * np.log(self.pmax - self.pmin)) if inside else -np.inf

    def _fmt(self, v):
        return repr(int(v)) if float(v).is_integer() else repr(float(v))

    def __repr__(self):
        s = f"{self.name}:Uniform(pmin={self._fmt(self.pmin)}, pmax={self._fmt(self.pmax)})"
        return s + (f"[{self.size}]" if self.size else "")

    __str__ = __repr__


def _value(params, p):
    v = params[p.name]
    return np.asarray(v, dtype=float)


# --------------------------------------------------------------------------- signals
def fourier_basis(toas_s, n_f, Tspan):
    """sin/cos Fourier design matrix, f_k = k/Tspan, k=1..n_f (sin even, cos odd)."""
    f = np.arange(1, n_f + 1) / Tspan
    arg = 2.0 * np.pi * toas_s[:, None] * f[None, :]
    F = np.empty((toas_s.size, 2 * n_f))
    F[:, ::2] = np.sin(arg)
    F[:, 1::2] = np.cos(arg)
    return F, f


def powerlaw_phi(f, Tspan, log10_A, gamma):
    """enterprise's powerlaw PSD times df.  Far outside any prior (a Metropolis proposal such as
    the reference's PTA jumps of 0.05 len(hind) x 10, pta_gibbs.py:290-295, reaching log10_A ~ 45,
    gamma ~ -40) the direct product overflows to inf x 0 = NaN, and the reference's
    get_lnlikelihood -- which it evaluates BEFORE the prior rejects the point (:298) -- dies in
    cho_factor; those entries are evaluated in log space instead (same value wherever the direct
    form is finite and nonzero)."""
    df = 1.0 / Tspan
    with np.errstate(over="ignore", invalid="ignore", under="ignore"):
        phi = (10.0 ** log10_A) ** 2 / 12.0 / np.pi ** 2 * FYR ** (gamma - 3) * f ** (-gamma) * df
    bad = ~(np.isfinite(phi) & (phi > 0))
    if np.any(bad):
        lphi = (2.0 * np.log(10.0) * log10_A - np.log(12.0 * np.pi ** 2) + (gamma - 3) * np.log(FYR)
                - gamma * np.log(f) + np.log(df))
        phi = np.where(bad, np.exp(np.minimum(lphi, 700.0)), phi)
    return phi


class FourierGP:
    """GP on a Fourier basis with a free-spectrum or power-law PSD."""

    def __init__(self, psrname, name, toas_s, Tspan, n_f, psd="spectrum", params=()):
        self.psrname = psrname
        self.name = name
        self.signal_id = f"{psrname}_{name}"
        self.psd = psd
        self.Tspan = float(Tspan)
        self.n_f = n_f
        self._F, self.freqs = fourier_basis(toas_s, n_f, Tspan)
        self.basis_key = ("fourier", n_f, round(self.Tspan, 3))
        self.params = list(params)

    def get_basis(self, params=None):
        return self._F

    def get_phi(self, params):
        if self.psd == "spectrum":
            rho = _value(params, self.params[0])
            return np.repeat(10.0 ** (2.0 * rho), 2)
        la = _value(params, self.params[0])
        ga = _value(params, self.params[1])
        return np.repeat(powerlaw_phi(self.freqs, self.Tspan, la, ga), 2)


class TimingModelGP:
    """Linear timing model as a GP with an (effectively) improper prior, phi = 1e40."""

    def __init__(self, psrname, M, use_svd=True):
        self.psrname = psrname
        self.name = "linear_timing_model"
        self.signal_id = f"{psrname}_{self.name}"
        if use_svd:
            self._M = np.linalg.svd(M, full_matrices=False)[0]
        else:
            self._M = M / np.linalg.norm(M, axis=0)
        self.basis_key = ("tm", psrname)
        self.params = []

    def get_basis(self, params=None):
        return self._M

    def get_phi(self, params):
        return 1e40 * np.ones(self._M.shape[1])


class MeasurementNoise:
    """White noise: N = efac^2 sigma^2 + 10**(2 log10_tnequad), per backend."""

    def __init__(self, psrname, sigma, backends=None, efac=None, equad=None):
        self.psrname = psrname
        self.name = "measurement_noise"
        self.signal_id = f"{psrname}_{self.name}"
        self.sigma = np.asarray(sigma, dtype=float)
        self.backends = (np.zeros(self.sigma.size, dtype=np.int64) if backends is None
                         else np.asarray(backends, dtype=np.int64))
        self.efac = list(efac or [])     # one Uniform per backend (or empty: efac = 1)
        self.equad = list(equad or [])
        self.params = self.efac + self.equad
        self.basis_key = None

    def get_basis(self, params=None):
        return None

    def get_phi(self, params):
        return None

    def backend_values(self, params):
        nb = int(self.backends.max()) + 1
        ef = np.ones(nb)
        eq = np.zeros(nb)
        for i, p in enumerate(self.efac):
            ef[i] = float(_value(params, p))
        for i, p in enumerate(self.equad):
            eq[i] = 10.0 ** (2.0 * float(_value(params, p)))
        return ef, eq

    def get_ndiag(self, params):
        ef, eq = self.backend_values(params)
        return ef[self.backends] ** 2 * self.sigma ** 2 + eq[self.backends]


def quantization_matrix(toas_s, dt=1.0, nmin=2):
    """Epoch (quantisation) matrix U [n_toa x n_epoch]: TOAs closer than dt seconds to
    the first TOA of their bucket share an epoch; epochs with fewer than nmin TOAs get no
    column (enterprise's create_quantization_matrix, *[upstream, not vendored]*)."""
    order = np.argsort(toas_s, kind="stable")
    buckets, ref = [], None
    for i in order:
        if ref is None or toas_s[i] - ref >= dt:
            buckets.append([i])
            ref = toas_s[i]
        else:
            buckets[-1].append(i)
    buckets = [b for b in buckets if len(b) >= nmin]
    U = np.zeros((toas_s.size, len(buckets)))
    for j, b in enumerate(buckets):
        U[b, j] = 1.0
    return U


class EcorrBasisGP:
    """Basis ECORR (enterprise EcorrBasisModel, selection by backend): one epoch column per
    quantisation bucket of each backend's TOAs, backends in order, phi = 10**(2 log10_ecorr_k)
    for the epochs of backend k.  The reference finds these columns by 'ecorr' in the
    signal name (pulsar_gibbs.py:98-99) and their prior by 'ecorr' in a parameter name
    (:111-118)."""

    def __init__(self, psrname, toas_s, backends, params, dt=1.0, nmin=2):
        self.psrname = psrname
        self.name = "basis_ecorr"
        self.signal_id = f"{psrname}_{self.name}"
        self.params = list(params)
        backends = np.asarray(backends, np.int64)
        cols, ebk = [], []
        for k in range(len(self.params)):
            sel = np.nonzero(backends == k)[0]
            Uk = quantization_matrix(toas_s[sel], dt, nmin)
            full = np.zeros((toas_s.size, Uk.shape[1]))
            full[sel] = Uk
            cols.append(full)
            ebk += [k] * Uk.shape[1]
        self._U = np.hstack(cols)
        self.epoch_backend = np.asarray(ebk, np.int64)
        self.basis_key = ("ecorr", psrname)

    def get_basis(self, params=None):
        return self._U

    def get_phi(self, params):
        v = np.array([10.0 ** (2.0 * float(_value(params, p))) for p in self.params])
        return v[self.epoch_backend]


# --------------------------------------------------------------------------- models
class PulsarModel:
    """Signal collection of one pulsar (enterprise SignalCollection analogue)."""

    def __init__(self, psrname, toas_s, residuals, signals):
        self.psrname = psrname
        self.toas = toas_s
        self.residuals = np.asarray(residuals, dtype=float)
        self.signals = list(signals)
        # column blocks: GP signals with the same basis_key share columns
        self._blocks = OrderedDict()
        for s in self.signals:
            if s.basis_key is None:
                continue
            self._blocks.setdefault(s.basis_key, []).append(s)
        self._T = np.hstack([b[0].get_basis() for b in self._blocks.values()])
        self.white = [s for s in self.signals if isinstance(s, MeasurementNoise)]

    def get_basis(self, params=None):
        return self._T

    def get_phi(self, params):
        return np.concatenate([np.sum([s.get_phi(params) for s in sigs], axis=0)
                               for sigs in self._blocks.values()])

    def get_ndiag(self, params):
        return np.sum([w.get_ndiag(params) for w in self.white], axis=0)


class PTA:
    """enterprise-``PTA``-shaped container over ``PulsarModel`` s."""

    def __init__(self, models):
        self.models = list(models)
        self.pulsars = [m.psrname for m in self.models]
        sig = OrderedDict()
        for m in self.models:
            for s in m.signals:
                sig[s.signal_id] = s
        self._signal_dict = sig
        pars = {}
        for m in self.models:
            for s in m.signals:
                for p in s.params:
                    pars[p.name] = p
        self._params = [pars[k] for k in sorted(pars)]

    @property
    def params(self):
        return list(self._params)

    @property
    def param_names(self):
        out = []
        for p in self._params:
            out += [f"{p.name}_{i}" for i in range(p.size)] if p.size else [p.name]
        return out

    @property
    def signals(self):
        return self._signal_dict

    def map_params(self, xs):
        ret, ct = {}, 0
        for p in self._params:
            n = p.size if p.size else 1
            ret[p.name] = xs[ct:ct + n] if n > 1 else float(xs[ct])
            ct += n
        return ret

    def _as_dict(self, params):
        if isinstance(params, dict):
            return params
        if params is None:
            return None
        flat = np.concatenate([np.atleast_1d(np.asarray(v, dtype=float)) for v in params])
        return self.map_params(flat)

    def get_residuals(self):
        return [m.residuals for m in self.models]

    def get_basis(self, params=None):
        return [m.get_basis() for m in self.models]

    def get_ndiag(self, params=None):
        params = self._as_dict(params) or {}
        return [m.get_ndiag(params) for m in self.models]

    def get_phi(self, params):
        params = self._as_dict(params)
        return [m.get_phi(params) for m in self.models]

    def get_phiinv(self, params, logdet=False):
        phis = self.get_phi(params)
        if logdet:
            return [(1.0 / p, float(np.sum(np.log(p)))) for p in phis]
        return [1.0 / p for p in phis]


# --------------------------------------------------------------------------- data
def load_simulated_array():
    """The 45 simulated pulsars (TOA epochs in MJD, errors in us, n fitted params)."""
    d = np.load(_DATA, allow_pickle=False)
    names = [str(n) for n in d["names"]]
    out = OrderedDict()
    o = d["offsets"]
    for i, n in enumerate(names):
        out[n] = dict(mjd=d["mjd"][o[i]:o[i + 1]], err_us=d["err_us"][o[i]:o[i + 1]],
                      nfit=int(d["nfit"][i]), pb_days=float(d["pb_days"][i]))
    return out


def synthetic_design_matrix(toas_s, n_cols, pb_days=0.0):
    """Deterministic stand-in for a tempo2 design matrix (offset, spin, astrometry, binary)."""
    t = toas_s - toas_s.mean()
    tn = t / np.max(np.abs(t))
    wy = 2.0 * np.pi * FYR
    pb = pb_days * DAY if pb_days > 0 else 0.4 / FYR  # isolated: a slow extra harmonic
    wb = 2.0 * np.pi / pb
    cols = [np.ones_like(t), tn, tn ** 2,
            np.sin(wy * t), np.cos(wy * t), tn * np.sin(wy * t), tn * np.cos(wy * t),
            np.sin(2 * wy * t), np.cos(2 * wy * t),
            np.sin(wb * t), np.cos(wb * t), np.sin(2 * wb * t), np.cos(2 * wb * t),
            tn * np.sin(wb * t), tn * np.cos(wb * t), tn ** 3,
            np.sin(3 * wb * t), np.cos(3 * wb * t), tn ** 4, np.sin(3 * wy * t)]
    if n_cols > len(cols):
        # DMX-like columns beyond the 20 smooth ones: indicators of consecutive windows with
        # equal TOA counts (window 0 left out: the windows would otherwise sum to the offset)
        n_win = n_cols - len(cols) + 1
        rank = np.argsort(np.argsort(toas_s, kind="stable"), kind="stable")
        win = (rank * n_win) // toas_s.size
        if n_win > toas_s.size // 2:
            raise ValueError("too many DMX-like windows for the TOAs")
        cols = cols + [(win == k).astype(float) for k in range(1, n_win)]
    return np.stack(cols[:n_cols], axis=1)


def _simulate_residuals(rng, F, f, Tspan, M, sigma, log10_A, gamma, red=None):
    phi = np.repeat(powerlaw_phi(f, Tspan, log10_A, gamma), 2)
    if red is not None:
        phi = phi + np.repeat(powerlaw_phi(f, Tspan, red[0], red[1]), 2)
    a = rng.standard_normal(F.shape[1]) * np.sqrt(phi)
    c = rng.standard_normal(M.shape[1]) * 1e-8
    return F @ a + M @ c + sigma * rng.standard_normal(sigma.size)


def single_pulsar_pta(psr="J1713+0747", n_f=30, rho_prior=(-9.0, -4.0), log10_A=np.log10(2e-15),
                      gamma=13.0 / 3.0, seed=0, tm_svd=True, n_toa=None, efac_vary=False,
                      n_backends=1, tm_cols=None, powerlaw_red=False):
    """Config 1 model: ``ef + gw free spectrum + tm`` (singlepulsar…ipynb:137-150).

    Signal order (white, gw, TM) gives T = [F | M] and gwid = 0..2 n_f - 1.
    ``n_toa`` > the data's TOA count synthesises a uniform-cadence pulsar (config 5).
    """
    rng = np.random.default_rng(seed)
    if n_toa is None:
        d = load_simulated_array()[psr]
        mjd, err = d["mjd"], d["err_us"] * 1e-6
        ncol = (d["nfit"] + 1) if tm_cols is None else tm_cols
        pb = d["pb_days"]
    else:
        mjd = np.sort(53000.0 + rng.uniform(0, 15 * 365.25, n_toa))
        err = 10 ** rng.uniform(np.log10(5e-8), np.log10(5e-6), n_toa)
        ncol = 16 if tm_cols is None else tm_cols
        pb = 10 ** rng.uniform(0, 2)
    toas = mjd * DAY
    Tspan = toas.max() - toas.min()
    backends = np.arange(toas.size) % n_backends
    efp = [Uniform(f"{psr}_b{i}_efac", 0.1, 5.0) for i in range(n_backends)] if efac_vary else []
    eqp = [Uniform(f"{psr}_b{i}_log10_tnequad", -8.5, -5.0) for i in range(n_backends)] \
        if efac_vary else []
    white = MeasurementNoise(psr, err, backends, efp, eqp)
    rho = Uniform("gw_log10_rho", rho_prior[0], rho_prior[1], size=n_f)
    gw = FourierGP(psr, "gw", toas, Tspan, n_f, "spectrum", [rho])
    sigs = [white, gw]
    if powerlaw_red:
        la = Uniform("red_log10_A", -20.0, -11.0)
        ga = Uniform("red_gamma", 0.0, 7.0)
        sigs.append(FourierGP(psr, "red", toas, Tspan, n_f, "powerlaw", [la, ga]))
    if ncol > 0:
        tm = TimingModelGP(psr, synthetic_design_matrix(toas, ncol, pb), use_svd=tm_svd)
        sigs.append(tm)
        Mb = tm.get_basis()
    else:
        # tm_cols = 0: the timing model is marginalised analytically outside T
        # (model_definition.py:185-186, MarginalizingTimingModel) -- no basis columns
        Mb = np.zeros((toas.size, 0))
    r = _simulate_residuals(rng, gw.get_basis(), gw.freqs, Tspan, Mb, err, log10_A, gamma)
    return PTA([PulsarModel(psr, toas, r, sigs)])


def ecorr_pulsar_pta(psr="J1713+0747", n_epoch=160, n_sub=(1, 6), n_backends=2, n_f=30,
                     rho_prior=(-9.0, -4.0), ecorr_prior=(-8.5, -5.0), log10_ecorr=-6.3,
                     log10_A=np.log10(2e-15), gamma=13.0 / 3.0, span_yr=15.0, n_tm=16, seed=0,
                     white_vary=False):
    """Single pulsar with basis ECORR (pta_gibbs_freespec.ipynb's
    J1713 model ``model_general(..., white_vary=True, select='backend')`` with fixed
    EFAC/EQUAD): n_epoch observing epochs over span_yr, each recorded by one backend
    (epoch % n_backends) as a burst of n_sub[0]..n_sub[1] sub-band TOAs a few tenths of a
    second apart (single-TOA epochs get no ECORR column, nmin = 2).  Signals in order
    [white, basis_ecorr, gw, tm]: T = [U | F | M], ecid = 0..n_e-1, gwid after.
    Parameters (sorted by name): [``{psr}_b{k}_efac``, ``{psr}_b{k}_log10_tnequad`` with
    ``white_vary``], ``{psr}_basis_ecorr_b{k}_log10_ecorr``, then ``gw_log10_rho`` (n_f).
    Residuals: power-law GWB + TM + white + epoch jitter."""
    rng = np.random.default_rng(seed)
    Tspan0 = span_yr * 365.25 * DAY
    t_ep = np.sort(rng.uniform(0.0, Tspan0, n_epoch)) + 53000.0 * DAY
    nsub = rng.integers(n_sub[0], n_sub[1] + 1, n_epoch)
    toas = np.concatenate([t + 0.2 * np.arange(k) for t, k in zip(t_ep, nsub)])
    backends = np.concatenate([np.full(k, e % n_backends) for e, k in enumerate(nsub)])
    sigma = 10 ** rng.uniform(np.log10(1e-7), np.log10(2e-6), toas.size)
    Tspan = toas.max() - toas.min()
    efp = [Uniform(f"{psr}_b{k}_efac", 0.1, 5.0) for k in range(n_backends)] if white_vary else []
    eqp = [Uniform(f"{psr}_b{k}_log10_tnequad", -8.5, -5.0) for k in range(n_backends)] if white_vary else []
    white = MeasurementNoise(psr, sigma, backends, efp, eqp)
    ep = [Uniform(f"{psr}_basis_ecorr_b{k}_log10_ecorr", *ecorr_prior) for k in range(n_backends)]
    ecorr = EcorrBasisGP(psr, toas, backends, ep)
    rho = Uniform("gw_log10_rho", rho_prior[0], rho_prior[1], size=n_f)
    gw = FourierGP(psr, "gw", toas, Tspan, n_f, "spectrum", [rho])
    tm = TimingModelGP(psr, synthetic_design_matrix(toas, n_tm), use_svd=True)
    r = _simulate_residuals(rng, gw.get_basis(), gw.freqs, Tspan, tm.get_basis(), sigma,
                            log10_A, gamma)
    U = ecorr.get_basis()
    r = r + U @ (rng.standard_normal(U.shape[1]) * 10.0 ** log10_ecorr)
    return PTA([PulsarModel(psr, toas, r, [white, ecorr, gw, tm])])


def array_pta(kind="curn_red", n_f=30, n_psr=None, gw_prior=(-9.0, -4.0), red_prior=(-10.0, -4.0),
              log10_A=np.log10(2e-15), gamma=13.0 / 3.0, seed=0):
    """Config 3/4 models over the simulated array (model_definition.py:184-234 order: TM, CRN, red, white).

    kind = 'curn'      common 'gw_crn' free spectrum only,
           'curn_red'  + per-pulsar 'red_noise' free spectrum on the same basis,
           'curn_plred' + per-pulsar power-law 'red_noise' (log10_A Uniform(-20, -11), gamma
                       Uniform(0, 7): model_definition.py's red_var block / enterprise's
                       powerlaw) on the same basis -- what PTABlockGibbs' default
                       redsample='mh' samples (pta_gibbs.py:278-340),
           'indep'     BASELINE configs[2]: no common process; every pulsar carries its
                       own 'gw' free spectrum ``{psr}_gw_log10_rho`` on its own T_span
                       (config 1's model for each of the 45 pulsars: signals white, gw,
                       TM -> T = [F | M]); ``pulsar_ptas`` splits it into the single-pulsar
                       PTAs that PulsarBlockGibbs takes.
    Common Tspan = the array's span (model_utils.get_tspan) for the CURN kinds.
    """
    if kind == "indep":
        return _indep_array(n_f, n_psr, gw_prior, log10_A, gamma, seed)
    rng = np.random.default_rng(seed)
    data = load_simulated_array()
    names = sorted(data)[: n_psr or len(data)]
    tmin = min(data[n]["mjd"].min() for n in names) * DAY
    tmax = max(data[n]["mjd"].max() for n in names) * DAY
    Tspan = tmax - tmin
    crn = Uniform("gw_crn_log10_rho", gw_prior[0], gw_prior[1], size=n_f)
    models = []
    for n in names:
        d = data[n]
        toas = d["mjd"] * DAY
        err = d["err_us"] * 1e-6
        M = synthetic_design_matrix(toas, d["nfit"] + 1, d["pb_days"])
        tm = TimingModelGP(n, M, use_svd=False)
        gw = FourierGP(n, "gw_crn", toas, Tspan, n_f, "spectrum", [crn])
        sigs = [tm, gw]
        if kind == "curn_red":
            rp = Uniform(f"{n}_red_noise_log10_rho", red_prior[0], red_prior[1], size=n_f)
            sigs.append(FourierGP(n, "red_noise", toas, Tspan, n_f, "spectrum", [rp]))
        elif kind == "curn_plred":
            la = Uniform(f"{n}_red_noise_log10_A", -20.0, -11.0)
            ga = Uniform(f"{n}_red_noise_gamma", 0.0, 7.0)
            sigs.append(FourierGP(n, "red_noise", toas, Tspan, n_f, "powerlaw", [la, ga]))
        elif kind != "curn":
            raise ValueError(f"unknown array kind {kind!r}")
        sigs.append(MeasurementNoise(n, err))
        r = _simulate_residuals(rng, gw.get_basis(), gw.freqs, Tspan, tm.get_basis(), err,
                                log10_A, gamma, red=(-14.5, 3.0) if kind in ("curn_red", "curn_plred") else None)
        models.append(PulsarModel(n, toas, r, sigs))
    return PTA(models)


def _indep_array(n_f, n_psr, gw_prior, log10_A, gamma, seed):
    rng = np.random.default_rng(seed)
    data = load_simulated_array()
    names = sorted(data)[: n_psr or len(data)]
    models = []
    for n in names:
        d = data[n]
        toas = d["mjd"] * DAY
        err = d["err_us"] * 1e-6
        Tspan = toas.max() - toas.min()                      # the pulsar's own span
        rho = Uniform(f"{n}_gw_log10_rho", gw_prior[0], gw_prior[1], size=n_f)
        gw = FourierGP(n, "gw", toas, Tspan, n_f, "spectrum", [rho])
        tm = TimingModelGP(n, synthetic_design_matrix(toas, d["nfit"] + 1, d["pb_days"]), use_svd=True)
        r = _simulate_residuals(rng, gw.get_basis(), gw.freqs, Tspan, tm.get_basis(), err, log10_A, gamma)
        models.append(PulsarModel(n, toas, r, [MeasurementNoise(n, err), gw, tm]))
    return PTA(models)


def pulsar_ptas(pta):
    """One single-pulsar PTA per pulsar of ``pta`` (what PulsarBlockGibbs takes, one
    pulsar's signals and parameters each)."""
    return [PTA([m]) for m in pta.models]


def config5_pulsar_pta(seed=1, n_toa=10_000, n_f=100, n_tm=16, n_bk=4, span_yr=15.0, rho_prior=(-9.0, -4.0),
                       efac_prior=(0.5, 2.0), equad_prior=(-8.5, -5.0), log10_A=np.log10(2e-15), gamma=13.0 / 3.0):
    """One pulsar of BASELINE configs[4] as an enterprise-shaped single-pulsar PTA (the shapes of
    ``config5_array``: 10^4 TOAs, n_bk backends with EFAC / log10 EQUAD, an n_f-bin free spectrum,
    an n_tm-column timing model; signals white, gw, tm -> T = [F | M]), for drivers that take a
    PTA -- e.g. the reference's own PulsarBlockGibbs in tools/calibrate_cpu_baseline.py."""
    rng = np.random.default_rng(seed)
    Tspan = span_yr * 365.25 * DAY
    psr = "C5P0000"
    toas = np.sort(rng.uniform(0.0, Tspan, n_toa))
    sigma = 10 ** rng.uniform(np.log10(0.05e-6), np.log10(5e-6), n_toa)
    bk = np.minimum((np.arange(n_toa) * n_bk) // n_toa, n_bk - 1)
    efp = [Uniform(f"{psr}_b{k}_efac", *efac_prior) for k in range(n_bk)]
    eqp = [Uniform(f"{psr}_b{k}_log10_tnequad", *equad_prior) for k in range(n_bk)]
    white = MeasurementNoise(psr, sigma, bk, efp, eqp)
    rho = Uniform("gw_log10_rho", rho_prior[0], rho_prior[1], size=n_f)
    gw = FourierGP(psr, "gw", toas, Tspan, n_f, "spectrum", [rho])
    tm = TimingModelGP(psr, synthetic_design_matrix(toas, n_tm), use_svd=True)
    ef = rng.uniform(*efac_prior, n_bk)[bk]
    eq = 10 ** rng.uniform(*equad_prior, n_bk)[bk]
    r = _simulate_residuals(rng, gw.get_basis(), gw.freqs, Tspan, tm.get_basis(), np.sqrt(ef ** 2 * sigma ** 2 + eq ** 2),
                            log10_A, gamma)
    return PTA([PulsarModel(psr, toas, r, [white, gw, tm])])


def config5_array(n_psr=200, n_toa=10_000, n_f=100, n_tm=16, n_bk=4, span_yr=15.0, seed=0,
                  rho_prior=(-9.0, -4.0), efac_prior=(0.5, 2.0), equad_prior=(-8.5, -5.0),
                  log10_A=np.log10(2e-15), gamma=13.0 / 3.0):
    """BASELINE configs[4]: n_psr independent synthetic pulsars, each its own
    PulsarBlockGibbs model ``ef/equad per backend + gw free spectrum + tm``
    (SURVEY.md §8d item 5): TOAs uniform over span_yr, sigma log-uniform in
    [0.05, 5] us, n_bk backends per pulsar (contiguous TOA blocks) with true EFAC in
    efac_prior and log10 EQUAD in equad_prior, n_f free-spectrum bins (f_k = k/span),
    an orthonormalised n_tm-column timing model; residuals = power-law red process +
    white noise.  Basis order [F | M] (signal order white, gw, tm), gwid = 0..2 n_f - 1.

    Parameter vector of every pulsar, sorted by name as enterprise does:
    ``{psr}_b{k}_efac, {psr}_b{k}_log10_tnequad`` (k = 0..n_bk-1), then
    ``{psr}_gw_log10_rho`` (n_f) -> white columns 0..2 n_bk - 1, gw columns after.
    Returns dict with per-pulsar lists T, r, sigma, backend and the shared layout
    (fidx, phiinv_fixed, white: [(col, kind, backend, pmin, pmax)], gw_cols, n_param,
    x0 (n_psr, n_param) drawn from the priors, names)."""
    rng = np.random.default_rng(seed)
    Tspan = span_yr * 365.25 * DAY
    T, R, S, B = [], [], [], []
    for p in range(n_psr):
        toas = np.sort(rng.uniform(0.0, Tspan, n_toa))
        sigma = 10 ** rng.uniform(np.log10(0.05e-6), np.log10(5e-6), n_toa)
        bk = np.minimum((np.arange(n_toa) * n_bk) // n_toa, n_bk - 1).astype(np.int32)
        F, f = fourier_basis(toas, n_f, Tspan)
        M = synthetic_design_matrix(toas, n_tm)
        M, _ = np.linalg.qr(M)
        ef = rng.uniform(*efac_prior, n_bk)[bk]
        eq = 10 ** rng.uniform(*equad_prior, n_bk)[bk]
        sig_w = np.sqrt(ef ** 2 * sigma ** 2 + eq ** 2)
        r = _simulate_residuals(rng, F, f, Tspan, M, sig_w, log10_A, gamma)
        T.append(np.ascontiguousarray(np.concatenate([F, M], axis=1)))
        R.append(r)
        S.append(sigma)
        B.append(bk)
    white, names = [], []
    for k in range(n_bk):
        white.append((2 * k, 0, k, *efac_prior))       # efac
        white.append((2 * k + 1, 1, k, *equad_prior))  # log10_tnequad
        names += [f"b{k}_efac", f"b{k}_log10_tnequad"]
    gw_cols = np.arange(2 * n_bk, 2 * n_bk + n_f)
    names += [f"gw_log10_rho_{i}" for i in range(n_f)]
    n_param = 2 * n_bk + n_f
    x0 = np.empty((n_psr, n_param))
    for col, kind, k, lo, hi in white:
        x0[:, col] = rng.uniform(lo, hi, n_psr)
    x0[:, gw_cols] = rng.uniform(*rho_prior, (n_psr, n_f))
    return dict(T=T, r=R, sigma=S, backend=B, fidx=np.arange(2 * n_f), phiinv_fixed=np.full(n_tm, 1e-40),
                white=white, gw_cols=gw_cols, n_param=n_param, x0=x0, names=names,
                rhomin=10 ** (2 * rho_prior[0]), rhomax=10 ** (2 * rho_prior[1]))
