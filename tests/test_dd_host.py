"""The double-double header of the prefix kernels (csrc/gibbs_dd.h), compiled for the HOST with
g++ and checked against mpmath (CPU; no GPU, nothing under oracle/ involved).

The same header is what gibbs_prefix.hip's k_tnt_dd / k_prefix_dd use on the device; this
pins its arithmetic (two-sum, two-product, div, sqrt, the Dot2 accumulator) and a serial
port of the Schur-complement recurrence to ~1e-30, independent of the GPU compiler.  The
device-side consequence of a broken contraction setting was exactly such a silent loss
(DESIGN.md §3.0), caught on the GPU by test_tnt_dd_and_prefix_dd_accuracy.
"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

mp = pytest.importorskip("mpmath")

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "pulsar_timing_gibbsspec_amd", "csrc", "gibbs_dd.h")

HARNESS = r"""
#include <cmath>
using std::fma; using std::sqrt; using std::log;
#define __device__
#define __forceinline__ inline
#include "gibbs_dd_host.h"
#include <vector>
extern "C" {
void dd_ops(const double* a, const double* b, double* out) {   // a, b: (hi, lo)
  gs_dd x = {a[0], a[1]}, y = {b[0], b[1]};
  gs_dd r[5] = {dd_add(x, y), dd_mul(x, y), dd_div(x, y), dd_sqrt(x), dd_mul_d(x, b[0])};
  for (int i = 0; i < 5; ++i) { out[2 * i] = r[i].hi; out[2 * i + 1] = r[i].lo; }
}
void dot2(int n, const double* ah, const double* al, const double* bh, const double* bl, double* out) {
  gs_dot2 s;
  for (int i = 0; i < n; ++i) s.fma_dd(gs_dd{ah[i], al[i]}, gs_dd{bh[i], bl[i]});
  gs_dd r = s.get(); out[0] = r.hi; out[1] = r.lo;
}
// k_prefix_dd's recurrence (serial): S0 = A_FF - W^T W, W = L^-1 A_MF, A_MM = L L^T; A row-major
// m x m (hi, lo) with the nM fixed columns first
void schur(int m, int nM, const double* A, const double* Al, double* S0) {
  const int NF = m - nM;
  std::vector<double> Lh(nM * nM, 0.0), Ll(nM * nM, 0.0), Wh(nM * NF), Wl(nM * NF);
  std::vector<gs_dd> ri(nM);
  auto L = [&](int i, int j) -> gs_dd { return {Lh[i * nM + j], Ll[i * nM + j]}; };
  for (int i = 0; i < nM; ++i)
    for (int j = 0; j <= i; ++j) { Lh[i * nM + j] = A[i * m + j]; Ll[i * nM + j] = Al[i * m + j]; }
  for (int k = 0; k < nM; ++k) {
    gs_dd s = dd_sqrt(L(k, k)); Lh[k * nM + k] = s.hi; Ll[k * nM + k] = s.lo;
    ri[k] = dd_div(gs_dd{1.0, 0.0}, s);   // k_prefix_dd: divisions as products with 1 / L_kk
    for (int i = k + 1; i < nM; ++i) { gs_dd v = dd_mul(L(i, k), ri[k]); Lh[i * nM + k] = v.hi; Ll[i * nM + k] = v.lo; }
    for (int i = k + 1; i < nM; ++i)
      for (int j = k + 1; j <= i; ++j) {
        gs_dd v = dd_sub(L(i, j), dd_mul(L(i, k), L(j, k))); Lh[i * nM + j] = v.hi; Ll[i * nM + j] = v.lo; }
  }
  for (int f = 0; f < NF; ++f)
    for (int i = 0; i < nM; ++i) {
      gs_dot2 s; s.init({A[i * m + nM + f], Al[i * m + nM + f]});
      for (int j = 0; j < i; ++j) s.fma_dd(dd_neg(L(i, j)), gs_dd{Wh[j * NF + f], Wl[j * NF + f]});
      gs_dd w = dd_mul(s.get(), ri[i]); Wh[i * NF + f] = w.hi; Wl[i * NF + f] = w.lo;
    }
  for (int f = 0; f < NF; ++f)
    for (int g = 0; g < NF; ++g) {
      gs_dot2 s; s.init({A[(nM + f) * m + nM + g], Al[(nM + f) * m + nM + g]});
      for (int i = 0; i < nM; ++i)
        s.fma_dd(gs_dd{-Wh[i * NF + f], -Wl[i * NF + f]}, gs_dd{Wh[i * NF + g], Wl[i * NF + g]});
      gs_dd r = s.get(); S0[2 * (f * NF + g)] = r.hi; S0[2 * (f * NF + g) + 1] = r.lo;
    }
}
}
"""


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    d = tmp_path_factory.mktemp("dd")
    src = open(HDR).read().replace("#include <hip/hip_runtime.h>", "").replace("#pragma once", "")
    (d / "gibbs_dd_host.h").write_text(src)
    (d / "h.cpp").write_text(HARNESS)
    so = d / "libdd.so"
    # default contraction for g++ on x86-64 without -mfma is off; make it explicit either way
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-ffp-contract=off", "-Wno-unknown-pragmas",
                    "-o", str(so), str(d / "h.cpp")], check=True, cwd=d)
    return C.CDLL(str(so))


def _P(a):
    return a.ctypes.data_as(C.c_void_p)


def _mp(h, lo):
    return mp.mpf(float(h)) + mp.mpf(float(lo))


def _split(x):
    h = float(x)
    return h, float(x - h)


def test_dd_primitives_against_mpmath(lib):
    mp.mp.dps = 60
    rng = np.random.default_rng(1)
    worst = 0.0
    for _ in range(200):
        ah, bh = rng.uniform(0.1, 10, 2) * 10.0 ** rng.integers(-8, 8, 2)
        a = np.array([ah, ah * rng.uniform(-1, 1) * 2 ** -53])
        b = np.array([bh, bh * rng.uniform(-1, 1) * 2 ** -53])
        out = np.zeros(10)
        lib.dd_ops(_P(a), _P(b), _P(out))
        x, y = _mp(*a), _mp(*b)
        want = [x + y, x * y, x / y, mp.sqrt(x), x * mp.mpf(float(b[0]))]
        for i, w in enumerate(want):
            worst = max(worst, float(abs(_mp(out[2 * i], out[2 * i + 1]) - w) / abs(w)))
    assert worst < 1e-30, worst


def test_dot2_against_mpmath(lib):
    mp.mp.dps = 60
    rng = np.random.default_rng(2)
    n = 10_000
    ah, bh = rng.standard_normal(n), rng.standard_normal(n)
    al, bl = ah * rng.uniform(-1, 1, n) * 2 ** -53, bh * rng.uniform(-1, 1, n) * 2 ** -53
    out = np.zeros(2)
    lib.dot2(n, _P(ah), _P(al), _P(bh), _P(bl), _P(out))
    want = mp.fsum(_mp(ah[i], al[i]) * _mp(bh[i], bl[i]) for i in range(n))
    # a sum with cancellation: relative to the sum of |terms|
    scale = mp.fsum(abs(_mp(ah[i], al[i]) * _mp(bh[i], bl[i])) for i in range(n))
    assert float(abs(_mp(*out) - want) / scale) < 1e-30


def test_schur_recurrence_against_mpmath(lib):
    """A_MM well conditioned, A_FF nearly absorbed by A_FM A_MM^-1 A_MF (the timing model
    absorbing the low frequencies): fp64 loses digits, the double-double recurrence does not."""
    mp.mp.dps = 60
    rng = np.random.default_rng(3)
    nM, NF, n = 6, 8, 40
    T = rng.standard_normal((n, nM + NF))
    T[:, nM:] += T[:, :nM] @ rng.standard_normal((nM, NF)) * 30.0   # F columns mostly in span(M)
    A = T.T @ T
    A = (A + A.T) / 2
    m = nM + NF
    Al = np.zeros_like(A)
    S0 = np.zeros(2 * NF * NF)
    lib.schur(m, nM, _P(np.ascontiguousarray(A)), _P(Al), _P(S0))
    Am = mp.matrix([[mp.mpf(float(A[i, j])) for j in range(m)] for i in range(m)])
    AMM = Am[:nM, :nM]
    want = mp.matrix(NF, NF)
    X = [mp.lu_solve(AMM, Am[:nM, nM + f]) for f in range(NF)]
    for f in range(NF):
        for g in range(NF):
            want[f, g] = Am[nM + f, nM + g] - mp.fsum(Am[k, nM + f] * X[g][k] for k in range(nM))
    got = np.array([[float(_mp(S0[2 * (f * NF + g)], S0[2 * (f * NF + g) + 1]) - want[f, g])
                     for g in range(NF)] for f in range(NF)])
    wmax = max(abs(want[f, g]) for f in range(NF) for g in range(NF))
    cancel = float(np.max(np.abs(A[nM:, nM:])) / wmax)
    assert cancel > 100                                  # the case is cancellation-heavy
    assert float(np.max(np.abs(got)) / wmax) < 1e-26     # fp64 would be ~cancel x 1e-16
