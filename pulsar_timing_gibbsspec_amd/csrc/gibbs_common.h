// Shared device helpers for the gfx950 Gibbs kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define GS_WAVE 64

// per-wave LDS scratch (doubles) of the tile b-draw (gibbs_tile.h): 272 transpose /
// factor rows + 64 vector + max(64, 16 NT) output (NT = NF / 16 + 1 <= 5).  Sized per NF,
// not at the 5-tile maximum: the LDS of a k_bdraw workgroup (model block + 4 scratches) sits
// at the 3-workgroups-per-CU edge for the simulated array (NF = 60, NMX = 17: 53320 B at 400
// doubles per wave vs 53832 B at 416), and dropping to 2 workgroups per CU cost 25 %
// (0.665 -> 0.835 ms per launch measured on MI355X).
#define GS_TILE_SCR_MAX 416
__host__ __device__ constexpr int gs_tile_scr(int NF) {
#ifdef GS_PHASE_PROF
  return GS_TILE_SCR_MAX + 8;  // + the phase-profile accumulators at 416..423
#else
  return 336 + (NF / 16 + 1 > 4 ? 16 * (NF / 16 + 1) : 64);  // output: max(64 lanes, 16 NT)
#endif
}

// ---------------------------------------------------------------- intra-wave LDS sync
// Lanes of one wavefront exchanging data through LDS: wavefront-scope release/acquire
// fences around the wave barrier (a bare wave barrier does not order the LDS accesses
// for the compiler backend).
// The wave's index in its workgroup as a wave-uniform SGPR value.  `threadIdx.x >> 6` is uniform
// too, but the compiler's divergence analysis does not know it, so everything derived from it
// (chain, system, pointers) would sit in VGPRs: the 12-wave fused sweep spilled 37 VGPRs that way,
// 6 with this (r04).
__device__ __forceinline__ int gs_wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }
// vmcnt(0) (gfx9 s_waitcnt layout: vmcnt[3:0] + [15:14] = 0, expcnt[6:4] and lgkmcnt[11:8] at their
// maxima): issued by every wave before a barrier that publishes LDS-DMA (global_load_lds) data, so
// the other waves' reads after the barrier see it whatever waits the compiler places around the
// barrier (a workgroup-scope release need not drain vmcnt on gfx9)
__device__ __forceinline__ void gs_wait_dma() { __builtin_amdgcn_s_waitcnt(0x0F70); }

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------------------------------------------------------- cross-lane
// Broadcast lane `l` of a double to every lane (two v_readlane_b32 -> SGPRs).
__device__ __forceinline__ double rdlane(double v, int l) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u & 0xffffffffull), l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// ---------------------------------------------------------------- Philox4x32-10
struct gs_u4 {
  uint32_t x, y, z, w;
};

// GS_PHILOX_MAD: each round's products as one v_mad_u64_u32 (both halves) instead of v_mul_lo_u32 +
// v_mul_hi_u32.  Measured on the headline (r06q): 1.924-1.938 ms per launch against 1.919-1.930 with
// the two multiplies -- not faster, off
#ifndef GS_PHILOX_MAD
#define GS_PHILOX_MAD 0
#endif
__device__ __forceinline__ gs_u4 philox4x32_10(gs_u4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
#if GS_PHILOX_MAD
    // one v_mad_u64_u32 per product (both halves) instead of v_mul_lo_u32 + v_mul_hi_u32
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
    const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
#else
    const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
#endif
    gs_u4 n;
    n.x = hi1 ^ c.y ^ k0;
    n.y = lo1;
    n.z = hi0 ^ c.w ^ k1;
    n.w = lo0;
    c = n;
  }
  return c;
}

// 53-bit uniform in [0,1) from two words (hi first).
__device__ __forceinline__ double gs_u53(uint32_t hi, uint32_t lo) {
  return (double)((((unsigned long long)hi << 32) | lo) >> 11) * 0x1.0p-53;
}

struct gs_key {
  uint32_t k0, k1;
};

__device__ __forceinline__ gs_u4 gs_counter(uint32_t slot, long long sweep, long long chain,
                                            int psr, int event) {
  gs_u4 c;
  c.x = slot;
  c.y = (uint32_t)sweep;
  c.z = (uint32_t)chain;
  c.w = ((uint32_t)psr << 8) | (uint32_t)(event & 0xff);
  return c;
}

// Sweep index of a Philox counter: the launch argument, plus the context's device-side
// sweep counter when one is attached (graph-captured sweeps advance it on the device).
__device__ __forceinline__ long long gs_sweep(int64_t s, const int64_t* dev) {
  return dev ? (long long)(s + *dev) : (long long)s;
}

// Two uniforms in [0,1) for one counter.
__device__ __forceinline__ void gs_uniform2(gs_u4 c, gs_key k, double& u1, double& u2) {
  const gs_u4 w = philox4x32_10(c, k.k0, k.k1);
  u1 = gs_u53(w.x, w.y);
  u2 = gs_u53(w.z, w.w);
}

// ---------------------------------------------------------------- short f64 math
// The hot kernels are VALU-issue bound (k_sweep_freespec: ~1.9k VALU instructions per
// draw), and the libm forms carry double-double corrections for correct rounding that the
// samplers do not need: the draws are compared with the reference at 1e-9.  These are
// within ~2 ulp (tools/probe/fastmath_probe.hip measures them against long double).
// GS_FAST_MATH=0 restores log / sincospi.
#ifndef GS_FAST_MATH
#define GS_FAST_MATH 1
#endif

// 1/x by v_rcp_f64 and two Newton steps (within an ulp of the IEEE quotient)
__device__ __forceinline__ double rcp_nr2(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = fma(r, fma(-x, r, 1.0), r);
  return fma(r, fma(-x, r, 1.0), r);
}

// log(x) for positive normal x (fdlibm's e_log.c reduction and Lg1..Lg7 polynomial, no
// special cases): x = 2^e m, m in [sqrt(1/2), sqrt(2)), f = m - 1 (exact),
// s = f / (2 + f) by v_rcp_f64 + one Newton step (s only enters the O(f^3) correction),
// log x = e ln2_hi - ((hfsq - (s (hfsq + R) + e ln2_lo)) - f).  ~35 VALU vs ~90.
__device__ __forceinline__ double gs_log_pos(double x) {
#if GS_FAST_MATH
  double m = __builtin_amdgcn_frexp_mant(x);  // [0.5, 1)
  int e = __builtin_amdgcn_frexp_exp(x);
  const bool lo = m < 0.70710678118654752440;
  m = lo ? m + m : m;
  e = lo ? e - 1 : e;
  const double f = m - 1.0;
  const double den = 2.0 + f;
  double rd = __builtin_amdgcn_rcp(den);
  rd = fma(rd, fma(-den, rd, 1.0), rd);
  const double s = f * rd, z = s * s, w = z * z;
  const double t1 = w * fma(w, fma(w, 0x1.39a09d078c69fp-3, 0x1.c71c51d8e78afp-3), 0x1.999999997fa04p-2);
  const double t2 =
      z * fma(w, fma(w, fma(w, 0x1.2f112df3e5244p-3, 0x1.7466496cb03dep-3), 0x1.2492494229359p-2),
              0x1.5555555555593p-1);
  const double R = t2 + t1;
  const double hfsq = 0.5 * f * f;
  const double dk = (double)e;
  return fma(dk, 0x1.62e42feep-1, -((hfsq - fma(s, hfsq + R, dk * 0x1.a39ef35793c76p-33)) - f));
#else
  return log(x);
#endif
}

// log of the marginalised likelihood's terms (lnl_terms' pivots, the sum of log phiinv): gs_log_pos,
// or libm's log with GS_LNL_LIBM=1 (A/B builds)
#ifndef GS_LNL_LIBM
#define GS_LNL_LIBM 0
#endif
__device__ __forceinline__ double gs_log_lnl(double x) {
#if GS_LNL_LIBM
  return log(x);
#else
  return gs_log_pos(x);
#endif
}

// exp(x) for x <= 0 (the grid pdfs' exponents; -inf and NaN-free inputs below -800 give 0):
// n = rint(x log2 e), r = x - n ln2 (two-term Cody-Waite), the degree-11 minimax polynomial
// of the device library's exp on |r| <= ln2/2, ldexp.  No overflow / special-case branches
// (x <= 0 by contract, clamped at -800 where exp is 0): ~17 VALU vs ~29.
#ifndef GS_EXP_MAGIC
#define GS_EXP_MAGIC 1
#endif
__device__ __forceinline__ double gs_exp_neg(double x) {
#if GS_FAST_MATH && GS_EXP_MAGIC
  // n by the round-to-integer constant 1.5 2^52 (n sits in the low word of t), 2^n built in
  // the exponent field: no v_rndne / v_cvt / v_ldexp.  x is clamped at -708 so 2^n stays
  // normal: exp(x) < 3.4e-308 below that is returned as exp(-708) -- in the grid pdfs those
  // points are ~1e-308 of the row maximum, below every comparison the draws make.
  x = fmax(x, -708.0);
  const double t = fma(x, 0x1.71547652b82fep+0, 0x1.8p52);
  const double n = t - 0x1.8p52;
  double r = fma(n, -0x1.62e42fefa39efp-1, x);
  r = fma(n, -0x1.abc9e3b39803fp-56, r);
  double p = fma(r, 0x1.ade156a5dcb37p-26, 0x1.28af3fca7ab0cp-22);
  p = fma(r, p, 0x1.71dee623fde64p-19);
  p = fma(r, p, 0x1.a01997c89e6b0p-16);
  p = fma(r, p, 0x1.a01a014761f6ep-13);
  p = fma(r, p, 0x1.6c16c1852b7b0p-10);
  p = fma(r, p, 0x1.1111111122322p-7);
  p = fma(r, p, 0x1.55555555502a1p-5);
  p = fma(r, p, 0x1.5555555555511p-3);
  p = fma(r, p, 0x1.000000000000bp-1);
  p = fma(r, p, 1.0);
  p = fma(r, p, 1.0);
  const int ni = (int)(unsigned)__double_as_longlong(t);  // n (low word of 1.5 2^52 + n)
  return p * __hiloint2double((ni + 1023) << 20, 0);
#elif GS_FAST_MATH
  x = fmax(x, -800.0);
  const double n = __builtin_rint(x * 0x1.71547652b82fep+0);
  double r = fma(n, -0x1.62e42fefa39efp-1, x);
  r = fma(n, -0x1.abc9e3b39803fp-56, r);
  double p = fma(r, 0x1.ade156a5dcb37p-26, 0x1.28af3fca7ab0cp-22);
  p = fma(r, p, 0x1.71dee623fde64p-19);
  p = fma(r, p, 0x1.a01997c89e6b0p-16);
  p = fma(r, p, 0x1.a01a014761f6ep-13);
  p = fma(r, p, 0x1.6c16c1852b7b0p-10);
  p = fma(r, p, 0x1.1111111122322p-7);
  p = fma(r, p, 0x1.55555555502a1p-5);
  p = fma(r, p, 0x1.5555555555511p-3);
  p = fma(r, p, 0x1.000000000000bp-1);
  p = fma(r, p, 1.0);
  p = fma(r, p, 1.0);
  return __builtin_amdgcn_ldexp(p, (int)n);
#else
  return exp(x);
#endif
}

// sin(2 pi u), cos(2 pi u) for u in [0, 1): q = rint(4u), r = u - q/4 in [-1/8, 1/8]
// (exact), Taylor polynomials of sin / cos (2 pi r) in r^2 through r^17 / r^16 (truncation
// < 0.6 ulp), quadrant by swap and sign.  ~30 VALU vs ~60 for sincospi.
__device__ __forceinline__ void gs_sincos2pi(double u, double& sn, double& cs) {
#if GS_FAST_MATH
  const double q = __builtin_rint(4.0 * u);
  const double r = fma(q, -0.25, u);
  const double z = r * r;
  double ps = 0x1.aaec32af93359p-4;
  ps = fma(ps, z, -0x1.6fadb9f155744p-1);
  ps = fma(ps, z, 0x1.e8f434d018d63p+1);
  ps = fma(ps, z, -0x1.e3074fde8871fp+3);
  ps = fma(ps, z, 0x1.50783487ee782p+5);
  ps = fma(ps, z, -0x1.32d2cce62bd86p+6);
  ps = fma(ps, z, 0x1.466bc6775aae2p+6);
  ps = fma(ps, z, -0x1.4abbce625be53p+5);
  ps = fma(ps, z, 0x1.921fb54442d18p+2);
  const double s0 = ps * r;
  double pc = 0x1.20c62c2f2d7f5p-2;
  pc = fma(pc, z, -0x1.b6e24f44b128fp+0);
  pc = fma(pc, z, 0x1.f9d38a3763cc3p+2);
  pc = fma(pc, z, -0x1.a6d1f2a204a8cp+4);
  pc = fma(pc, z, 0x1.e1f506891babbp+5);
  pc = fma(pc, z, -0x1.55d3c7e3cbffap+6);
  pc = fma(pc, z, 0x1.03c1f081b5ac4p+6);
  pc = fma(pc, z, -0x1.3bd3cc9be45dep+4);
  const double c0 = fma(pc, z, 1.0);
  const int qi = (int)q & 3;  // angle = 2 pi r + q pi / 2
  const double a = (qi & 1) ? c0 : s0, b = (qi & 1) ? s0 : c0;
  sn = (qi & 2) ? -a : a;                   // q = 2, 3
  cs = ((qi + 1) & 2) ? -b : b;             // q = 1, 2
#else
  sincospi(2.0 * u, &sn, &cs);
#endif
}

// sqrt(x) for finite x >= 0: x v_rsq_f64(x) with two Newton steps on the reciprocal root (~1 ulp;
// 0 at x = 0) instead of the IEEE sequence's scaling, fixups and class checks (~15 VALU -> 9)
__device__ __forceinline__ double gs_sqrt_nn(double x) {
#if GS_FAST_MATH
  double y = __builtin_amdgcn_rsq(x);
  const double hx = 0.5 * x;
  y = y * fma(-hx * y, y, 1.5);
  y = y * fma(-hx * y, y, 1.5);
  return x > 0.0 ? x * y : 0.0;
#else
  return sqrt(x);
#endif
}

// Two independent standard normals from two uniforms in [0, 1) (Box-Muller).
__device__ __forceinline__ void gs_box_muller(double u1, double u2, double& n1, double& n2) {
  const double r = gs_sqrt_nn(-2.0 * gs_log_pos(1.0 - u1));
  double s, co;
  gs_sincos2pi(u2, s, co);
  n1 = r * co;
  n2 = r * s;
}

// Two independent standard normals (Box-Muller) for one counter.
__device__ __forceinline__ void gs_normal2(gs_u4 c, gs_key k, double& n1, double& n2) {
  double u1, u2;
  gs_uniform2(c, k, u1, u2);
  gs_box_muller(u1, u2, n1, n2);
}

// ---------------------------------------------------------------- separately rounded ops
// a * b and a + b each rounded to nearest, never fused into an fma with a neighbouring operation:
// the reference's numpy arithmetic (tau = b_s^2 + b_c^2, q = x + z sigma scale, ...).  HIP's
// __dmul_rn / __dadd_rn are plain `*` / `+` here and still contract under -ffp-contract=fast; the
// operations carry the no-contract flag only when the pragma is in their own scope.
__device__ __forceinline__ double gs_mul_rn(double a, double b) {
#pragma clang fp contract(off)
  return a * b;
}
__device__ __forceinline__ double gs_add_rn(double a, double b) {
#pragma clang fp contract(off)
  return a + b;
}

// ---------------------------------------------------------------- Metropolis jump scale
// scale = np.random.choice([0.1, 0.5, 1, 3, 10], p=[.1, .15, .5, .15, .1]) of every one-parameter
// MH block of the reference (pulsar_gibbs.py:377-381, 430-433; pta_gibbs.py:290-293): numpy's
// choice draws u and takes searchsorted(cumsum(p), u, side='right').
__device__ __forceinline__ double gs_mh_scale(double u) {
  if (u < 0.1) return 0.1;
  if (u < 0.25) return 0.5;
  if (u < 0.75) return 1.0;
  if (u < 0.9) return 3.0;
  return 10.0;
}

// ---------------------------------------------------------------- numpy npy_logaddexp
__device__ __forceinline__ double np_logaddexp(double x, double y) {
  if (x == y) return x + 0.693147180559945309417232121458176568;  // x + log(2)
  const double t = x - y;
  if (t > 0) return x + log1p(exp(-t));
  if (t <= 0) return y + log1p(exp(t));
  return t;  // NaN
}

