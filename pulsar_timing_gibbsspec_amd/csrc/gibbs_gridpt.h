// Per-grid-point work of the red-noise grid conditional (default mode), shared by
// k_rho_red_wave (gibbs_grid.hip) and the ceiling probe (tools/probe/grid_probe.hip), so the
// probe prices exactly the kernel's op mix.
#pragma once
#include "gibbs_common.h"

// exp(x), x <= 0, by Tang's table method: x = (64 m + j) ln2/64 + r, |r| <= ln2/128,
// exp(x) = 2^m 2^(j/64) (1 + expm1(r)), expm1 by its degree-5 Taylor polynomial (truncation
// 3.6e-17), 2^(j/64) from a 64-entry LDS table (correctly rounded), m and j from the low word
// of the round-to-integer sum, 2^m built in the exponent field.  x clamped at -708 as
// gs_exp_neg.  12 f64 instructions + an LDS read instead of gs_exp_neg's 17.
static __constant__ double GS_EXP2_64[64] = {
    0x1.0000000000000p+0, 0x1.02c9a3e778061p+0, 0x1.059b0d3158574p+0, 0x1.0874518759bc8p+0,
    0x1.0b5586cf9890fp+0, 0x1.0e3ec32d3d1a2p+0, 0x1.11301d0125b51p+0, 0x1.1429aaea92de0p+0,
    0x1.172b83c7d517bp+0, 0x1.1a35beb6fcb75p+0, 0x1.1d4873168b9aap+0, 0x1.2063b88628cd6p+0,
    0x1.2387a6e756238p+0, 0x1.26b4565e27cddp+0, 0x1.29e9df51fdee1p+0, 0x1.2d285a6e4030bp+0,
    0x1.306fe0a31b715p+0, 0x1.33c08b26416ffp+0, 0x1.371a7373aa9cbp+0, 0x1.3a7db34e59ff7p+0,
    0x1.3dea64c123422p+0, 0x1.4160a21f72e2ap+0, 0x1.44e086061892dp+0, 0x1.486a2b5c13cd0p+0,
    0x1.4bfdad5362a27p+0, 0x1.4f9b2769d2ca7p+0, 0x1.5342b569d4f82p+0, 0x1.56f4736b527dap+0,
    0x1.5ab07dd485429p+0, 0x1.5e76f15ad2148p+0, 0x1.6247eb03a5585p+0, 0x1.6623882552225p+0,
    0x1.6a09e667f3bcdp+0, 0x1.6dfb23c651a2fp+0, 0x1.71f75e8ec5f74p+0, 0x1.75feb564267c9p+0,
    0x1.7a11473eb0187p+0, 0x1.7e2f336cf4e62p+0, 0x1.82589994cce13p+0, 0x1.868d99b4492edp+0,
    0x1.8ace5422aa0dbp+0, 0x1.8f1ae99157736p+0, 0x1.93737b0cdc5e5p+0, 0x1.97d829fde4e50p+0,
    0x1.9c49182a3f090p+0, 0x1.a0c667b5de565p+0, 0x1.a5503b23e255dp+0, 0x1.a9e6b5579fdbfp+0,
    0x1.ae89f995ad3adp+0, 0x1.b33a2b84f15fbp+0, 0x1.b7f76f2fb5e47p+0, 0x1.bcc1e904bc1d2p+0,
    0x1.c199bdd85529cp+0, 0x1.c67f12e57d14bp+0, 0x1.cb720dcef9069p+0, 0x1.d072d4a07897cp+0,
    0x1.d5818dcfba487p+0, 0x1.da9e603db3285p+0, 0x1.dfc97337b9b5fp+0, 0x1.e502ee78b3ff6p+0,
    0x1.ea4afa2a490dap+0, 0x1.efa1bee615a27p+0, 0x1.f50765b6e4540p+0, 0x1.fa7c1819e90d8p+0};

__device__ __forceinline__ double exp_neg_t64(double x, const double* __restrict__ tb) {
  x = fmax(x, -708.0);
  const double t = fma(x, 0x1.71547652b82fep+6, 0x1.8p52);
  const double n = t - 0x1.8p52;
  double r = fma(n, -0x1.62e42fefa39efp-7, x);
  r = fma(n, -0x1.abc9e3b39803fp-62, r);
  double q = fma(r, 0x1.1111111111111p-7, 0x1.5555555555555p-5);
  q = fma(r, q, 0x1.5555555555555p-3);
  q = fma(r, q, 0.5);
  q = fma(r, q, 1.0);
  const double em1 = r * q;
  const int ni = (int)(unsigned)__double_as_longlong(t);
  const double T = tb[ni & 63];
  return fma(T, em1, T) * __hiloint2double(((ni >> 6) + 1023) << 20, 0);
}

// f64 constant held in an SGPR pair (two s_mov_b32, scalar issue) for a VOP3 operand: gfx950's
// VOP3 f64 ops take no literal, and under VGPR pressure the compiler rematerialises each use as
// two v_mov_b32 (VALU issue)
__device__ __forceinline__ double gs_sconst(double v) {
  asm("" : "+s"(v));
  return v;
}

// exp_neg_t64 with its coefficients in SGPRs (the same arithmetic, bit-identical results)
__device__ __forceinline__ double exp_neg_t64s(double x, const double* __restrict__ tb) {
  x = fmax(x, -708.0);
  const double t = fma(x, gs_sconst(0x1.71547652b82fep+6), gs_sconst(0x1.8p52));
  const double n = t - gs_sconst(0x1.8p52);
  double r = fma(n, gs_sconst(-0x1.62e42fefa39efp-7), x);
  r = fma(n, gs_sconst(-0x1.abc9e3b39803fp-62), r);
  double q = fma(r, gs_sconst(0x1.1111111111111p-7), gs_sconst(0x1.5555555555555p-5));
  q = fma(r, q, gs_sconst(0x1.5555555555555p-3));
  q = fma(r, q, 0.5);
  q = fma(r, q, 1.0);
  const double em1 = r * q;
  const int ni = (int)(unsigned)__double_as_longlong(t);
  const double T = tb[ni & 63];
  return fma(T, em1, T) * __hiloint2double(((ni >> 6) + 1023) << 20, 0);
}

// One lane's G consecutive grid points of one row: h = (tau/2) / (gw + rho_g) with four
// reciprocals from one (R = 1/(a0 a1 a2 a3), 1/(a0 a1) = a2 a3 R, 1/a0 = a1 / (a0 a1), ...: one
// v_rcp_f64 + Newton steps per four points), pdf' = h exp(-h); cum[j] = the lane's running
// sum, returned total.  Products of four (gw + rho_g) stay within 1e-80..1e240.
template <int G>
__device__ __forceinline__ double red_lane_cumsum(double th, double gw, const double* rg, const double* tb,
                                                  double* cum) {
  static_assert(G % 4 == 0, "groups of four points");
  double loc = 0.0;
#pragma unroll
  for (int j = 0; j < G; j += 4) {
    const double a0 = gw + rg[j], a1 = gw + rg[j + 1], a2 = gw + rg[j + 2], a3 = gw + rg[j + 3];
    const double p01 = a0 * a1, p23 = a2 * a3;
    const double R = rcp_nr2(p01 * p23);
    const double r01 = p23 * R, r23 = p01 * R;
    const double h[4] = {th * (a1 * r01), th * (a0 * r01), th * (a3 * r23), th * (a2 * r23)};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      loc = fma(h[q], exp_neg_t64(-h[q], tb), loc);
      cum[j + q] = loc;
    }
  }
  return loc;
}
