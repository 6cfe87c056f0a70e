// rho|b grid conditionals (gfx950, fp64): a4 Gumbel-max, a6 common (CURN)
// product-of-pdfs CDF, a7 per-pulsar red CDF, plus the tau reduction.
//
// All kernels reproduce numpy's operation order exactly — the product over
// pulsars is sequential in pulsar order (np.prod), the CDF is a sequential
// np.cumsum, normalised by its max (the last element) with a true division,
// and the draw is searchsorted(cdf, u, 'left') - 1 with -1 wrapping to the top
// grid point (pta_gibbs.py:205-212) — so grid indices match the reference bit
// for bit on identical inputs.  Mappings: a6 one wavefront per row (45 x 1000
// pdf terms per row); a7/a4 one lane per row (1000 terms per row).
// Rows are laid out [frequency][chain] so lanes of a wave read consecutive
// chains (coalesced).  The grid rho_g = 10**linspace(...), log rho_g and
// 0.5*log10 rho_g are computed on the host with numpy and passed in
// (grid3 = [rho | log rho | 0.5 log10 rho]), bit-identical to the reference's.
#include <cstdlib>

#include "gibbs_common.h"
#include "gibbs_internal.h"
#include "gibbs_gridpt.h"

namespace {

constexpr double LN10 = 2.302585092994045684;  // np.log(10)

// ------------------------------------------------------------ tau
// tau[p][k][c] = (b_sin^2 + b_cos^2) * scale  (scale 1: pta_gibbs.py:194-195; 0.5: pulsar_gibbs.py:209)
__global__ void k_tau(TauArgs A) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int NFR = A.NF / 2;
  const int64_t n = (int64_t)A.n_psr * NFR * A.n_chain;
  if (t >= n) return;
  const int c = (int)(t % A.n_chain);
  const int k = (int)((t / A.n_chain) % NFR);
  const int p = (int)(t / ((int64_t)A.n_chain * NFR));
  const int64_t sys = (int64_t)p * A.n_chain + c;
  const double bs = A.b[sys * A.ldb + A.fidx[p * A.NF + 2 * k]];
  const double bc = A.b[sys * A.ldb + A.fidx[p * A.NF + 2 * k + 1]];
  // b_sin^2 + b_cos^2 rounded as numpy (pta_gibbs.py:194-195): no fma contraction
  const double s2c2 = gs_add_rn(gs_mul_rn(bs, bs), gs_mul_rn(bc, bc));
  A.tau[t] = A.half ? s2c2 / 2 : s2c2;
}

// ------------------------------------------------------------ a6: common CDF
// One WAVEFRONT per row r = k * n_chain + c (GS_CURN_WPB rows per workgroup);
// tau/irn [n_psr][n_f][n_chain]; irn may be NULL (zeros).
//  1. lanes split the grid: pdf[g] = prod_p ratio*exp(-ratio/2)*ln10, the product
//     sequential in pulsar order (np.prod), into LDS;
//  2. lane 0 runs the sequential cumsum in place (np.cumsum, bit-exact order);
//  3. all lanes count cdf[g] / total < u (searchsorted 'left') with a ballot.
#ifndef GS_CURN_WPB
#define GS_CURN_WPB 4
#endif
__global__ __launch_bounds__(64 * GS_CURN_WPB) void k_rho_curn(GridArgs A) {
  extern __shared__ double sh[];
  const int wave = gs_wave_id(), lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * GS_CURN_WPB + wave;
  const int64_t nrow = (int64_t)A.n_f * A.n_chain;
  if (r >= nrow) return;  // whole wavefront exits together (no block barrier below)
  double* pdf = sh + (int64_t)wave * A.ngrid;
  const int c = (int)(r % A.n_chain), k = (int)(r / A.n_chain);
  const int P = A.n_psr;
  const int64_t pstride = nrow;
  for (int g = lane; g < A.ngrid; g += 64) {
    const double rg = A.grid3[g];
    double prod = 1.0;
    for (int p = 0; p < P; ++p) {
      const double tau = A.tau[p * pstride + r];
      const double irn = A.irn ? A.irn[p * pstride + r] : 0.0;
      const double ratio = tau / (irn + rg);
      prod *= ratio * exp(-ratio / 2) * LN10;
    }
    pdf[g] = prod;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (lane == 0) {
    double cum = 0.0;
    int g = 0;
    for (; g + 8 <= A.ngrid; g += 8) {
      double v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = pdf[g + q];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        cum += v[q];
        pdf[g + q] = cum;
      }
    }
    for (; g < A.ngrid; ++g) {
      cum += pdf[g];
      pdf[g] = cum;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  double u;
  if (A.u) {
    u = A.u[(int64_t)c * A.n_f + k];
  } else {
    double u2;
    gs_uniform2(gs_counter(k, gs_sweep(A.sweep, A.sweep_dev), A.chain_base + c, 0, GS_EV_CURN), A.key, u, u2);
  }
  const double total = pdf[A.ngrid - 1];
  int cnt = 0;
  for (int g0 = 0; g0 < A.ngrid; g0 += 64) {
    const int g = g0 + lane;
    const bool lt = g < A.ngrid && (pdf[g] / total < u);
    cnt += __popcll(__ballot(lt));
  }
  if (lane == 0) {
    int idx = cnt - 1;
    if (idx < 0) idx += A.ngrid;
    if (A.idx_out) A.idx_out[r] = idx;
    A.x[(int64_t)c * A.ldx + A.xcol[k]] = A.grid3[2 * A.ngrid + idx];
  }
}

// ------------------------------------------------------------ a6': CURN from tau sums
// Without per-pulsar red noise the common pdf depends on tau only through
// S_k = sum_p tau_p,k: prod_p (tau_p/rho) e^(-tau_p/(2 rho)) ln10 = const * rho^-P
// e^(-S/(2 rho)), and the constant cancels in cdf / max.  So a pulsar-sharded run
// exchanges S (one all-reduce of n_f x n_chain doubles) instead of every tau, and the
// draw is O(1) per grid point: log pdf = -P log rho_g - S / (2 rho_g), evaluated
// against its maximum (no underflow for any P).  Same draw as k_rho_curn up to
// rounding of the pdf (1e-15 relative: an index can only differ when u falls within
// that of a cdf value).  One wavefront per row; lane l owns the contiguous grid
// points [l G, (l+1) G), G = ceil(ngrid / 64); wave scan of the lane sums.
__global__ __launch_bounds__(256) void k_tau_sum(int n_psr, int64_t nrow, const double* tau, double* S) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrow) return;
  double s = 0.0;
  for (int p = 0; p < n_psr; ++p) s += tau[p * nrow + r];  // sequential in pulsar order
  S[r] = s;
}

// ---- the CURN tau sums in exact fixed point (pulsar-sharded runs: order-free exchange)
// S_k = sum_p tau_p,k with every tau truncated to the grid 2^e0 and summed as integers in three
// 48-bit digits held in int64 (exact for < 2^15 pulsars): integer addition is associative, so
// the per-rank partial digits all-reduce (RCCL int64 sum, any ring / tree order) to the same
// integers on every rank and for every number of shards, and gs_fx_to_double rounds them to the
// same S.  e0 = floor(log2 rhomin) - 64 puts the truncation ~2^-64 below the smallest grid rho,
// where S / (2 rho_g) cannot see it; 144 bits reach rhomin * 2^80.
constexpr int FX_BITS = 48;
constexpr unsigned long long FX_MASK = (1ull << FX_BITS) - 1;

__global__ __launch_bounds__(256) void k_tau_sum_fx(int n_psr, int64_t nrow, const double* tau, int e0,
                                                    long long* acc, int* ovf) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrow) return;
  long long d0 = 0, d1 = 0, d2 = 0;
  bool bad = false;
  for (int p = 0; p < n_psr; ++p) {
    const double v = tau[p * nrow + r];
    if (v == 0.0) continue;
    if (!(v > 0.0) || v == __builtin_inf()) {
      bad = true;
      continue;
    }
    int E;
    const double fr = frexp(v, &E);                           // v = fr 2^E, fr in [0.5, 1)
    const unsigned long long M = (unsigned long long)ldexp(fr, 53);  // exact 53-bit integer
    const int sh = E - 53 - e0;                                // v = M 2^sh 2^e0
    if (sh + 53 > 3 * FX_BITS) bad = true;                     // beyond the top digit
    unsigned long long dg[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int t = sh - FX_BITS * i;                          // digit i = floor(M 2^t) mod 2^48
      const unsigned long long u = t >= 0 ? (t < 64 ? M << t : 0ull) : (-t < 64 ? M >> (-t) : 0ull);
      dg[i] = u & FX_MASK;
    }
    d0 += (long long)dg[0];
    d1 += (long long)dg[1];
    d2 += (long long)dg[2];
  }
  acc[r] = d0;
  acc[nrow + r] = d1;
  acc[2 * nrow + r] = d2;
  if (bad && ovf) *ovf = 1;
}

// k_tau and k_tau_sum_fx fused (CURN from the tau sums, no per-pulsar red noise): thread (k, c)
// forms tau_p,k = b_sin^2 + b_cos^2 of every pulsar from b and adds its digits; tau never goes to
// HBM.  Same digits as the two kernels (integer sums: any order).
__device__ __forceinline__ bool fx_add(double v, int e0, long long& d0, long long& d1, long long& d2) {
  if (v == 0.0) return true;
  if (!(v > 0.0) || v == __builtin_inf()) return false;
  int E;
  const double fr = frexp(v, &E);
  const unsigned long long M = (unsigned long long)ldexp(fr, 53);
  const int sh = E - 53 - e0;
  unsigned long long dg[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int t = sh - FX_BITS * i;
    const unsigned long long u = t >= 0 ? (t < 64 ? M << t : 0ull) : (-t < 64 ? M >> (-t) : 0ull);
    dg[i] = u & FX_MASK;
  }
  d0 += (long long)dg[0];
  d1 += (long long)dg[1];
  d2 += (long long)dg[2];
  return sh + 53 <= 3 * FX_BITS;
}

// One workgroup per chain, its 4 waves taking every 4th pulsar: lane j < NF reads b column
// fidx[p][j] of system (p, c) (a b row's free-spectrum columns: one coalesced read per wave and
// pulsar), the even lane 2k forms tau_k = b_sin^2 + b_cos^2 with its neighbour's value and adds its
// digits; the four waves' digits are summed in LDS.  (Round 3 ran one thread per (k, c) row over
// all pulsars: 960 waves of 600-byte-strided gathers, 0.038 ms per configs[3] sweep.)
__global__ __launch_bounds__(256) void k_tau_sum_fx_b(TauArgs A, int e0, long long* acc, int* ovf) {
  __shared__ long long dsum[3][4][64];
  const int wave = gs_wave_id(), lane = threadIdx.x & 63;
  const int c = blockIdx.x;
  const int NFR = A.NF / 2;
  const int64_t nrow = (int64_t)NFR * A.n_chain;
  const bool act = lane < A.NF;
  long long d0 = 0, d1 = 0, d2 = 0;
  bool ok = true;
#pragma unroll 4
  for (int p = wave; p < A.n_psr; p += 4) {
    const int64_t sys = (int64_t)p * A.n_chain + c;
    const double bv = act ? A.b[sys * A.ldb + A.fidx[p * A.NF + lane]] : 0.0;
    const double bc = __shfl_xor(bv, 1);
    if (act && !(lane & 1)) ok &= fx_add(gs_add_rn(gs_mul_rn(bv, bv), gs_mul_rn(bc, bc)), e0, d0, d1, d2);  // numpy's tau rounding
  }
  dsum[0][wave][lane] = d0;
  dsum[1][wave][lane] = d1;
  dsum[2][wave][lane] = d2;
  if (!ok && ovf) *ovf = 1;
  __syncthreads();
  if (wave == 0 && act && !(lane & 1)) {
    const int64_t t = (int64_t)(lane >> 1) * A.n_chain + c;
#pragma unroll
    for (int i = 0; i < 3; ++i) acc[i * nrow + t] = dsum[i][0][lane] + dsum[i][1][lane] + dsum[i][2][lane] + dsum[i][3][lane];
  }
}

__global__ __launch_bounds__(256) void k_fx_to_double(int64_t nrow, int e0, const long long* acc, double* S) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrow) return;
  long long d0 = acc[r], d1 = acc[nrow + r], d2 = acc[2 * nrow + r];
  d1 += d0 >> FX_BITS;  // carries (digits are sums of nonnegative 48-bit values)
  d0 &= (long long)FX_MASK;
  d2 += d1 >> FX_BITS;
  d1 &= (long long)FX_MASK;
  // four exact, non-overlapping terms, summed high to low with two-sums: the same bits on
  // every rank (deterministic, ~correctly rounded)
  const double t3 = ldexp((double)(d2 >> 24), 3 * FX_BITS - 24 + e0);
  const double t2 = ldexp((double)(d2 & 0xffffff), 2 * FX_BITS + e0);
  const double t1 = ldexp((double)d1, FX_BITS + e0);
  const double t0 = ldexp((double)d0, e0);
  double hi = t3, lo = 0.0;
  const double terms[3] = {t2, t1, t0};
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const double sm = hi + terms[i];
    const double bb = sm - hi;
    lo += (hi - (sm - bb)) + (terms[i] - bb);
    hi = sm;
  }
  S[r] = hi + lo;
}

constexpr int CS_MAXG = 32;  // grid points per lane (ngrid <= 2048)

__global__ __launch_bounds__(256) void k_rho_curn_sum(GridArgs A) {
  const int wave = gs_wave_id(), lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + wave;
  const int64_t nrow = (int64_t)A.n_f * A.n_chain;
  if (r >= nrow) return;
  const int c = (int)(r % A.n_chain), k = (int)(r / A.n_chain);
  const double S = A.tau[r];
  const double P = (double)A.n_psr;
  const int G = (A.ngrid + 63) / 64;
  const int g0 = lane * G;
  double lp[CS_MAXG];
  double mx = -__builtin_inf();
#pragma unroll
  for (int j = 0; j < CS_MAXG; ++j) {
    const int g = g0 + j;
    lp[j] = -__builtin_inf();
    if (j < G && g < A.ngrid) {
      lp[j] = -P * A.grid3[A.ngrid + g] - S / (2.0 * A.grid3[g]);
      mx = fmax(mx, lp[j]);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
  double loc = 0.0;  // this lane's cumulative sums, kept in lp[]
#pragma unroll
  for (int j = 0; j < CS_MAXG; ++j) {
    if (j < G) {
      loc += gs_exp_neg(lp[j] - mx);  // -inf past the grid -> 0
      lp[j] = loc;
    }
  }
  // inclusive wave scan of the lane totals
  double incl = loc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double v = __shfl_up(incl, o);
    if (lane >= o) incl += v;
  }
  const double off = incl - loc;
  const double total = __shfl(incl, 63);
  double u;
  if (A.u) {
    u = A.u[(int64_t)c * A.n_f + k];
  } else {
    double u2;
    gs_uniform2(gs_counter(k, gs_sweep(A.sweep, A.sweep_dev), A.chain_base + c, 0, GS_EV_CURN), A.key, u, u2);
  }
  int cnt = 0;  // searchsorted(cdf / total, u, 'left'): points with cdf / total < u
#pragma unroll
  for (int j = 0; j < CS_MAXG; ++j)
    if (j < G && g0 + j < A.ngrid) cnt += ((off + lp[j]) / total < u) ? 1 : 0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  if (lane == 0) {
    int idx = cnt - 1;
    if (idx < 0) idx += A.ngrid;
    if (A.idx_out) A.idx_out[r] = idx;
    A.x[(int64_t)c * A.ldx + A.xcol[k]] = A.grid3[2 * A.ngrid + idx];
  }
}

// k_rho_curn_sum over 64 rows per wave (ngrid <= 1024): the lane-per-row loads and Philox
// uniform as k_rho_red_wave, each lane's 16 grid points prepared once per wave as
// c_g = -P log rho_g and w_g = 1 / (2 rho_g), so a row costs one FMA (log pdf = c_g - S w_g),
// the wave maximum, the LDS-table exp and the scan / count per point.
// RPW rows per wave: 64 at the round-2 default; the CURN line's 30 x 2048 rows are then only 960
// waves (under one per SIMD), so fewer rows per wave buy occupancy for the per-wave grid setup.
constexpr int CSW_G = 16;
#ifndef GS_CSW_RPW
#define GS_CSW_RPW 16
#endif

// One row of k_rho_curn_sum_wave, wave-wide: lane l holds points [16 l, 16 l + 16) as cg, wg
// (valid: the 16 ballot masks of the on-grid points); returns searchsorted(cdf / total, u) - 1 (-1
// before wrapping).  Shared with k_rho_curn_sum_cert16's f64 redo of unproven rows.
__device__ __forceinline__ int curn_sum_row_f64(double nS, double ui, const double* cg, const double* wg,
                                                const unsigned long long* valid, const double* tb, int lane) {
  double lp[CSW_G];
  double mx = -__builtin_inf();
#pragma unroll
  for (int j = 0; j < CSW_G; ++j) {
    lp[j] = fma(nS, wg[j], cg[j]);
    mx = fmax(mx, lp[j]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
  double loc = 0.0;
#pragma unroll
  for (int j = 0; j < CSW_G; ++j) {
    loc += exp_neg_t64(lp[j] - mx, tb);
    lp[j] = loc;
  }
  double incl = loc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double v = __shfl_up(incl, o);
    if (lane >= o) incl += v;
  }
  const double total = rdlane(incl, 63);
  const double thr = ui * total - (incl - loc);
  int cnt = 0;
#pragma unroll
  for (int j = 0; j < CSW_G; ++j) cnt += __popcll(__ballot(lp[j] < thr) & valid[j]);
  return cnt - 1;
}

template <int RPW>
__global__ __launch_bounds__(256) void k_rho_curn_sum_wave(GridArgs A) {
  __shared__ double tb[64];
  const int wave = gs_wave_id(), lane = threadIdx.x & 63;
  if (threadIdx.x < 64) tb[threadIdx.x] = GS_EXP2_64[threadIdx.x];
  __syncthreads();
  const int64_t nrow = (int64_t)A.n_f * A.n_chain;
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + wave) * RPW;
  if (r0 >= nrow) return;
  const int64_t r = r0 + lane;
  const bool rok = lane < RPW && r < nrow;
  const int64_t rr = rok ? r : r0;
  const int c = (int)(rr % A.n_chain), k = (int)(rr / A.n_chain);
  double u = 0.0;
  if (A.u) {
    u = A.u[(int64_t)c * A.n_f + k];
  } else if (lane < RPW) {
    double u2;
    gs_uniform2(gs_counter(k, gs_sweep(A.sweep, A.sweep_dev), A.chain_base + c, 0, GS_EV_CURN), A.key, u, u2);
  }
  const double S = A.tau[rr];
  const double P = (double)A.n_psr;
  double cg[CSW_G], wg[CSW_G];
#pragma unroll
  for (int j = 0; j < CSW_G; ++j) {
    const int g = CSW_G * lane + j;
    const bool ok = g < A.ngrid;
    cg[j] = ok ? -P * A.grid3[A.ngrid + g] : -1e300;  // past the grid: exp -> ~0, never counted
    wg[j] = ok ? 0.5 / A.grid3[g] : 0.0;
  }
  unsigned long long valid[CSW_G];
#pragma unroll
  for (int j = 0; j < CSW_G; ++j) valid[j] = __ballot(CSW_G * lane + j < A.ngrid);
  const int nr = (int)min((int64_t)RPW, nrow - r0);
  int myidx = 0;
  for (int i = 0; i < nr; ++i) {
    int idx = curn_sum_row_f64(-rdlane(S, i), rdlane(u, i), cg, wg, valid, tb, lane);
    if (idx < 0) idx += A.ngrid;
    myidx = (lane == i) ? idx : myidx;
  }
  if (rok) {
    if (A.idx_out) A.idx_out[r] = myidx;
    A.x[(int64_t)c * A.ldx + A.xcol[k]] = A.grid3[2 * A.ngrid + myidx];
  }
}

// ------------------------------------------------------------ a6 fast: CURN product in log space
// The same draw as k_rho_curn without numpy's operation order (GS_OPT_GRID_EXACT = 0,
// the default): log pdf_g = -sum_p log(irn_p + rho_g) - 1/2 sum_p tau_p / (irn_p + rho_g)
// + const (sum_p log tau_p and P log ln10 cancel in cdf / max).  The ratio sum is kept as one
// fraction N / D over the product D of (irn + rho), taken CF_K pulsars at a time: for a group,
// D_grp(rho) = prod_i (rho + irn_i) and N_grp(rho) = sum_i tau_i prod_{j != i} (rho + irn_j) are
// polynomials in rho whose coefficients (all positive: no cancellation) depend on the row only,
// so lane q computes group q's once per row and every grid point evaluates them by Horner
// (CF_K + CF_K - 1 FMAs), then N <- N D_grp + D N_grp, D <- D D_grp: 2 CF_K + 2 f64 ops per
// (point, group), 2.5 per (point, pulsar) at CF_K = 4 instead of 4 (add, two multiplies and an
// FMA per pulsar).  D and N are rescaled together every RN groups by one power of two per
// lane (the lane's 16 neighbouring grid points keep D within a few decades of each other).  One
// log, one division and one exp per grid point at the end.  pdf rounding differs from numpy's
// by ~1e-15 relative, so the index can only differ when u falls that close to a cdf value
// (tested equal to the reference on every fixture sweep and to the numpy-order kernel on random
// rows).  One wavefront per row, lane l owns grid points [l G, (l+1) G), wave scan of the lane
// sums.
constexpr int CF_MAXG = 16;  // grid points per lane (ngrid <= 1024)

#ifndef GS_CF_MINW
#define GS_CF_MINW 3
#endif
// Group coefficients handed from lane q to the whole wave through the wave's LDS slot (one
// broadcast ds_read per coefficient pair, LDS pipe) instead of two v_readlane_b32 per coefficient
// (VALU: ~9 issue cycles each on MI355X, tools/probe/mfma_probe.hip -- 18 per group, a fifth of
// the group's VALU time at CF_K = 4).
#ifndef GS_CF_LDS
#define GS_CF_LDS 1
#endif
// CF_K = 5 for pulsar counts where it needs fewer groups x ops (45 = 9 x 5: 108 f64 ops per grid
// point instead of 12 groups x 10 = 120), else 4; GS_CF_AUTOK=0 keeps 4.
#ifndef GS_CF_AUTOK
#define GS_CF_AUTOK 1
#endif
// The tail's exp by Tang's 64-entry table (exp_neg_t64, 12 f64 instructions + one LDS read) instead
// of gs_exp_neg's degree-11 polynomial (17, and 2 v_mov_b32 per f64 coefficient at this pressure)
#ifndef GS_CF_TEXP
#define GS_CF_TEXP 1
#endif
template <int CF_K>
__global__ __launch_bounds__(256, GS_CF_MINW) void k_rho_curn_fast(GridArgs A) {
  constexpr int CS = 2 * CF_K + 2;  // LDS doubles per group (even: pairs stay 16-byte aligned)
#if GS_CF_LDS
  __shared__ __attribute__((aligned(16))) double cfl[4][64 * CS];
#endif
#if GS_CF_TEXP
  __shared__ double etb[64];
  if (threadIdx.x < 64) etb[threadIdx.x] = GS_EXP2_64[threadIdx.x];
  __syncthreads();
#endif
  const int wave = gs_wave_id(), lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + wave;
  const int64_t nrow = (int64_t)A.n_f * A.n_chain;
  if (r >= nrow) return;
  const int c = (int)(r % A.n_chain), k = (int)(r / A.n_chain);
  const int G = (A.ngrid + 63) / 64;
  const int g0 = lane * G;
  double rg[CF_MAXG], dd[CF_MAXG], nn[CF_MAXG];
  double rmin = 1e300;
#pragma unroll
  for (int j = 0; j < CF_MAXG; ++j) {
    const int g = min(g0 + j, A.ngrid - 1);
    rg[j] = A.grid3[g];
    rmin = fmin(rmin, rg[j]);
    dd[j] = 1.0;
    nn[j] = 0.0;
  }
  // D and N are rescaled every RN groups: (2 rho_min)^(CF_K RN) must stay normal.  RN = 2 (one
  // rescale per 2 CF_K pulsars) for rho_min >= 1e-30 (CF_K = 5; 1e-38 at CF_K = 4: every prior
  // box of the reference's examples), else every group (rho_min down to ~1e-61).
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) rmin = fmin(rmin, __shfl_xor(rmin, o));
  const int RN = __builtin_amdgcn_readfirstlane((int)(rmin >= (CF_K == 4 ? 1e-38 : 1e-30)) + 1);
  int ex = 0;  // the lane's common binary exponent of dd (and nn)
  const int P = A.n_psr;
  // 64 groups (64 CF_K pulsars) at a time: lane q builds group q's coefficients from its
  // pulsars' (tau, irn), ascending powers: D_grp = sum_e pc[e] rho^e, N_grp = sum_e qc[e] rho^e
  for (int p0 = 0; p0 < P; p0 += 64 * CF_K) {
    const int ng = min(64, (P - p0 + CF_K - 1) / CF_K);
    double pc[CF_K + 1], qc[CF_K];
#pragma unroll
    for (int e = 0; e <= CF_K; ++e) pc[e] = e == 0 ? 1.0 : 0.0;
#pragma unroll
    for (int e = 0; e < CF_K; ++e) qc[e] = 0.0;
    if (lane < ng) {
#pragma unroll
      for (int i = 0; i < CF_K; ++i) {
        const int p = p0 + CF_K * lane + i;
        if (p < P) {
          const double tau = A.tau[(int64_t)p * nrow + r];
          const double irn = A.irn ? A.irn[(int64_t)p * nrow + r] : 0.0;
          // N <- N (rho + irn) + tau D, D <- D (rho + irn), on the coefficients
#pragma unroll
          for (int e = CF_K - 1; e >= 0; --e) qc[e] = fma(irn, qc[e], (e > 0 ? qc[e - 1] : 0.0) + tau * pc[e]);
#pragma unroll
          for (int e = CF_K; e >= 0; --e) pc[e] = fma(irn, pc[e], e > 0 ? pc[e - 1] : 0.0);
        }
      }
    }
#if GS_CF_LDS
    double* cw = cfl[wave];
    if (lane < ng) {
#pragma unroll
      for (int e = 0; e <= CF_K; ++e) cw[lane * CS + e] = pc[e];
#pragma unroll
      for (int e = 0; e < CF_K; ++e) cw[lane * CS + CF_K + 1 + e] = qc[e];
    }
    wave_lds_sync();
#endif
    for (int q = 0; q < ng; ++q) {
      double a[CF_K + 1], b[CF_K];
#if GS_CF_LDS
      const double2* cq = reinterpret_cast<const double2*>(cw + q * CS);
      double co[CS];
#pragma unroll
      for (int e = 0; e < CS / 2; ++e) {
        const double2 v = cq[e];
        co[2 * e] = v.x;
        co[2 * e + 1] = v.y;
      }
#pragma unroll
      for (int e = 0; e <= CF_K; ++e) a[e] = co[e];
#pragma unroll
      for (int e = 0; e < CF_K; ++e) b[e] = co[CF_K + 1 + e];
#else
#pragma unroll
      for (int e = 0; e <= CF_K; ++e) a[e] = rdlane(pc[e], q);
#pragma unroll
      for (int e = 0; e < CF_K; ++e) b[e] = rdlane(qc[e], q);
#endif
#pragma unroll
      for (int j = 0; j < CF_MAXG; ++j) {
        const double x = rg[j];
        double pd = fma(a[CF_K], x, a[CF_K - 1]);
#pragma unroll
        for (int e = CF_K - 2; e >= 0; --e) pd = fma(pd, x, a[e]);
        double qn = fma(b[CF_K - 1], x, b[CF_K - 2]);
#pragma unroll
        for (int e = CF_K - 3; e >= 0; --e) qn = fma(qn, x, b[e]);
        // N pd (a multiply into N's own register) + D qn (v_fmac onto it): no register copy
        // per point (fma(N, pd, D qn) tied the v_fmac to the D qn temporary: one v_mov_b64 more)
        nn[j] = fma(dd[j], qn, nn[j] * pd);
        dd[j] *= pd;
      }
      if ((q % RN) == RN - 1 || q == ng - 1) {
        const int e = __builtin_amdgcn_frexp_exp(dd[0]);
        ex += e;
#pragma unroll
        for (int j = 0; j < CF_MAXG; ++j) {
          dd[j] = ldexp(dd[j], -e);
          nn[j] = ldexp(nn[j], -e);
        }
      }
    }
#if GS_CF_LDS
    wave_lds_sync();  // the next 64-group block rewrites the slot
#endif
  }
  constexpr double LN2 = 0.693147180559945309417232121458176568;
  // pdf_g = 2^-ex / dd e^(-N / 2D): with y = 1 / dd = fr 2^e (frexp, exact), pdf_g = fr e^(lp_g) and
  // lp_g = (e - ex) ln2 - nn y / 2 -- no log per point (round 3 took -log dd: ~25 more f64 ops)
  double lp[CF_MAXG], fr[CF_MAXG];
  double mx = -__builtin_inf();
#pragma unroll
  for (int j = 0; j < CF_MAXG; ++j) {
    lp[j] = -__builtin_inf();
    fr[j] = 0.0;
    if (j < G && g0 + j < A.ngrid) {
      const double y = rcp_nr2(dd[j]);
      int e;
      fr[j] = frexp(y, &e);
      lp[j] = fma((double)(e - ex), LN2, -0.5 * (nn[j] * y));
      mx = fmax(mx, lp[j]);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
  double loc = 0.0;
#pragma unroll
  for (int j = 0; j < CF_MAXG; ++j) {
    if (j < G) {
#if GS_CF_TEXP
      loc += fr[j] * exp_neg_t64s(lp[j] - mx, etb);
#else
      loc += fr[j] * gs_exp_neg(lp[j] - mx);
#endif
      lp[j] = loc;
    }
  }
  double incl = loc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double v = __shfl_up(incl, o);
    if (lane >= o) incl += v;
  }
  const double off = incl - loc;
  const double total = __shfl(incl, 63);
  double u;
  if (A.u) {
    u = A.u[(int64_t)c * A.n_f + k];
  } else {
    double u2;
    gs_uniform2(gs_counter(k, gs_sweep(A.sweep, A.sweep_dev), A.chain_base + c, 0, GS_EV_CURN), A.key, u, u2);
  }
  // searchsorted(cdf / total, u): cdf < u total - (the lane offset), no division per point
  const double thr = u * total - off;
  int cnt = 0;
#pragma unroll
  for (int j = 0; j < CF_MAXG; ++j)
    if (j < G && g0 + j < A.ngrid) cnt += (lp[j] < thr) ? 1 : 0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  if (lane == 0) {
    int idx = cnt - 1;
    if (idx < 0) idx += A.ngrid;
    if (A.idx_out) A.idx_out[r] = idx;
    A.x[(int64_t)c * A.ldx + A.xcol[k]] = A.grid3[2 * A.ngrid + idx];
  }
}

// ------------------------------------------------------------ a7: red CDF
// rows r = (p * n_f + k) * n_chain + c, one LANE per row; gw [n_f][n_chain] = phi_gw.
// One pass over the grid keeps the (sequential, exact) running sum at 16 chunk
// ends; the crossing chunk is then recomputed from its exact entry value, so the
// cumsum seen at every compared position is bit-identical to np.cumsum.
#define GS_RED_NCH 16
// EXACT = false (GS_OPT_GRID_EXACT = 0, the default): ratio = tau * rcp(a) refined by two
// Newton steps instead of the IEEE division (within an ulp of it; same index unless u falls
// within ~1e-16 of a cdf value).
template <bool EXACT>
__device__ __forceinline__ double red_ratio(double tau, double a) {
  if (EXACT) return tau / a;
  double ra = __builtin_amdgcn_rcp(a);
  ra = fma(ra, fma(-a, ra, 1.0), ra);
  ra = fma(ra, fma(-a, ra, 1.0), ra);
  return tau * ra;
}

// one grid point's pdf: ratio * exp(-ratio/2) * ln10 (pta_gibbs.py:265-266); the default
// mode uses the short exp (gibbs_common.h, <= 2 ulp), EXACT the device library's
template <bool EXACT>
__device__ __forceinline__ double red_pdf(double tau, double a) {
  // numpy's rounding: no fma contraction (-ffp-contract=fast would fuse the product into the
  // caller's running sum, which numpy does not)
#pragma clang fp contract(off)
  const double ratio = red_ratio<EXACT>(tau, a);
  return ratio * (EXACT ? exp(-ratio / 2) : gs_exp_neg(-0.5 * ratio)) * LN10;
}

template <bool EXACT>
__global__ void k_rho_red(GridArgs A) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nrow = (int64_t)A.n_psr * A.n_f * A.n_chain;
  if (r >= nrow) return;
  const int c = (int)(r % A.n_chain);
  const int k = (int)((r / A.n_chain) % A.n_f);
  const int p = (int)(r / ((int64_t)A.n_chain * A.n_f));
  double u;
  if (A.u) {
    u = A.u[((int64_t)c * A.n_psr + p) * A.n_f + k];
  } else {
    double u2;
    gs_uniform2(gs_counter(k, gs_sweep(A.sweep, A.sweep_dev), A.chain_base + c, p + A.psr_base, GS_EV_RED), A.key, u, u2);
  }
  const double tau = A.tau[r];
  const double gw = A.irn[(int64_t)k * A.n_chain + c];
  const int ch = (A.ngrid + GS_RED_NCH - 1) / GS_RED_NCH;
  double ck[GS_RED_NCH];
  double cum = 0.0;
  // The grid is wave-uniform (scalar loads): unrolled by 8 so a group's loads are issued
  // together instead of one load + wait per point; the running sum stays sequential.
#pragma unroll
  for (int j = 0; j < GS_RED_NCH; ++j) {
    const int g1 = min(A.ngrid, (j + 1) * ch);
#pragma unroll 8
    for (int g = j * ch; g < g1; ++g) {
#pragma clang fp contract(off)
      cum += red_pdf<EXACT>(tau, gw + A.grid3[g]);
    }
    ck[j] = cum;
  }
  const double total = cum;
  // cdf < u as numpy computes it, cumsum / max < u (EXACT); otherwise cumsum < u * max,
  // which differs only when u falls within an ulp of a cdf value (no divisions)
  const double ut = u * total;
  auto below = [&](double cs) { return EXACT ? (cs / total < u) : (cs < ut); };
  // first chunk whose end crosses u; everything before it counts
  int jx = GS_RED_NCH;
  double entry = 0.0;
#pragma unroll
  for (int j = GS_RED_NCH - 1; j >= 0; --j) {
    if (!below(ck[j])) {
      jx = j;
      entry = j > 0 ? ck[j - 1] : 0.0;
    }
  }
  int cnt;
  if (jx == GS_RED_NCH) {
    cnt = A.ngrid;  // u above every cdf value
  } else {
    cnt = jx * ch;
    double cc = entry;
    const int g1 = min(A.ngrid, (jx + 1) * ch);
#pragma unroll 4
    for (int g = jx * ch; g < g1; ++g) {
#pragma clang fp contract(off)
      cc += red_pdf<EXACT>(tau, gw + A.grid3[g]);
      cnt += below(cc) ? 1 : 0;
    }
  }
  int idx = cnt - 1;
  if (idx < 0) idx += A.ngrid;
  if (A.idx_out) A.idx_out[r] = idx;
  A.x[(int64_t)c * A.ldx + A.xcol[p * A.n_f + k]] = A.grid3[2 * A.ngrid + idx];
}

// ------------------------------------------------------------ a7 fast: red CDF, wave per row
// The default (non-exact) mode.  A wave takes 64 consecutive rows (one per lane for the loads
// and the Philox uniform) and then walks them one at a time with all 64 lanes on the grid:
// lane l owns grid points [16 l, 16 l + 16) (held in registers for the whole wave), sums
// its pdf values sequentially, and a wave scan of the lane sums gives every point's cdf.
// Against the lane-per-row kernel: no second pass over the crossing chunk, no wave-count
// tail (43k one-row-per-lane waves at configs[3] sizes are 5.3 rounds of the chip), and
// every grid point is evaluated once.  Per point: h = (tau/2) / (gw + rho_g) (rcp + two
// Newton steps), pdf' = h exp(-h) with the short exp -- the reference's
// ratio exp(-ratio/2) ln10 (pta_gibbs.py:265-266) up to the constant 2 ln10, which cancels
// in cdf / max.  Sums differ from np.cumsum's sequential order by rounding (~1e-16 relative),
// so an index can only differ when u falls that close to a cdf value.
constexpr int RW_G = 16;  // grid points per lane (ngrid <= 1024)
typedef float gs_f2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_rho_red_wave(GridArgs A) {
  __shared__ double tb[64];
  const int wave = gs_wave_id(), lane = threadIdx.x & 63;
  if (threadIdx.x < 64) tb[threadIdx.x] = GS_EXP2_64[threadIdx.x];
  __syncthreads();
  const int64_t nrow = (int64_t)A.n_psr * A.n_f * A.n_chain;
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + wave) * 64;
  if (r0 >= nrow) return;
  const int64_t r = r0 + lane;
  const bool rok = r < nrow;
  const int64_t rr = rok ? r : r0;
  const int c = (int)(rr % A.n_chain);
  const int k = (int)((rr / A.n_chain) % A.n_f);
  const int p = (int)(rr / ((int64_t)A.n_chain * A.n_f));
  double u;
  if (A.u) {
    u = A.u[((int64_t)c * A.n_psr + p) * A.n_f + k];
  } else {
    double u2;
    gs_uniform2(gs_counter(k, gs_sweep(A.sweep, A.sweep_dev), A.chain_base + c, p + A.psr_base, GS_EV_RED), A.key, u, u2);
  }
  const double th = 0.5 * A.tau[rr];
  const double gw = A.irn[(int64_t)k * A.n_chain + c];
  // this lane's grid points; past the grid a huge rho_g makes the pdf ~tau 1e-60 (and those
  // points are never counted)
  double rg[RW_G];
#pragma unroll
  for (int j = 0; j < RW_G; ++j) {
    const int g = RW_G * lane + j;
    rg[j] = g < A.ngrid ? A.grid3[g] : 1e60;  // a^4 stays finite
  }
  unsigned long long valid[RW_G];  // lanes whose point j is on the grid (wave-uniform)
#pragma unroll
  for (int j = 0; j < RW_G; ++j) valid[j] = __ballot(RW_G * lane + j < A.ngrid);
  const int nr = (int)min((int64_t)64, nrow - r0);
  int myidx = 0;
  for (int i = 0; i < nr; ++i) {
    const double thi = rdlane(th, i), gwi = rdlane(gw, i), ui = rdlane(u, i);
    double cum[RW_G];
    const double loc = red_lane_cumsum<RW_G>(thi, gwi, rg, tb, cum);
    double incl = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const double v = __shfl_up(incl, o);
      if (lane >= o) incl += v;
    }
    const double total = rdlane(incl, 63);
    const double thr = ui * total - (incl - loc);  // cum_j + (exclusive lane prefix) < u * total
    int cnt = 0;
#pragma unroll
    for (int j = 0; j < RW_G; ++j) cnt += __popcll(__ballot(cum[j] < thr) & valid[j]);
    int idx = cnt - 1;
    if (idx < 0) idx += A.ngrid;
    myidx = (lane == i) ? idx : myidx;
  }
  if (rok) {
    if (A.idx_out) A.idx_out[r] = myidx;
    A.x[(int64_t)c * A.ldx + A.xcol[p * A.n_f + k]] = A.grid3[2 * A.ngrid + myidx];
  }
}

// ------------------------------------------------------------ a7 default: certified two-level draw
// k_rho_red_wave's row walk with every grid point evaluated in FP32, and the index accepted only
// when it is provably the exact-arithmetic one; otherwise the row is redone in FP64 (the
// k_rho_red_wave arithmetic).  Per point (all f32, two points per packed v_pk_* op): a = gw' +
// rho'_g, y = 1/a (v_rcp_f32), t = tl y, x = tl2 y, E = 2^-x (v_exp_f32), pdf' = t E, with the
// row's scales
// th = (tau/2) = thm 2^e, tl = thm log2e, tl2 = th log2e 2^S, gw' = gw 2^S, rho'_g = rho_g 2^S
// (S = -ilogb(rho_min): every a in [1, 2^120)), so pdf' = h e^-h up to a row constant
// (h = th / (gw + rho_g) = x ln2): no f32 underflow in the ratios, only in e^-h itself.
//
// E = 2^(xm - x) with xm = the row's smallest x (at rho_max): the row constant 2^xm cancels in
// cdf / max, and the largest E is ~1, so the row never underflows as a whole.  The exponent
// xm - x is one FMA, fma(-tl2, y, xm): 7 x + 6 xm eps of absolute error, within the 8 x + 7 xm of
// the separately rounded x and difference that the bound below is written for.
//
// Certificate.  Relative error of each pdf' (first order, eps = 2^-24): the inputs' f32
// roundings and the add (3 eps), v_rcp_f32 (2 eps), tl (3 eps), the products (2 eps), v_exp_f32
// (2 eps) and the exponents' own errors carried through 2^(xm - x) (ln2 (8 eps x + 7 eps xm)):
// below (12 + 5.6 x + 4.9 xm) eps.  Sums of positives: 21 additions per prefix (16 in the lane,
// 6 in the scan) and 3 roundings in the thresholds.  So every computed cum_j and the total are
// within D = eps (80 T + 18 w + 12 xm T) + 2e-35 of the exact ones, T = total, w = sum pdf' x,
// the last term for points whose E is subnormal or flushed (t <= 1.45, <= 1024 points), with a
// margin of ~2 on every term.  The exact index is #{j : cum*_j < u T*} - 1; if no computed cum_j
// lies in [u T - 2D, u T + 2D) that count equals the computed one, and the f64 cdfs (within
// ~1e-15 of exact) give the same index too.  Otherwise (probability
// below), or if the f32 row degenerates (T not a normal float), the wave redoes the row in f64.  Indices are therefore those of exact
// arithmetic wherever the f32 path answers, the same contract as the f64 wave kernel's (which
// differs from numpy's order only within ~1e-16 of a cdf value); an unproven row is redone with
// that kernel's f64 arithmetic, so the default mode returns GS_OPT_GRID_EXACT = 2's index on every
// row.  Fallback rate: u lands within 2D of one of the ~1000 cdf values with probability
// ~ 1000 x 4 D / T, about 1 % of rows (measured 1.3 % on rows spanning 16 decades of tau).
__global__ __launch_bounds__(256) void k_rho_red_cert(GridArgs A, int32_t* n_fallback) {
  __shared__ double tb[64];  // the f64 redo's exp table
  const int wave = gs_wave_id(), lane = threadIdx.x & 63;
  if (threadIdx.x < 64) tb[threadIdx.x] = GS_EXP2_64[threadIdx.x];
  __syncthreads();
  const int64_t nrow = (int64_t)A.n_psr * A.n_f * A.n_chain;
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + wave) * 64;
  if (r0 >= nrow) return;
  const int64_t r = r0 + lane;
  const bool rok = r < nrow;
  const int64_t rr = rok ? r : r0;
  const int c = (int)(rr % A.n_chain);
  const int k = (int)((rr / A.n_chain) % A.n_f);
  const int p = (int)(rr / ((int64_t)A.n_chain * A.n_f));
  double u;
  if (A.u) {
    u = A.u[((int64_t)c * A.n_psr + p) * A.n_f + k];
  } else {
    double u2;
    gs_uniform2(gs_counter(k, gs_sweep(A.sweep, A.sweep_dev), A.chain_base + c, p + A.psr_base, GS_EV_RED), A.key, u, u2);
  }
  const double tau = A.tau[rr];
  const double gw = A.irn[(int64_t)k * A.n_chain + c];
  const int S = -ilogb(A.grid3[0]);  // rho_min 2^S in [1, 2)
  // the lane's points in pairs for the packed f32 ops (v_pk_add / v_pk_mul / v_pk_fma_f32)
  gs_f2 rg2[RW_G / 2], on2[RW_G / 2];
#pragma unroll
  for (int j = 0; j < RW_G; ++j) {
    const int g = RW_G * lane + j;
    // off-grid slots: a = inf -> y = 0 -> t = 0, and the exponent's xm is masked by on = 0, so
    // e = 0 and E = 1: pdf' exactly 0
    rg2[j / 2][j % 2] = g < A.ngrid ? (float)ldexp(A.grid3[g], S) : __builtin_inff();
    on2[j / 2][j % 2] = g < A.ngrid ? 1.0f : 0.0f;
  }
  unsigned long long valid[RW_G];
#pragma unroll
  for (int j = 0; j < RW_G; ++j) valid[j] = __ballot(RW_G * lane + j < A.ngrid);
  const int nr = (int)min((int64_t)64, nrow - r0);
  const double sc = 1.4426950408889634 * 0.5 * ldexp(1.0, S);
  const float rgmax32 = (float)ldexp(A.grid3[A.ngrid - 1], S);
  int myidx = 0, nfb = 0;
  for (int i = 0; i < nr; ++i) {
    const double taui = rdlane(tau, i), gwi = rdlane(gw, i), ui = rdlane(u, i);
    int e;
    const double thm = frexp(0.5 * taui, &e);
    const float tl = (float)thm * 1.44269504f;
    const float tl2 = (float)(taui * sc);
    const float gw32 = (float)ldexp(gwi, S);
    // the row's smallest exponent (largest rho): E = 2^(xm - x) <= 1, the row maximum of e^-h
    // scaled to ~1, so the row never underflows as a whole
    const float xm = tl2 * __builtin_amdgcn_rcpf(gw32 + rgmax32);
    // Per pair of points: a = gw' + rho', y = 1/a, t = tl y, e = xm - tl2 y (one FMA: the
    // exponent's error is within the two-rounding form's the certificate assumes), E = 2^e,
    // pdf' = t E; w' = sum pdf' (-e), so that sum pdf' x = xm T + w' (x = xm - e).
    const gs_f2 gw2 = {gw32, gw32}, tlv = {tl, tl}, ntl2v = {-tl2, -tl2}, xm2 = {xm, xm};
    float cum[RW_G];
    float loc = 0.0f;
    gs_f2 w2 = {0.0f, 0.0f};
#pragma unroll
    for (int j = 0; j < RW_G; j += 2) {
      const gs_f2 a = gw2 + rg2[j / 2];
      const gs_f2 y = {__builtin_amdgcn_rcpf(a[0]), __builtin_amdgcn_rcpf(a[1])};
      const gs_f2 t = tlv * y;
      const gs_f2 e = __builtin_elementwise_fma(ntl2v, y, xm2 * on2[j / 2]);
      const gs_f2 E = {__builtin_amdgcn_exp2f(e[0]), __builtin_amdgcn_exp2f(e[1])};
      const gs_f2 pdf = t * E;
      w2 = __builtin_elementwise_fma(pdf, -e, w2);
      loc += pdf[0];
      cum[j] = loc;
      loc += pdf[1];
      cum[j + 1] = loc;
    }
    const float w = w2[0] + w2[1];
    float incl = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float v = __shfl_up(incl, o);
      if (lane >= o) incl += v;
    }
    float excl = __shfl_up(incl, 1);
    if (lane == 0) excl = 0.0f;
    float wsum = w;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) wsum += __shfl_xor(wsum, o);
    const float T = __shfl(incl, 63);
    wsum = fmaf(xm, T, wsum);  // sum pdf' x
    int idx = 0;
    bool done = false;
    if (T > 1e-33f && T < 3e38f && wsum < 3e38f) {  // wave-uniform
      // + the absolute error of points whose 2^(xm - x) is subnormal or flushed (t <= 1.45)
      const float D = 5.9604645e-08f * (80.0f * T + 18.0f * wsum + 12.0f * xm * T) + 2e-35f;
      const float uT = (float)ui * T;
      const float tlo = (uT - 2.0f * D) - excl, thr = (uT + 2.0f * D) - excl;
      int clo = 0, chi = 0;
#pragma unroll
      for (int j = 0; j < RW_G; ++j) {
        clo += __popcll(__ballot(cum[j] < tlo) & valid[j]);
        chi += __popcll(__ballot(cum[j] < thr) & valid[j]);
      }
      if (clo == chi) {
        idx = clo - 1;
        done = true;
      }
    }
    if (!done) {
      // unproven row (~1 % of rows: 1000 cdf values, each known to ~1e-6): redone in f64 with
      // k_rho_red_wave's arithmetic, so the default mode returns GS_OPT_GRID_EXACT = 2's index
      // on every row
      ++nfb;
      double rg[RW_G], cumd[RW_G];
#pragma unroll
      for (int j = 0; j < RW_G; ++j) {
        const int g = RW_G * lane + j;
        rg[j] = g < A.ngrid ? A.grid3[g] : 1e60;
      }
      const double locd = red_lane_cumsum<RW_G>(0.5 * taui, gwi, rg, tb, cumd);
      double incd = locd;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const double v = __shfl_up(incd, o);
        if (lane >= o) incd += v;
      }
      const double total = rdlane(incd, 63);
      const double thd = ui * total - (incd - locd);
      int cnt = 0;
#pragma unroll
      for (int j = 0; j < RW_G; ++j) cnt += __popcll(__ballot(cumd[j] < thd) & valid[j]);
      idx = cnt - 1;
    }
    if (idx < 0) idx += A.ngrid;
    myidx = (lane == i) ? idx : myidx;
  }
  if (rok) {
    if (A.idx_out) A.idx_out[r] = myidx;
    A.x[(int64_t)c * A.ldx + A.xcol[p * A.n_f + k]] = A.grid3[2 * A.ngrid + myidx];
  }
  if (n_fallback && lane == 0 && nfb) atomicAdd(n_fallback, nfb);
}

// ------------------------------------------------------------ a7 default: certified draw, 16 lanes per row
// k_rho_red_cert's arithmetic and certificate with the row spread over ONE DPP row of 16 lanes
// instead of the whole wave: row group g = lane >> 4 walks row 4 it + g of the wave's 64 rows, lane
// l = lane & 15 owning grid points [64 l, 64 l + 64) (ngrid <= 1024).
//
// Pass 1 keeps no per-point state: each lane sums its 64 pdf' = y E (the row constant tl of
// k_rho_red_cert cancels in cdf / total and is dropped) in four packed accumulators, and the lane
// totals are prefixed by a 4-step DPP row_shr scan (total: row_newbcast:15).  The searchsorted
// count is then taken at lane level: a lane whose last prefix is below a threshold contributes all
// of its points, one whose first prefix is not below contributes none, and the ONE lane that
// straddles it is recomputed by the whole row group, 4 points per lane (same f32 ops), prefixed by
// a second row scan and compared.  The counts are summed over the row by an integer DPP scan (lo
// and hi thresholds packed in one word).  Two straddling lanes (rounding can in principle break the
// lane-level order) or an unproven row take the f64 redo of k_rho_red_cert, wave-wide.
//
// Certificate: every prefix used (lane ends, first points, recomputed points, the total) is a sum
// of the exact prefix's terms with <= 24 roundings on any term's path (8 per accumulator + 3 to
// combine, 4 in the lane scan, 1 for the first point or 3 + 4 + 2 for a recomputed point), and
// pdf' = y E carries (8 + 5.6 x + 4.9 xm) eps (k_rho_red_cert's list without tl's 3 and one
// product), 3 roundings in the thresholds: D = eps (72 T + 18 w + 12 xm T) + 2e-35 (2 (8 + 24 +
// 3) < 72).  The lane-level classes are sound with each value D-accurate on its own: an "all"
// lane's points are truly below (C_j <= C_last <= end + D < uT - D), a "none" lane's truly not
// below, and the straddler's points are counted from D-accurate values, so the counts at uT -+ 2D
// bracket the exact count, and equal counts prove it.
// Measured (configs[3] rows near the posterior, 2048 chains, tools/ab_red_grid.py): 0.75 ms per
// launch with 1.34 % of rows redone in f64 (round-3 k_rho_red_cert: 1.22 ms, 1.45 %; the first
// 16-lane version, which kept the 64 running sums per lane and counted per group on the SALU:
// 1.12 ms, 2.6 %), indices equal to the f64 kernel's on every row.
constexpr int RQ_P = 64;  // grid points per lane (16 lanes per row)

template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {  // row-local DPP move, 0 from outside the row
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, true));
}
__device__ __forceinline__ float row_scan16(float x) {  // inclusive prefix over each 16-lane row
  x += dpp_f32<0x111>(x);                                // row_shr:1
  x += dpp_f32<0x112>(x);                                // row_shr:2
  x += dpp_f32<0x114>(x);                                // row_shr:4
  x += dpp_f32<0x118>(x);                                // row_shr:8
  return x;
}
__device__ __forceinline__ int row_scan16_i(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);
  return x;
}
__device__ __forceinline__ float row_last(float x) {  // lane 15 of each row to the whole row
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x15f, 0xf, 0xf, false));  // row_newbcast:15
}
__device__ __forceinline__ int row_last_i(int x) { return __builtin_amdgcn_mov_dpp(x, 0x15f, 0xf, 0xf, false); }

typedef float gs_f4 __attribute__((ext_vector_type(4)));

// Points 64 s + 4 l + q (q < 4) of row group g's lane s, recomputed by lane l: their prefixes
// within lane s's range, and the number below thresholds lo / hi among the nv valid ones.
struct StrCount {
  int lo, hi;
};
__device__ __forceinline__ StrCount red_straddler(const gs_f4* rlin4, int s, int l, int g, float excl, float gw32,
                                                  float ntl2, float xm, int ngrid, float tlo, float thr) {
  const gs_f4 rq = rlin4[16 * s + l];
  float P[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float y = __builtin_amdgcn_rcpf(gw32 + rq[q]);
    P[q] = y * __builtin_amdgcn_exp2f(fmaf(ntl2, y, xm));
  }
  const float q1 = P[0] + P[1], q2 = q1 + P[2], q3 = q2 + P[3];
  const float ex16 = dpp_f32<0x111>(row_scan16(q3));
  const float base = __shfl(excl, 16 * g + s) + ex16;
  const float c[4] = {base + P[0], base + q1, base + q2, base + q3};
  const int nv = min(max(ngrid - RQ_P * s - 4 * l, 0), 4);
  StrCount r = {0, 0};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    r.lo += (q < nv && c[q] < tlo) ? 1 : 0;
    r.hi += (q < nv && c[q] < thr) ? 1 : 0;
  }
  return r;
}

__global__ __launch_bounds__(256) void k_rho_red_cert16(GridArgs A, int32_t* n_fallback) {
  __shared__ double tb[64];          // the f64 redo's exp table
  __shared__ gs_f2 rgs[16 * RQ_P / 2];  // the scaled f32 grid, pair-major, for pass 1
  __shared__ gs_f4 rlin4[16 * RQ_P / 4];  // the same grid in point order, for the straddler recompute
  const int wave = gs_wave_id(), lane = threadIdx.x & 63;
  const int g = lane >> 4, l = lane & 15;
  const int S = -ilogb(A.grid3[0]);  // rho_min 2^S in [1, 2)
  if (threadIdx.x < 64) tb[threadIdx.x] = GS_EXP2_64[threadIdx.x];
  // off-grid slots: a = inf -> y = 0 -> E = 2^xm, finite (xm <= 100 below): pdf' exactly 0.
  // Pair-major (rgs[pair * 16 + lane]): the 16 lanes of a row read 16 consecutive 8-byte words per
  // point pair, bank-conflict free.
  for (int q = threadIdx.x; q < 16 * RQ_P; q += 256) {
    const int ln = q / RQ_P, jj = q % RQ_P;  // grid point q = 64 ln + jj
    const float v = q < A.ngrid ? (float)ldexp(A.grid3[q], S) : __builtin_inff();
    reinterpret_cast<float*>(rgs)[((jj / 2) * 16 + ln) * 2 + (jj & 1)] = v;
    reinterpret_cast<float*>(rlin4)[q] = v;
  }
  __syncthreads();
  const int64_t nrow = (int64_t)A.n_psr * A.n_f * A.n_chain;
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + wave) * 64;
  if (r0 >= nrow) return;
  const int64_t r = r0 + lane;
  const bool rok = r < nrow;
  const int64_t rr = rok ? r : r0;
  const int c = (int)(rr % A.n_chain);
  const int k = (int)((rr / A.n_chain) % A.n_f);
  const int p = (int)(rr / ((int64_t)A.n_chain * A.n_f));
  double u;
  if (A.u) {
    u = A.u[((int64_t)c * A.n_psr + p) * A.n_f + k];
  } else {
    double u2;
    gs_uniform2(gs_counter(k, gs_sweep(A.sweep, A.sweep_dev), A.chain_base + c, p + A.psr_base, GS_EV_RED), A.key, u, u2);
  }
  const double tau = A.tau[rr];
  const double gw = A.irn[(int64_t)k * A.n_chain + c];
  const gs_f2* rgl = rgs + l;  // this lane's point pairs at rgl[16 jp]
  const int nval = min(max(A.ngrid - RQ_P * l, 0), RQ_P);  // valid points of this lane
  const int nr = (int)min((int64_t)64, nrow - r0);
  const double sc = 1.4426950408889634 * 0.5 * ldexp(1.0, S);
  const float rgmax32 = (float)ldexp(A.grid3[A.ngrid - 1], S);
  int myidx = 0, nfb = 0;
  for (int it = 0; 4 * it < nr; ++it) {
    const int src = min(4 * it + g, nr - 1);  // this row group's row (a short last batch repeats one)
    const double taui = __shfl(tau, src), gwi = __shfl(gw, src), ui = __shfl(u, src);
    const float tl2 = (float)(taui * sc);
    const float gw32 = (float)ldexp(gwi, S);
    // the row's smallest exponent x (at rho_max), capped at 100 so an off-grid slot's 2^xm stays
    // finite; every on-grid e = xm - x is still <= 0 (a row with x > 226 everywhere underflows to
    // T = 0 and takes the f64 redo)
    const float xm = fminf(tl2 * __builtin_amdgcn_rcpf(gw32 + rgmax32), 100.0f);
    const gs_f2 gw2 = {gw32, gw32}, ntl2v = {-tl2, -tl2}, xm2 = {xm, xm};
    // pass 1: a = gw' + rho', y = 1/a, e = xm - tl2 y (one FMA), E = 2^e, pdf' = y E; the lane's
    // sum of pdf' and of pdf' e (so that sum pdf' x = xm T - sum pdf' e)
    gs_f2 acc[4] = {{0.0f, 0.0f}, {0.0f, 0.0f}, {0.0f, 0.0f}, {0.0f, 0.0f}};
    gs_f2 wacc[2] = {{0.0f, 0.0f}, {0.0f, 0.0f}};
    float p0 = 0.0f;
#pragma unroll
    for (int jp = 0; jp < RQ_P / 2; ++jp) {
      const gs_f2 a = gw2 + rgl[16 * jp];
      const gs_f2 y = {__builtin_amdgcn_rcpf(a[0]), __builtin_amdgcn_rcpf(a[1])};
      const gs_f2 ex = __builtin_elementwise_fma(ntl2v, y, xm2);
      const gs_f2 E = {__builtin_amdgcn_exp2f(ex[0]), __builtin_amdgcn_exp2f(ex[1])};
      const gs_f2 P = y * E;
      if (jp == 0) p0 = P[0];
      acc[jp & 3] += P;
      wacc[jp & 1] = __builtin_elementwise_fma(P, ex, wacc[jp & 1]);
    }
    const gs_f2 s2 = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    const gs_f2 w2 = wacc[0] + wacc[1];
    const float incl = row_scan16(s2[0] + s2[1]);
    const float excl = dpp_f32<0x111>(incl);  // row_shr:1: the previous lane's prefix, 0 on lane 0
    const float T = row_last(incl);
    const float wsum = fmaf(xm, T, -row_last(row_scan16(w2[0] + w2[1])));  // sum pdf' x over the row
    const bool okrow = T > 1e-33f && T < 3e38f && wsum < 3e38f;          // uniform per row group
    const float D = 5.9604645e-08f * (72.0f * T + 18.0f * wsum + 12.0f * xm * T) + 2e-35f;
    const float uT = (float)ui * T;
    const float tlo = uT - 2.0f * D, thr = uT + 2.0f * D;
    // lane classes for each threshold: all points below / none below / straddling (lanes past the
    // grid: none)
    const float c0 = excl + p0;
    const bool has = nval > 0;
    const bool lo_all = has && incl < tlo, hi_all = has && incl < thr;
    const bool lo_str = has && !lo_all && c0 < tlo, hi_str = has && !hi_all && c0 < thr;
    const unsigned long long m_lo = __ballot(lo_str), m_hi = __ballot(hi_str);
    const unsigned f_lo = (unsigned)(m_lo >> (16 * g)) & 0xffffu, f_hi = (unsigned)(m_hi >> (16 * g)) & 0xffffu;
    const int s_lo = f_lo ? __builtin_ctz(f_lo) : -1, s_hi = f_hi ? __builtin_ctz(f_hi) : -1;
    int cl = lo_all ? nval : 0, ch = hi_all ? nval : 0;
    // pass A: the lo straddler (else the hi one); pass B: a hi straddler in another lane
    const int sA = s_lo >= 0 ? s_lo : s_hi;
    if (__ballot(sA >= 0)) {
      const StrCount n = red_straddler(rlin4, max(sA, 0), l, g, excl, gw32, -tl2, xm, A.ngrid, tlo, thr);
      cl += (sA >= 0 && sA == s_lo) ? n.lo : 0;
      ch += (sA >= 0 && sA == s_hi) ? n.hi : 0;
    }
    const bool needB = s_hi >= 0 && s_lo >= 0 && s_hi != s_lo;
    if (__ballot(needB)) {
      const StrCount n = red_straddler(rlin4, max(s_hi, 0), l, g, excl, gw32, -tl2, xm, A.ngrid, tlo, thr);
      ch += needB ? n.hi : 0;
    }
    const int tot = row_last_i(row_scan16_i(cl | (ch << 16)));
    const int clo = tot & 0xffff, chi = tot >> 16;
    const bool proven = okrow && __builtin_popcount(f_lo) <= 1 && __builtin_popcount(f_hi) <= 1 && clo == chi;
    int idx = clo - 1;
    // unproven rows: k_rho_red_cert's f64 redo, the whole wave on one row (~1 % of rows)
    unsigned long long fbm = __ballot(!proven && l == 0 && 4 * it + g < nr);
    while (fbm) {
      const int gg = __builtin_ctzll(fbm) >> 4;
      fbm &= fbm - 1;
      ++nfb;
      const int rrow = 4 * it + gg;
      const double tr = rdlane(tau, rrow), gr = rdlane(gw, rrow), ur = rdlane(u, rrow);
      double rgd[RW_G], cumd[RW_G];
#pragma unroll
      for (int j = 0; j < RW_G; ++j) {
        const int gi = RW_G * lane + j;
        rgd[j] = gi < A.ngrid ? A.grid3[gi] : 1e60;
      }
      const double locd = red_lane_cumsum<RW_G>(0.5 * tr, gr, rgd, tb, cumd);
      double incd = locd;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const double v = __shfl_up(incd, o);
        if (lane >= o) incd += v;
      }
      const double total = rdlane(incd, 63);
      const double thd = ur * total - (incd - locd);
      int cnt = 0;
#pragma unroll
      for (int j = 0; j < RW_G; ++j) cnt += __popcll(__ballot(cumd[j] < thd && RW_G * lane + j < A.ngrid));
      idx = (g == gg) ? cnt - 1 : idx;
    }
    if (idx < 0) idx += A.ngrid;
    const int mine = __shfl(idx, 16 * (lane & 3));  // row 4 it + gg lives in row group gg
    myidx = ((lane >> 2) == it) ? mine : myidx;
  }
  if (rok) {
    if (A.idx_out) A.idx_out[r] = myidx;
    A.x[(int64_t)c * A.ldx + A.xcol[p * A.n_f + k]] = A.grid3[2 * A.ngrid + myidx];
  }
  if (n_fallback && lane == 0 && nfb) atomicAdd(n_fallback, nfb);
}

// ------------------------------------------------------------ a6' default: certified CURN-from-sums draw
// k_rho_curn_sum_wave's draw (log pdf_g = -P log rho_g - S w_g, w_g = 1/(2 rho_g), pta_gibbs.py:181-214
// with irn = 0) in f32 with k_rho_red_cert16's row layout, certificate shape and lane-level counts:
// 16 lanes per row, lane l owning grid points [64 l, 64 l + 64), unproven rows redone with the f64
// wave arithmetic (curn_sum_row_f64), so the default mode returns GS_OPT_GRID_EXACT = 2's index on
// every row.
//
// The exponent is taken relative to a reference point m near the row's mode (rho* = S / (2 P); any
// m is correct, a near one keeps the terms small): in log2 units e_g = -t1 - t2 with
// t1 = P' (log rho_g - log rho_m), t2 = S' (w_g - w_m), P' = P log2e, S' = S log2e.  The grid's
// log rho and w are held as f32 (hi, lo) pairs (~48 bits), so each difference is two f32
// subtractions and an add, relatively accurate to ~2 eps plus 2^-48 of the values, and t1, t2 have
// opposite signs (log rho rises, w falls along the grid): X_g = |t1 - t2| = |t1| + |t2|.  Per point
// the exponent's error is below 6.1 eps X_g + 2^-46 (P' L + S' w_m) (L = max |log rho|), so pdf'_g =
// 2^e_g carries eps (2 + 4.3 X_g) + 2^-46 (P' L + S' w_m) relative; with the 24 roundings of any
// prefix (k_rho_red_cert16's sums) every value used is within
//   D = eps (56 T + 9 W) + 2^-44 (P' L + S' w_m) T + 2e-35,   W = sum_g pdf'_g X_g,
// a margin of ~2 on every term.  Off-grid slots hold log rho = 1e30, so 2^e is exactly 0 there
// (S' w_m < 2^80 by the fixed-point window of S, far below P' 1e30).
__device__ __forceinline__ StrCount cs_straddler(const gs_f4* pts, int s, int l, int g, float excl, gs_f4 ref,
                                                 float Pp, float Sp, int ngrid, float tlo, float thr) {
  float P[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const gs_f4 t = pts[RQ_P * s + 4 * l + q];
    const float dl = (t[0] - ref[0]) + (t[1] - ref[1]);
    const float dw = (t[2] - ref[2]) + (t[3] - ref[3]);
    P[q] = __builtin_amdgcn_exp2f(-(Pp * dl) - (Sp * dw));
  }
  const float q1 = P[0] + P[1], q2 = q1 + P[2], q3 = q2 + P[3];
  const float ex16 = dpp_f32<0x111>(row_scan16(q3));
  const float base = __shfl(excl, 16 * g + s) + ex16;
  const float c[4] = {base + P[0], base + q1, base + q2, base + q3};
  const int nv = min(max(ngrid - RQ_P * s - 4 * l, 0), 4);
  StrCount r = {0, 0};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    r.lo += (q < nv && c[q] < tlo) ? 1 : 0;
    r.hi += (q < nv && c[q] < thr) ? 1 : 0;
  }
  return r;
}

// 8 point pairs per unrolled step at 3 waves/SIMD: a full unroll hoists all 256 table loads (391 VGPRs).
// CS_RPW rows per wave (4 at a time): the CURN line's 30 x 2048 rows are 960 waves at 64 (under one
// per SIMD: 0.060 ms), 3840 at 16 (0.0435 ms; 8: 0.0465, 32: 0.0458; f64 wave kernel 0.078).
#ifndef GS_CS_RPW
#define GS_CS_RPW 16
#endif
constexpr int CS_RPW = GS_CS_RPW;
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void k_rho_curn_sum_cert16(GridArgs A, int32_t* n_fallback) {
  __shared__ double tb[64];                   // the f64 redo's exp table
  __shared__ gs_f2 tab2[4][16 * RQ_P / 2];    // (log rho hi, lo, w hi, lo), pair-major for pass 1
  __shared__ gs_f4 pts[16 * RQ_P];            // the same per point, in order (straddler, reference)
  const int wave = gs_wave_id(), lane = threadIdx.x & 63;
  const int g = lane >> 4, l = lane & 15;
  const int n = A.ngrid;
  if (threadIdx.x < 64) tb[threadIdx.x] = GS_EXP2_64[threadIdx.x];
  for (int q = threadIdx.x; q < 16 * RQ_P; q += 256) {
    const bool on = q < n;
    const int qq = on ? q : n - 1;
    const double lr = A.grid3[n + qq], w = 0.5 / A.grid3[qq];
    const float lh = (float)lr, wh = (float)w;
    const gs_f4 v = {on ? lh : 1e30f, on ? (float)(lr - (double)lh) : 0.0f, wh, (float)(w - (double)wh)};
    pts[q] = v;
    const int ln = q / RQ_P, jj = q % RQ_P, o = ((jj / 2) * 16 + ln) * 2 + (jj & 1);
#pragma unroll
    for (int t = 0; t < 4; ++t) reinterpret_cast<float*>(tab2[t])[o] = v[t];
  }
  __syncthreads();
  const int64_t nrow = (int64_t)A.n_f * A.n_chain;
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + wave) * CS_RPW;
  if (r0 >= nrow) return;
  const int64_t r = r0 + lane;
  const bool rok = lane < CS_RPW && r < nrow;
  const int64_t rr = rok ? r : r0;
  const int c = (int)(rr % A.n_chain), k = (int)(rr / A.n_chain);
  double u;
  if (A.u) {
    u = A.u[(int64_t)c * A.n_f + k];
  } else {
    double u2;
    gs_uniform2(gs_counter(k, gs_sweep(A.sweep, A.sweep_dev), A.chain_base + c, 0, GS_EV_CURN), A.key, u, u2);
  }
  const double Srow = A.tau[rr];
  const double P = (double)A.n_psr;
  const float Pp = (float)(P * 1.4426950408889634);
  const double lr0 = A.grid3[n], lrn = A.grid3[2 * n - 1];
  const float L = (float)fmax(fabs(lr0), fabs(lrn));
  const float ih = n > 1 ? (float)((n - 1) / (lrn - lr0)) : 0.0f;  // grid points per unit log rho
  const int nval = min(max(n - RQ_P * l, 0), RQ_P);
  const int nr = (int)min((int64_t)CS_RPW, nrow - r0);
  const gs_f2* t0 = tab2[0] + l;
  const gs_f2* t1p = tab2[1] + l;
  const gs_f2* t2p = tab2[2] + l;
  const gs_f2* t3p = tab2[3] + l;
  int myidx = 0, nfb = 0;
  for (int it = 0; 4 * it < nr; ++it) {
    const int src = min(4 * it + g, nr - 1);
    const double S = __shfl(Srow, src), ui = __shfl(u, src);
    const float Sp = (float)(S * 1.4426950408889634);
    // the reference point: the grid point nearest the continuous mode rho* = S / (2 P), clamped
    const float lm = __builtin_amdgcn_logf((float)(S / (2.0 * P))) * 0.69314718f;  // ln rho*
    float mf = (lm - (float)lr0) * ih + 0.5f;
    mf = (mf == mf) ? fminf(fmaxf(mf, 0.0f), (float)(n - 1)) : 0.0f;
    const int m = (int)mf;
    const gs_f4 ref = pts[m];
    const gs_f2 r0h = {ref[0], ref[0]}, r0l = {ref[1], ref[1]}, r1h = {ref[2], ref[2]}, r1l = {ref[3], ref[3]};
    const gs_f2 Pp2 = {Pp, Pp}, Sp2 = {Sp, Sp};
    gs_f2 acc[4] = {{0.0f, 0.0f}, {0.0f, 0.0f}, {0.0f, 0.0f}, {0.0f, 0.0f}};
    gs_f2 wacc[2] = {{0.0f, 0.0f}, {0.0f, 0.0f}};
    float p0 = 0.0f;
#pragma unroll 8
    for (int jp = 0; jp < RQ_P / 2; ++jp) {
      const gs_f2 dl = (t0[16 * jp] - r0h) + (t1p[16 * jp] - r0l);
      const gs_f2 dw = (t2p[16 * jp] - r1h) + (t3p[16 * jp] - r1l);
      const gs_f2 a = Pp2 * dl, b = Sp2 * dw;
      const gs_f2 e = -a - b;
      const gs_f2 E = {__builtin_amdgcn_exp2f(e[0]), __builtin_amdgcn_exp2f(e[1])};
      const gs_f2 d = a - b;
      const gs_f2 X = {__builtin_fabsf(d[0]), __builtin_fabsf(d[1])};
      if (jp == 0) p0 = E[0];
      acc[jp & 3] += E;
      wacc[jp & 1] = __builtin_elementwise_fma(E, X, wacc[jp & 1]);
    }
    const gs_f2 s2 = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    const gs_f2 w2 = wacc[0] + wacc[1];
    const float incl = row_scan16(s2[0] + s2[1]);
    const float excl = dpp_f32<0x111>(incl);
    const float T = row_last(incl);
    const float W = row_last(row_scan16(w2[0] + w2[1]));
    const float swm = Sp * ref[2];  // S' w_m
    const bool okrow = T > 1e-33f && T < 3e38f && W < 3e38f && swm < 1e30f;
    const float D = 5.9604645e-08f * (56.0f * T + 9.0f * W) + 5.684342e-14f * (Pp * L + swm) * T + 2e-35f;
    const float uT = (float)ui * T;
    const float tlo = uT - 2.0f * D, thr = uT + 2.0f * D;
    const float c0 = excl + p0;
    const bool has = nval > 0;
    const bool lo_all = has && incl < tlo, hi_all = has && incl < thr;
    const bool lo_str = has && !lo_all && c0 < tlo, hi_str = has && !hi_all && c0 < thr;
    const unsigned long long m_lo = __ballot(lo_str), m_hi = __ballot(hi_str);
    const unsigned f_lo = (unsigned)(m_lo >> (16 * g)) & 0xffffu, f_hi = (unsigned)(m_hi >> (16 * g)) & 0xffffu;
    const int s_lo = f_lo ? __builtin_ctz(f_lo) : -1, s_hi = f_hi ? __builtin_ctz(f_hi) : -1;
    int cl = lo_all ? nval : 0, ch = hi_all ? nval : 0;
    const int sA = s_lo >= 0 ? s_lo : s_hi;
    if (__ballot(sA >= 0)) {
      const StrCount nn = cs_straddler(pts, max(sA, 0), l, g, excl, ref, Pp, Sp, n, tlo, thr);
      cl += (sA >= 0 && sA == s_lo) ? nn.lo : 0;
      ch += (sA >= 0 && sA == s_hi) ? nn.hi : 0;
    }
    const bool needB = s_hi >= 0 && s_lo >= 0 && s_hi != s_lo;
    if (__ballot(needB)) {
      const StrCount nn = cs_straddler(pts, max(s_hi, 0), l, g, excl, ref, Pp, Sp, n, tlo, thr);
      ch += needB ? nn.hi : 0;
    }
    const int tot = row_last_i(row_scan16_i(cl | (ch << 16)));
    const int clo = tot & 0xffff, chi = tot >> 16;
    const bool proven = okrow && __builtin_popcount(f_lo) <= 1 && __builtin_popcount(f_hi) <= 1 && clo == chi;
    int idx = clo - 1;
    unsigned long long fbm = __ballot(!proven && l == 0 && 4 * it + g < nr);
    while (fbm) {  // unproven rows: k_rho_curn_sum_wave's f64 arithmetic, the whole wave on one row
      const int gg = __builtin_ctzll(fbm) >> 4;
      fbm &= fbm - 1;
      ++nfb;
      const int rrow = 4 * it + gg;
      double cg[CSW_G], wg[CSW_G];
      unsigned long long valid[CSW_G];
#pragma unroll
      for (int j = 0; j < CSW_G; ++j) {
        const int gi = CSW_G * lane + j;
        const bool ok = gi < n;
        cg[j] = ok ? -P * A.grid3[n + gi] : -1e300;
        wg[j] = ok ? 0.5 / A.grid3[gi] : 0.0;
        valid[j] = __ballot(ok);
      }
      const int id = curn_sum_row_f64(-rdlane(Srow, rrow), rdlane(u, rrow), cg, wg, valid, tb, lane);
      idx = (g == gg) ? id : idx;
    }
    if (idx < 0) idx += n;
    const int mine = __shfl(idx, 16 * (lane & 3));
    myidx = ((lane >> 2) == it) ? mine : myidx;
  }
  if (rok) {
    if (A.idx_out) A.idx_out[r] = myidx;
    A.x[(int64_t)c * A.ldx + A.xcol[k]] = A.grid3[2 * n + myidx];
  }
  if (n_fallback && lane == 0 && nfb) atomicAdd(n_fallback, nfb);
}

// ------------------------------------------------------------ a4: Gumbel-max
// rows r = k * n_chain + c (one pulsar, systems = chains); tau half-convention.
// logpdf = log tau - logaddexp(log irn, log rho) - exp(...); argmax(logpdf + G),
// G = -log(-log1p(-U))  (numpy legacy gumbel), first maximum on ties.
__global__ void k_rho_gumbel(GridArgs A) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nrow = (int64_t)A.n_f * A.n_chain;
  if (r >= nrow) return;
  const int c = (int)(r % A.n_chain), k = (int)(r / A.n_chain);
  const double ltau = log(A.tau[r]);
  const double lirn = log(A.irn[r]);
  double best = -__builtin_inf();
  int bi = 0;
  for (int g = 0; g < A.ngrid; ++g) {
    double u;
    if (A.u) {
      u = A.u[((int64_t)c * A.n_f + k) * A.ngrid + g];
    } else {
      double u2;
      gs_uniform2(gs_counter((uint32_t)(k * 1024 + g), gs_sweep(A.sweep, A.sweep_dev), A.chain_base + c, 0, GS_EV_GUMBEL), A.key,
                  u, u2);
    }
    const double lr = ltau - np_logaddexp(lirn, A.grid3[A.ngrid + g]);
    const double lp = lr - exp(lr);
    const double gum = 0.0 - 1.0 * log(-log1p(-u));
    const double v = lp + gum;
    if (v > best) {
      best = v;
      bi = g;
    }
  }
  if (A.idx_out) A.idx_out[r] = bi;
  A.x[(int64_t)c * A.ldx + A.xcol[k]] = A.grid3[2 * A.ngrid + bi];
}

// ------------------------------------------------------------ phi from x
// out[j][c] = 10**(2 x[c][cols[j]])  (enterprise free_spectrum phi, sin column)
__global__ void k_phi_from_x(int n_chain, int ncol, const double* x, int ldx, const int32_t* cols,
                             double* out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)n_chain * ncol) return;
  const int c = (int)(t % n_chain), j = (int)(t / n_chain);
  out[t] = pow(10.0, 2.0 * x[(int64_t)c * ldx + cols[j]]);
}

// Per-pulsar power-law red phi at the sin columns: out[p][k][c] = exp((a_pk la_p + c_pk) +
// g_pk ga_p) with (la_p, ga_p) = x[c][pl_col[2p]], x[c][pl_col[2p+1]] and lnphi [n_psr x 3 x n_f]
// = (c, a, g) -- the red_sig[p].get_phi(params)[::2] of pta_gibbs.py:198, rounded as gs_hyper_mh
// computes it.
__global__ void k_phi_powerlaw(int n_psr, int n_chain, int n_f, const double* x, int ldx, const int32_t* pl_col,
                               const double* lnphi, double* out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)n_psr * n_f * n_chain) return;
  const int c = (int)(t % n_chain);
  const int64_t pk = t / n_chain;
  const int p = (int)(pk / n_f), k = (int)(pk % n_f);
  const double* xc = x + (int64_t)c * ldx;
  const double la = xc[pl_col[2 * p]], ga = xc[pl_col[2 * p + 1]];
  const double* L = lnphi + (int64_t)p * 3 * n_f;
  out[t] = exp(gs_add_rn(gs_add_rn(gs_mul_rn(L[n_f + k], la), L[k]), gs_mul_rn(L[2 * n_f + k], ga)));
}

// ------------------------------------------------------------ PTA record / gate / phiinv
// record: x_rec[c][:] = x[c][:], xlast[c] = x[c][n_param-1]  (pta_gibbs.py:666)
__global__ void k_pta_record(int n_chain, int n_param, const double* x, double* x_rec, double* xlast) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)n_chain * n_param) return;
  if (x_rec) x_rec[t] = x[t];
  if ((t % n_param) == n_param - 1) xlast[t / n_param] = x[t];
}

// gate[c] = all_j x[c][j] != xlast[c]  (pta_gibbs.py:703); one wavefront per chain.
// phiinv_F[p*n_chain + c][2k + {0,1}] = 1 / (10**(2 x_gw[k]) + 10**(2 x_red[p][k]))
__global__ void k_pta_gate_phiinv(PtaGateArgs A) {
  const int c = blockIdx.x;
  const int lane = threadIdx.x;
  const double* xc = A.x + (int64_t)c * A.n_param;
  const double xl = A.xlast ? A.xlast[c] : __builtin_nan("");
  bool same = false;
  for (int j = lane; j < A.n_param; j += 64) same |= (xc[j] == xl);
  const bool gate = __ballot(same) == 0ull;
  if (lane == 0) A.gate[c] = A.xlast ? (gate ? 1 : 0) : 1;
  if (A.n_f <= 64) {
    // the common part once per frequency (lane k), shared by every pulsar through a lane
    // shuffle: phi_gw (+ irn) and, without per-pulsar red noise, its reciprocal (the CURN
    // sweep's phiinv is the same for all pulsars: n_f instead of n_psr n_f pows per chain)
    __shared__ double phg_s[64], ping_s[64];  // one wave per workgroup
    const int kk = lane < A.n_f ? lane : 0;
    double phg = pow(10.0, 2.0 * xc[A.gw_col[kk]]);
    if (A.irn) phg = phg + A.irn[(int64_t)kk * A.n_chain + c];
    phg_s[lane] = phg;
    ping_s[lane] = 1.0 / phg;
    wave_lds_sync();
    for (int t = lane; t < A.n_psr * A.n_f; t += 64) {
      const int p = t / A.n_f, k = t % A.n_f;
      double pinv;
      if (A.irn_pp) {
        const double phi = phg_s[k] + A.irn_pp[((int64_t)p * A.n_f + k) * A.n_chain + c];
        pinv = 1.0 / phi;
      } else if (A.red_col) {
        const double phi = phg_s[k] + pow(10.0, 2.0 * xc[A.red_col[p * A.n_f + k]]);
        pinv = 1.0 / phi;
      } else {
        pinv = ping_s[k];
      }
      double* o = A.phiinv_F + ((int64_t)p * A.n_chain + c) * (2 * A.n_f);
      o[2 * k] = pinv;
      o[2 * k + 1] = pinv;
    }
  } else {
    for (int t = lane; t < A.n_psr * A.n_f; t += 64) {
      const int p = t / A.n_f, k = t % A.n_f;
      double phi = pow(10.0, 2.0 * xc[A.gw_col[k]]);
      if (A.red_col) phi = phi + pow(10.0, 2.0 * xc[A.red_col[p * A.n_f + k]]);
      if (A.irn) phi = phi + A.irn[(int64_t)k * A.n_chain + c];
      if (A.irn_pp) phi = phi + A.irn_pp[((int64_t)p * A.n_f + k) * A.n_chain + c];
      const double pinv = 1.0 / phi;
      double* o = A.phiinv_F + ((int64_t)p * A.n_chain + c) * (2 * A.n_f);
      o[2 * k] = pinv;
      o[2 * k + 1] = pinv;
    }
  }
}

__global__ void k_counter_add(int64_t* counter, int64_t inc) {
  if (threadIdx.x == 0) *counter += inc;
}

inline dim3 grid1(int64_t n, int bs) { return dim3((unsigned)((n + bs - 1) / bs)); }

}  // namespace

int launch_tau(hipStream_t s, const TauArgs& a) {
  const int64_t n = (int64_t)a.n_psr * (a.NF / 2) * a.n_chain;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_tau, grid1(n, 256), dim3(256), 0, s, a);
  return 0;
}

int launch_rho_curn(hipStream_t s, const GridArgs& a) {
  const int64_t n = (int64_t)a.n_f * a.n_chain;
  if (n == 0) return 0;
  if (a.exact != 1 && a.ngrid <= 64 * CF_MAXG) {
    // CF_K = 5 where ceil(P / 5) groups of 12 ops beat ceil(P / 4) groups of 10 per grid point
    const int p4 = (a.n_psr + 3) / 4 * 10, p5 = (a.n_psr + 4) / 5 * 12;
    if (GS_CF_AUTOK && p5 < p4)
      hipLaunchKernelGGL(k_rho_curn_fast<5>, grid1(n, 4), dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL(k_rho_curn_fast<4>, grid1(n, 4), dim3(256), 0, s, a);
    return 0;
  }
  const size_t lds = (size_t)GS_CURN_WPB * a.ngrid * sizeof(double);
  hipLaunchKernelGGL(k_rho_curn, grid1(n, GS_CURN_WPB), dim3(64 * GS_CURN_WPB), lds, s, a);
  return 0;
}

int launch_counter_add(hipStream_t s, int64_t* counter, int64_t inc) {
  hipLaunchKernelGGL(k_counter_add, dim3(1), dim3(64), 0, s, counter, inc);
  return 0;
}

int launch_tau_sum_fx(hipStream_t s, int n_psr, int64_t nrow, const double* tau, int e0, long long* acc, int* ovf) {
  if (nrow == 0) return 0;
  hipLaunchKernelGGL(k_tau_sum_fx, grid1(nrow, 256), dim3(256), 0, s, n_psr, nrow, tau, e0, acc, ovf);
  return 0;
}

int launch_tau_sum_fx_b(hipStream_t s, const TauArgs& a, int e0, long long* acc, int* ovf) {
  if ((int64_t)(a.NF / 2) * a.n_chain == 0) return 0;
  if (a.NF > 64) return 1;  // one lane per free-spectrum column
  hipLaunchKernelGGL(k_tau_sum_fx_b, dim3((unsigned)a.n_chain), dim3(256), 0, s, a, e0, acc, ovf);
  return 0;
}

int launch_fx_to_double(hipStream_t s, int64_t nrow, int e0, const long long* acc, double* S) {
  if (nrow == 0) return 0;
  hipLaunchKernelGGL(k_fx_to_double, grid1(nrow, 256), dim3(256), 0, s, nrow, e0, acc, S);
  return 0;
}

int launch_tau_sum(hipStream_t s, int n_psr, int64_t nrow, const double* tau, double* S) {
  if (nrow == 0) return 0;
  hipLaunchKernelGGL(k_tau_sum, grid1(nrow, 256), dim3(256), 0, s, n_psr, nrow, tau, S);
  return 0;
}

int launch_rho_curn_sum(hipStream_t s, const GridArgs& a) {
  const int64_t n = (int64_t)a.n_f * a.n_chain;
  if (n == 0) return 0;
  if (a.ngrid <= 16 * RQ_P && a.exact == 0)
    hipLaunchKernelGGL(k_rho_curn_sum_cert16, grid1(n, 4 * CS_RPW), dim3(256), 0, s, a, a.n_fallback);
  else if (a.ngrid <= 64 * CSW_G)
    hipLaunchKernelGGL(k_rho_curn_sum_wave<GS_CSW_RPW>, grid1(n, 4 * GS_CSW_RPW), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(k_rho_curn_sum, grid1(n, 4), dim3(256), 0, s, a);
  return 0;
}

int launch_rho_red(hipStream_t s, const GridArgs& a) {
  const int64_t n = (int64_t)a.n_psr * a.n_f * a.n_chain;
  if (n == 0) return 0;
  if (a.exact == 1)
    hipLaunchKernelGGL(k_rho_red<true>, grid1(n, 64), dim3(64), 0, s, a);
  else if (a.ngrid <= 16 * RQ_P && a.exact == 0)
    hipLaunchKernelGGL(k_rho_red_cert16, grid1(n, 256), dim3(256), 0, s, a, a.n_fallback);
  else if (a.ngrid <= 64 * RW_G && (a.exact == 0 || a.exact == 3))
    hipLaunchKernelGGL(k_rho_red_cert, grid1(n, 256), dim3(256), 0, s, a, a.n_fallback);
  else if (a.ngrid <= 64 * RW_G)
    hipLaunchKernelGGL(k_rho_red_wave, grid1(n, 256), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(k_rho_red<false>, grid1(n, 64), dim3(64), 0, s, a);
  return 0;
}

int launch_rho_gumbel(hipStream_t s, const GridArgs& a) {
  const int64_t n = (int64_t)a.n_f * a.n_chain;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_rho_gumbel, grid1(n, 64), dim3(64), 0, s, a);
  return 0;
}

int launch_phi_from_x(hipStream_t s, int n_chain, int ncol, const double* x, int ldx, const int32_t* cols,
                      double* out) {
  const int64_t n = (int64_t)n_chain * ncol;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_phi_from_x, grid1(n, 256), dim3(256), 0, s, n_chain, ncol, x, ldx, cols, out);
  return 0;
}

int launch_phi_powerlaw(hipStream_t s, int n_psr, int n_chain, int n_f, const double* x, int ldx,
                        const int32_t* pl_col, const double* lnphi, double* out) {
  const int64_t n = (int64_t)n_psr * n_f * n_chain;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_phi_powerlaw, grid1(n, 256), dim3(256), 0, s, n_psr, n_chain, n_f, x, ldx, pl_col, lnphi,
                     out);
  return 0;
}

int launch_pta_record(hipStream_t s, int n_chain, int n_param, const double* x, double* x_rec, double* xlast) {
  const int64_t n = (int64_t)n_chain * n_param;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_pta_record, grid1(n, 256), dim3(256), 0, s, n_chain, n_param, x, x_rec, xlast);
  return 0;
}

int launch_pta_gate_phiinv(hipStream_t s, const PtaGateArgs& a) {
  if (a.n_chain == 0) return 0;
  hipLaunchKernelGGL(k_pta_gate_phiinv, dim3(a.n_chain), dim3(64), 0, s, a);
  return 0;
}
