// (a10) White-noise Metropolis block and the per-chain TNT it forces (gfx950, fp64).
//
// Reference: PulsarBlockGibbs.update_white_params pulsar_gibbs.py:332-406 (steady
// state :373-404), get_lnlikelihood_white :523-546, get_lnprior :613-617, and the
// per-sweep TNT recompute :500-502 / :664-665.
//
// The white likelihood is a sum over TOAs; grouping a pulsar's TOAs by backend
// makes it a sum of per-backend terms S_k, and a single-parameter proposal only
// changes one backend's term.  Each MH step therefore re-sums only that backend's
// TOAs (n_toa / n_bk of the reference's full recompute, which also redoes T b every
// step although b is fixed) and the acceptance uses dlnL = -(S_k' - S_k) / 2.
#include <cstdlib>

#include "gibbs_common.h"
#include "gibbs_internal.h"

namespace {

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Effect of one white parameter value on its backend's (efac^2, t2equad^2, tnequad^2).
__device__ __forceinline__ void apply_white(int kind, double v, double& ef2, double& t2, double& tn) {
  if (kind == GS_WHITE_EFAC) {
    ef2 = v * v;
  } else if (kind == GS_WHITE_TNEQUAD) {
    tn = pow(10.0, 2.0 * v);
  } else {
    t2 = pow(10.0, 2.0 * v);
  }
}

// sum over TOAs [lo, hi) of log N + y^2 / N, N = ef2 (sigma^2 + t2) + tn (whole wave).
__device__ __forceinline__ double backend_sum(const double* __restrict__ s2, const double* __restrict__ y,
                                              int lo, int hi, double ef2, double t2, double tn, int lane) {
  double s = 0.0;
  for (int i = lo + lane; i < hi; i += GS_WAVE) {
    const double N = ef2 * (s2[i] + t2) + tn;
    const double yy = y[i];
    s += log(N) + yy * yy / N;
  }
  return wave_sum(s);
}

constexpr int MH_WPB = 4;

// grid (ceil(n_chain / MH_WPB), n_psr); one wavefront per (pulsar, chain) system.
__global__ __launch_bounds__(64 * MH_WPB) void k_white_mh(WhiteMhArgs A) {
  __shared__ double sb[MH_WPB][4][GS_WHITE_MAX_BK + 1];  // ef2, t2, tn, S per backend
  __shared__ double sx[MH_WPB][GS_WHITE_MAX_W];         // current white parameter values
  const int wave = gs_wave_id(), lane = threadIdx.x & 63;
  const int p = blockIdx.y;
  const int c = blockIdx.x * MH_WPB + wave;
  if (c >= A.n_chain) return;  // no workgroup barriers below
  const gs_white_desc* D = A.wdesc + p;  // bk_off is indexed at run time: keep it in memory
  const int64_t n_sys = (int64_t)A.n_psr * A.n_chain;
  const int64_t sys = (int64_t)p * A.n_chain + c;
  const long long gchain = A.chain_base + c;
  const int nbk = D->n_bk, nw = D->n_w;
  double* ef2 = sb[wave][0];
  double* t2 = sb[wave][1];
  double* tn = sb[wave][2];
  double* S = sb[wave][3];
  double* xs = sx[wave];
  const int64_t woff = D->w_off;
  const double* s2 = A.sigma2 + D->toa_off;
  const double* y = A.y + c * A.ldy + D->toa_off;
  double* x = A.x + (A.x_per_sys ? sys : (int64_t)c) * A.ldx;
  const int32_t* wcol = A.wcol + woff;
  const int32_t* wkind = A.wkind + woff;
  const int32_t* wbk = A.wbk + woff;
  const int32_t* bko = D->bk_off;

  if (lane < nbk) {
    ef2[lane] = 1.0;
    t2[lane] = 0.0;
    tn[lane] = 0.0;
  }
  wave_lds_sync();
  if (lane < nw) {
    const double v = x[wcol[lane]];
    xs[lane] = v;
    const int k = wbk[lane];
    double e = 1.0, t = 0.0, q = 0.0;
    apply_white(wkind[lane], v, e, t, q);
    if (wkind[lane] == GS_WHITE_EFAC) ef2[k] = e;
    else if (wkind[lane] == GS_WHITE_TNEQUAD) tn[k] = q;
    else t2[k] = t;
  }
  wave_lds_sync();
  for (int k = 0; k < nbk; ++k) {
    const double s = backend_sum(s2, y, bko[k], bko[k + 1], ef2[k], t2[k], tn[k], lane);
    if (lane == 0) S[k] = s;
  }
  wave_lds_sync();

  const int steps = A.nsteps_chain ? A.nsteps_chain[A.x_per_sys ? sys : (int64_t)c] : A.n_steps;
  const double sig = 0.05 * nw;  // sigmas = 0.05 * len(wind)  (:376)
  int nacc = 0;
  for (int st = 0; st < steps; ++st) {
    double sc, z, u;
    int w;
    if (A.inj) {
      const double* q = A.inj + ((int64_t)st * n_sys + sys) * 4;
      sc = q[0];
      w = (int)q[1];
      z = q[2];
      u = q[3];
    } else {
      double u1, u2, v1, v2, u4;
      const int ps = p + A.psr_base;
      gs_uniform2(gs_counter(3u * st, gs_sweep(A.sweep, A.sweep_dev), gchain, ps, GS_EV_WHITE), A.key, u1, u2);
      gs_uniform2(gs_counter(3u * st + 1, gs_sweep(A.sweep, A.sweep_dev), gchain, ps, GS_EV_WHITE), A.key, v1, v2);
      gs_uniform2(gs_counter(3u * st + 2, gs_sweep(A.sweep, A.sweep_dev), gchain, ps, GS_EV_WHITE), A.key, u, u4);
      sc = gs_mh_scale(u1);
      w = min((int)(u2 * nw), nw - 1);
      z = sqrt(-2.0 * log(1.0 - v1)) * cospi(2.0 * v2);
    }
    // q[par] += randn * sigmas * scale  (:383)
    const double xo = xs[w];
    const double xq = gs_add_rn(xo, gs_mul_rn(gs_mul_rn(z, sig), sc));  // numpy's rounding (no fma)
    if (A.q_rec && lane < nw)
      A.q_rec[((int64_t)st * n_sys + sys) * GS_WHITE_MAX_W + lane] = (lane == w) ? xq : xs[lane];
    // Uniform prior: -inf outside [pmin, pmax] -> diff = -inf, rejected (:613-617, :398)
    if (xq >= A.wmin[woff + w] && xq <= A.wmax[woff + w]) {
      const int k = wbk[w];
      double e = ef2[k], t = t2[k], q = tn[k];
      apply_white(wkind[w], xq, e, t, q);
      const double sn = backend_sum(s2, y, bko[k], bko[k + 1], e, t, q, lane);
      const double diff = (-0.5 * sn) - (-0.5 * S[k]);
      if (diff > log(u)) {
        ++nacc;
        if (lane == 0) {
          ef2[k] = e;
          t2[k] = t;
          tn[k] = q;
          S[k] = sn;
          xs[w] = xq;
        }
      }
      wave_lds_sync();
    }
  }
  if (lane < nw) x[wcol[lane]] = xs[lane];
  if (A.n_acc && lane == 0) A.n_acc[sys] = nacc;
}

// y = r - T b: grid (ceil(n_toa_max / 256), n_psr, ceil(n_chain / RES_CT)); one thread
// per TOA, RES_CT chains per thread; T column-major so each load is coalesced and
// b is wave-uniform (scalar loads).
constexpr int RES_CT = 8;

__global__ __launch_bounds__(256) void k_white_resid(WhiteResidArgs A) {
  const gs_tnt_desc D = A.tdesc[blockIdx.y];
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= D.n_toa) return;
  const int p = blockIdx.y;
  const int c0 = blockIdx.z * RES_CT;
  const int m = (int)D.m;
  const int64_t n = D.n_toa;
  const double* Tt = A.Tt + D.T_off;
  const double* bb[RES_CT];
#pragma unroll
  for (int q = 0; q < RES_CT; ++q)
    bb[q] = A.b + ((int64_t)p * A.n_chain + min(c0 + q, A.n_chain - 1)) * A.ldb;
  double acc[RES_CT];
#pragma unroll
  for (int q = 0; q < RES_CT; ++q) acc[q] = 0.0;
  for (int j = 0; j < m; ++j) {
    const double t = Tt[(int64_t)j * n + i];
#pragma unroll
    for (int q = 0; q < RES_CT; ++q) acc[q] = fma(t, bb[q][j], acc[q]);
  }
  const double r = A.r[D.toa_off + i];
#pragma unroll
  for (int q = 0; q < RES_CT; ++q)
    if (c0 + q < A.n_chain) A.y[(int64_t)(c0 + q) * A.ldy + D.toa_off + i] = r - acc[q];
}


typedef double gs_d4_t __attribute__((ext_vector_type(4)));

// y = r - T b as an fp64 MFMA GEMM: Y (chains x TOAs) = B (chains x m) T^T, one wavefront per
// 16 x 16 tile (16 chains of a pulsar x 16 TOAs), K = m in v_mfma_f64_16x16x4f64 steps: the A
// operand is b[c0 + i][j0 + k] (lane i = l & 15, k = l >> 4), the B operand T[t0 + i][j0 + k]
// from the column-major copy (16 consecutive TOAs per k: coalesced).  Output C layout: register
// s of lane (i, k) is Y[c0 + 4 s + k][t0 + i].  grid (ceil(n_toa_max / 64), n_psr,
// ceil(n_chain / 16)), 4 waves per workgroup (consecutive TOA tiles).
__global__ __launch_bounds__(256) void k_white_resid_mfma(WhiteResidArgs A) {
  const gs_tnt_desc D = A.tdesc[blockIdx.y];
  const int w = gs_wave_id(), l = threadIdx.x & 63, i = l & 15, k = l >> 4;
  const int64_t t0 = ((int64_t)blockIdx.x * 4 + w) * 16;
  if (t0 >= D.n_toa) return;  // wave-uniform, no barriers
  const int p = blockIdx.y;
  const int c0 = blockIdx.z * 16;
  const int m = (int)D.m;
  const int64_t n = D.n_toa;
  const double* Tt = A.Tt + D.T_off;
  const int ca = min(c0 + i, A.n_chain - 1);
  const double* brow = A.b + ((int64_t)p * A.n_chain + ca) * A.ldb;
  const int64_t tb = min(t0 + i, n - 1);
  gs_d4_t acc = {0.0, 0.0, 0.0, 0.0};
  int j0 = 0;
  for (; j0 + 16 <= m; j0 += 16) {  // 4 steps per iteration, loads issued together
    double av[4], bv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = j0 + 4 * u + k;
      av[u] = brow[j];
      bv[u] = Tt[(int64_t)j * n + tb];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u], bv[u], acc, 0, 0, 0);
  }
  for (; j0 < m; j0 += 4) {
    const int j = j0 + k;
    const double a = (j < m) ? brow[j] : 0.0;
    const double b = (j < m) ? Tt[(int64_t)j * n + tb] : 0.0;
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
  const int64_t t = t0 + i;
  if (t < n) {
    const double r = A.r[D.toa_off + t];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int c = c0 + 4 * s + k;
      if (c < A.n_chain) A.y[(int64_t)c * A.ldy + D.toa_off + t] = r - acc[s];
    }
  }
}

// Per-backend noise values of system (p, c) into LDS (whole workgroup).
// xrow: the row of x holding this system's white parameters (chain c, or system
// p * n_chain + c under GS_OPT_X_PER_SYS)
__device__ __forceinline__ void stage_white(const WhiteTntArgs& A, const gs_white_desc& W, int64_t xrow,
                                            double* ef2, double* t2, double* tn) {
  const int tid = threadIdx.x;
  if (tid < W.n_bk) {
    ef2[tid] = 1.0;
    t2[tid] = 0.0;
    tn[tid] = 0.0;
  }
  __syncthreads();
  if (tid < W.n_w) {
    const int64_t o = W.w_off + tid;
    const int k = A.wbk[o], kind = A.wkind[o];
    double e = 1.0, t = 0.0, q = 0.0;
    apply_white(kind, A.x[xrow * A.ldx + A.wcol[o]], e, t, q);
    if (kind == GS_WHITE_EFAC) ef2[k] = e;
    else if (kind == GS_WHITE_TNEQUAD) tn[k] = q;
    else t2[k] = t;
  }
  __syncthreads();
}

typedef double d4 __attribute__((ext_vector_type(4)));
typedef d4 gs_d4_t;

// TNT_c: grid (n_sys, nb (nb + 1) / 2) lower 16 x 16 tile pairs, mirrored on store;
// 4 wavefronts split the TOAs, v_mfma_f64_16x16x4f64 (layout as k_tnt).
__global__ __launch_bounds__(256) void k_white_tnt(WhiteTntArgs A) {
  __shared__ double red[3][4][64];
  __shared__ double sb[3][GS_WHITE_MAX_BK + 1];
  const int64_t sys = blockIdx.x;
  const int p = (int)(sys / A.n_chain), c = (int)(sys % A.n_chain);
  const int q = blockIdx.y;
  int bi = (int)((sqrt(8.0 * q + 1.0) - 1.0) * 0.5);
  while ((bi + 1) * (bi + 2) / 2 <= q) ++bi;
  while (bi * (bi + 1) / 2 > q) --bi;
  const int bj = q - bi * (bi + 1) / 2;
  const gs_tnt_desc D = A.tdesc[p];
  const gs_white_desc W = A.wdesc[p];
  const int m = (int)D.m;
  if (bi * 16 >= m) return;
  stage_white(A, W, A.x_per_sys ? sys : (int64_t)c, sb[0], sb[1], sb[2]);
  const int w = gs_wave_id(), l = threadIdx.x & 63;
  const int i = l & 15, k = l >> 4;
  const int ci = bi * 16 + i, cj = bj * 16 + i;
  const double* Tp = A.T + D.T_off;
  const double* s2 = A.sigma2 + D.toa_off;
  const int32_t* bk = A.bk + D.toa_off;
  const int64_t n = D.n_toa;
  d4 acc = {0.0, 0.0, 0.0, 0.0};
  for (int64_t t0 = (int64_t)w * 4; t0 < n; t0 += 16) {
    const int64_t t = t0 + k;
    const bool ok = t < n;
    double invN = 0.0;
    if (ok) {
      const int kb = bk[t];
      invN = 1.0 / (sb[0][kb] * (s2[t] + sb[1][kb]) + sb[2][kb]);
    }
    const double a = (ok && ci < m) ? Tp[t * m + ci] * invN : 0.0;
    const double b = (ok && cj < m) ? Tp[t * m + cj] : 0.0;
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
  if (w > 0)
    for (int r = 0; r < 4; ++r) red[w - 1][r][l] = acc[r];
  __syncthreads();
  if (w == 0) {
    double* out = A.TNT + D.tnt_off + (int64_t)c * A.tnt_cstride;
    for (int r = 0; r < 4; ++r) {
      const double v = acc[r] + red[0][r][l] + red[1][r][l] + red[2][r][l];
      const int row = bi * 16 + (l >> 4) + 4 * r, col = bj * 16 + (l & 15);
      if (row < m && col < m) {
        out[(int64_t)row * m + col] = v;
        out[(int64_t)col * m + row] = v;
      }
    }
  }
}

// ---------------------------------------------------------------- batched SYRK
// TNT_c and d_c in ONE pass over T per system (configs 5 and white-noise pulsars):
// the system's T is augmented by r as column m, so the lower 16 x 16 tiles of
// [T | r]^T N_c^-1 [T | r] hold TNT_c and, in row m, d_c.  One workgroup (8 waves)
// per system streams T through LDS in chunks of SY_TC TOAs (double-buffered, one
// barrier per chunk); wave w accumulates tiles w, w + 8, ... in registers with
// v_mfma_f64_16x16x4f64 (A = T[t][bi*16+i] / N[t], B = T[t][bj*16+i]; the k_tnt
// layout).  Workgroups are mapped XCD-major so the chains of one pulsar share an
// XCD's L2 for T.  Roofline: fp64 MFMA (n m^2 flop per system against 8 n m bytes).
constexpr int SY_WAVES = 8;
constexpr int SY_TC = 32;

__host__ __device__ constexpr int sy_ld(int nb) { return 16 * nb + ((nb & 1) ? 0 : 16); }

// Tile ownership: block rows are paired (w, NB-1-w), so wave w owns the lower tiles
// (w, 0..w) and (NB-1-w, 0..NB-1-w): NB+1 tiles, one scaled A operand per row and one
// B operand per block column per 4-TOA step shared by both rows (NB+2 LDS reads and 2
// multiplies per NB+1 MFMAs).  The wave index is made uniform (readfirstlane) so the
// ownership tests are scalar branches and the MFMAs issue back to back.
// BAL (NB = 2 SY_WAVES - 2, e.g. m + 1 = 217 -> NB = 14): the paired rows leave the last wave idle
// (NH = SY_WAVES - 1 waves with NB + 1 tiles each); instead the last wave takes the NB diagonal tiles
// and every pair wave keeps its NB - 1 off-diagonal ones -- at most 2 NB - 1 MFMAs per 4-TOA step on
// a SIMD (its two waves) instead of 2 NB + 2, and no idle SIMD slot.
#ifndef GS_SY_BAL
#define GS_SY_BAL 1
#endif
#ifndef GS_SY_GLDS
#define GS_SY_GLDS 1
#endif
typedef __attribute__((address_space(3))) void* gs_white_lds_vptr;
template <int NB>
__global__ __launch_bounds__(64 * SY_WAVES) void k_white_syrk(WhiteTntArgs A) {
  extern __shared__ double lds[];
  __shared__ double sb[3][GS_WHITE_MAX_BK + 1];
  constexpr bool BAL = GS_SY_BAL && NB == 2 * SY_WAVES - 2;
  constexpr int NH = (NB + 1) / 2;  // waves with paired rows
  constexpr int LDC = sy_ld(NB), WC = 16 * NB;
  const int64_t n_sys = (int64_t)A.n_psr * A.n_chain;
  // XCD-major: consecutive workgroup ids go round-robin over the 8 XCDs
  const int64_t per = (n_sys + 7) / 8;
  const int64_t sys = (int64_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
  if (sys >= n_sys) return;  // uniform over the workgroup
  const int p = (int)(sys / A.n_chain), c = (int)(sys % A.n_chain);
  const gs_tnt_desc D = A.tdesc[p];
  const gs_white_desc W = A.wdesc[p];
  stage_white(A, W, A.x_per_sys ? sys : (int64_t)c, sb[0], sb[1], sb[2]);
  const int m = (int)D.m;
  const int tid = threadIdx.x, l = tid & 63, i = l & 15, k = l >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r1 = w, r2 = NB - 1 - w;  // owned block rows (r1 <= r2 for w < NH)
  const bool act = w < NH;
  const bool two = act && r2 != r1;
  const int64_t n = D.n_toa;
  const double* Tp = A.T + D.T_off;
  const double* rp = A.r + D.toa_off;
  const double* s2 = A.sigma2 + D.toa_off;
  const int32_t* bk = A.bk + D.toa_off;
  double* buf0 = lds;
  double* buf1 = lds + SY_TC * LDC + SY_TC;  // [SY_TC x LDC] chunk + SY_TC inverse N

  // NB + 1 accumulator slots: tile (r2, j) in slot j (j <= r2), tile (r1, j) in slot
  // NB - j (j <= r1 < r2): disjoint, and both slot indices are static in the j loop
  gs_d4_t acc[NB + 1];
#pragma unroll
  for (int j = 0; j <= NB; ++j) acc[j] = gs_d4_t{0.0, 0.0, 0.0, 0.0};

  // chunk loader: thread tid owns column tid & 255 of rows (tid >> 8) + 2 e, e < 8
  const int lcol = tid & 255, lrow = tid >> 8;
  const bool colok = lcol < WC;
  double reg[GS_SY_GLDS ? 1 : SY_TC / 2];
  double rinv = 0.0;
  auto load = [&](int64_t t0) {
#pragma unroll
    for (int e = 0; e < (GS_SY_GLDS ? 0 : SY_TC / 2); ++e) {
      const int64_t t = t0 + lrow + 2 * e;
      double v = 0.0;
      if (colok && t < n) v = (lcol < m) ? Tp[t * m + lcol] : ((lcol == m) ? rp[t] : 0.0);
      reg[e] = v;
    }
    if (tid < SY_TC) {
      const int64_t t = t0 + tid;
      rinv = 0.0;
      if (t < n) {
        const int kb = bk[t];
        rinv = 1.0 / (sb[0][kb] * (s2[t] + sb[1][kb]) + sb[2][kb]);
      }
    }
  };
  auto store = [&](double* b) {
    if (colok)
#pragma unroll
      for (int e = 0; e < (GS_SY_GLDS ? 0 : SY_TC / 2); ++e) b[(lrow + 2 * e) * LDC + lcol] = reg[e];
    if (tid < SY_TC) b[SY_TC * LDC + tid] = rinv;
  };

  const int64_t nch = (n + SY_TC - 1) / SY_TC;
  // LDS-DMA staging (GS_SY_GLDS; rows of an even number of columns at a 16-byte aligned start): the T
  // rows of the next chunk go straight into LDS by global_load_lds_dwordx4 (one wave-instruction per
  // 128 columns of a row, lane-linear), so no 32-VGPR register copy of the chunk is live across the
  // MFMAs; the r column and 1/N come from 32 threads through registers.  Rows past n are never
  // loaded: the buffers start zeroed and those rows get 1/N = 0 and r = 0, so their stale (finite)
  // columns contribute nothing.
  // 16-byte units where every row starts 16-byte aligned (m and the pulsar's offset even), else 4-byte
  // ones (any m); compiled without the register path (GS_SY_GLDS: 193 VGPRs, none spilled, against 256
  // with 26 spilled when both are in the kernel)
  constexpr bool gl = GS_SY_GLDS;
  const bool w16 = (m % 2 == 0) && (D.T_off % 2 == 0);  // uniform
  double rr = 0.0;
  auto load_gl = [&](int64_t t0, double* b) {
    if (tid < SY_TC) {  // ordinary loads first, used at once: no DMA is in flight yet
      const int64_t t = t0 + tid;
      rinv = 0.0;
      rr = 0.0;
      if (t < n) {
        const int kb = bk[t];
        rinv = 1.0 / (sb[0][kb] * (s2[t] + sb[1][kb]) + sb[2][kb]);
        rr = rp[t];
      }
    }
#pragma unroll
    for (int e = 0; e < SY_TC / SY_WAVES; ++e) {
      const int row = w + SY_WAVES * e;
      const int64_t t = t0 + row;
      if (t >= n) continue;
      if (w16) {
        const int nu = m >> 1;  // 16-byte units per row, 64 per wave-instruction
        for (int base = 0; base < nu; base += 64)
          if (base + l < nu)
            __builtin_amdgcn_global_load_lds((const void*)(Tp + t * m + 2 * (base + l)),
                                             (gs_white_lds_vptr)(b + row * LDC + 2 * base), 16, 0, 0);
      } else {
        const int nu = 2 * m;   // 4-byte units
        const float* src = reinterpret_cast<const float*>(Tp + t * m);
        for (int base = 0; base < nu; base += 64)
          if (base + l < nu)
            __builtin_amdgcn_global_load_lds((const void*)(src + base + l),
                                             (gs_white_lds_vptr)(reinterpret_cast<float*>(b + row * LDC) + base), 4, 0,
                                             0);
      }
    }
  };
  auto store_gl = [&](double* b) {
    if (tid < SY_TC) {
      b[tid * LDC + m] = rr;
      b[SY_TC * LDC + tid] = rinv;
    }
  };
  if (gl) {
    for (int i = tid; i < 2 * (SY_TC * LDC + SY_TC); i += 64 * SY_WAVES) lds[i] = 0.0;
    __syncthreads();
    load_gl(0, buf0);
    store_gl(buf0);
  } else {
    load(0);
    store(buf0);
  }
  if (gl) gs_wait_dma();
  __syncthreads();
  // the chunk loop, instantiated once per role so each role's registers are allocated on their own
  // (role 1: the diagonal-tile wave of BAL; role 0: the paired-row waves).  Measured (r05e/r05f):
  // the diagonal wave in slots 0..NB-1 of the shared accumulator array 389-392 config5 sweeps/s,
  // with its own accumulator array 373 (= the unbalanced kernel's 372-374).
  auto stream = [&](auto role, auto dma) {
    for (int64_t ch = 0; ch < nch; ++ch) {
      const double* cur = (ch & 1) ? buf1 : buf0;
      double* nxt = (ch & 1) ? buf0 : buf1;
      if constexpr (decltype(dma)::value == 1) {
        if (ch + 1 < nch) load_gl((ch + 1) * SY_TC, nxt);  // nxt was last read before the previous barrier
      } else {
        if (ch + 1 < nch) load((ch + 1) * SY_TC);
      }
      // keep the next chunk's global loads here, ahead of the MFMAs: their latency is
      // hidden behind this chunk's math (the scheduler would otherwise sink them)
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (decltype(role)::value == 1) {
        // the diagonal tiles (j, j), j < NB: A = row j / N, B = row j; one 4-TOA step at a time
        // (an unrolled step loop hoists every step's products and spills)
#pragma unroll 1
        for (int kk = 0; kk < SY_TC / 4; ++kk) {
          const double* row = cur + (4 * kk + k) * LDC + i;
          const double iv = cur[SY_TC * LDC + 4 * kk + k];
#pragma unroll
          for (int j = 0; j < NB; ++j) {
            const double bj = row[16 * j];
            acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(bj * iv, bj, acc[j], 0, 0, 0);
          }
        }
      } else if (act) {
#pragma unroll
        for (int kk = 0; kk < SY_TC / 4; ++kk) {
          const double* row = cur + (4 * kk + k) * LDC + i;
          const double iv = cur[SY_TC * LDC + 4 * kk + k];
          const double a1 = row[16 * r1] * iv;
          const double a2 = row[16 * r2] * iv;
          double bv[NB];  // every B operand of the step in flight at once
#pragma unroll
          for (int j = 0; j < NB; ++j) bv[j] = row[16 * j];
#pragma unroll
          for (int j = 0; j < NB; ++j) {
            // BAL: the diagonal tiles belong to the last wave
            if (BAL ? j < r2 : j <= r2) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a2, bv[j], acc[j], 0, 0, 0);
            if (two && (BAL ? j < r1 : j <= r1))
              acc[NB - j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, bv[j], acc[NB - j], 0, 0, 0);
          }
        }
      }
      if constexpr (decltype(dma)::value == 1) {
        if (ch + 1 < nch) store_gl(nxt);
      } else {
        if (ch + 1 < nch) store(nxt);
      }
      if constexpr (decltype(dma)::value == 1) gs_wait_dma();  // nxt's DMA complete before the barrier
      __syncthreads();
    }
  };
  const bool diagw = BAL && w == SY_WAVES - 1;
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using IG = std::integral_constant<int, GS_SY_GLDS ? 1 : 0>;
  if (diagw)
    stream(I1{}, IG{});
  else
    stream(I0{}, IG{});
  if (!act && !diagw) return;

  double* out = A.TNT + D.tnt_off + (int64_t)c * A.tnt_cstride;
  double* dout = A.d + D.d_off + (int64_t)c * A.d_cstride;
  auto emit = [&](int bi, int bj, const gs_d4_t v4) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = bi * 16 + k + 4 * r, col = bj * 16 + i;
      const double v = v4[r];
      if (row < m && col < m) {
        out[(int64_t)row * m + col] = v;
        out[(int64_t)col * m + row] = v;
      } else if (row == m && col < m) {
        dout[col] = v;
      }
    }
  };
  if constexpr (BAL) {
    if (diagw) {
#pragma unroll
      for (int j = 0; j < NB; ++j) emit(j, j, acc[j]);
      return;
    }
  }
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    if (BAL ? j < r2 : j <= r2) emit(r2, j, acc[j]);
    if (two && (BAL ? j < r1 : j <= r1)) emit(r1, j, acc[NB - j]);
  }
}


// Small-m batched SYRK (r-augmented block count NB <= 6: one pulsar's m <= 95): the paired-row
// workgroup of k_white_syrk would leave 5 of its 8 waves idle, so instead 8 CHAINS of one
// pulsar share each LDS chunk of [T | r] (32 TOAs x 16 NB) -- T is common to all chains, only
// N differs -- and each wave accumulates its chain's NB (NB + 1) / 2 lower tiles with the
// chain's 1/N_t (staged per wave from its white parameters).  grid (ceil(C / 8), n_psr).
constexpr int MC_WAVES = 8, MC_CH = 32;
template <int NB>
__global__ __launch_bounds__(64 * MC_WAVES) void k_white_syrk_mc(WhiteTntArgs A) {
  extern __shared__ double lds[];
  __shared__ double wb[2][MC_WAVES][MC_CH];
  __shared__ double sp[MC_WAVES][3][GS_WHITE_MAX_BK + 1];
  constexpr int LDB = 16 * NB;
  constexpr int NT = NB * (NB + 1) / 2;
  constexpr int LPT = MC_CH * LDB / (64 * MC_WAVES);
  const int tid = threadIdx.x, l = tid & 63, i = l & 15, k = l >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int p = blockIdx.y;
  const int c = blockIdx.x * MC_WAVES + w;
  const bool live = c < A.n_chain;
  const gs_tnt_desc D = A.tdesc[p];
  const gs_white_desc* W = A.wdesc + p;
  const int m = (int)D.m;
  const int64_t n = D.n_toa;
  const int64_t sys = (int64_t)p * A.n_chain + (live ? c : 0);
  // per-wave (efac^2, t2equad^2, tnequad^2) of every backend of the chain
  if (l < W->n_bk) {
    sp[w][0][l] = 1.0;
    sp[w][1][l] = 0.0;
    sp[w][2][l] = 0.0;
  }
  wave_lds_sync();
  if (l < W->n_w && live) {
    const int64_t o = W->w_off + l;
    const int kb = A.wbk[o], kind = A.wkind[o];
    double e = 1.0, t = 0.0, q = 0.0;
    apply_white(kind, A.x[(A.x_per_sys ? sys : (int64_t)c) * A.ldx + A.wcol[o]], e, t, q);
    if (kind == GS_WHITE_EFAC) sp[w][0][kb] = e;
    else if (kind == GS_WHITE_TNEQUAD) sp[w][2][kb] = q;
    else sp[w][1][kb] = t;
  }
  __syncthreads();
  const double* Tp = A.T + D.T_off;
  const double* rp = A.r + D.toa_off;
  const double* s2 = A.sigma2 + D.toa_off;
  const int32_t* bk = A.bk + D.toa_off;

  gs_d4_t acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = gs_d4_t{0.0, 0.0, 0.0, 0.0};
  double reg[LPT];
  double wreg = 0.0;
  auto load = [&](int64_t t0) {
#pragma unroll
    for (int u = 0; u < LPT; ++u) {
      const int idx = tid + 64 * MC_WAVES * u;
      const int row = idx / LDB, col = idx % LDB;
      const int64_t t = t0 + row;
      double v = 0.0;
      if (t < n) v = (col < m) ? Tp[t * m + col] : ((col == m) ? rp[t] : 0.0);
      reg[u] = v;
    }
    wreg = 0.0;
    if (l < MC_CH && live) {
      const int64_t t = t0 + l;
      if (t < n) {
        const int kb = bk[t];
        wreg = 1.0 / (sp[w][0][kb] * (s2[t] + sp[w][1][kb]) + sp[w][2][kb]);
      }
    }
  };
  auto store = [&](int buf) {
    double* dst = lds + buf * (MC_CH * LDB);
#pragma unroll
    for (int u = 0; u < LPT; ++u) dst[tid + 64 * MC_WAVES * u] = reg[u];
    if (l < MC_CH) wb[buf][w][l] = wreg;
  };
  const int64_t nch = (n + MC_CH - 1) / MC_CH;
  load(0);
  store(0);
  __syncthreads();
  for (int64_t ch = 0; ch < nch; ++ch) {
    const int cb = (int)(ch & 1);
    if (ch + 1 < nch) load((ch + 1) * MC_CH);
    __builtin_amdgcn_sched_barrier(0);
    const double* cur = lds + cb * (MC_CH * LDB);
    const int nk = (int)min((int64_t)(MC_CH / 4), (n - ch * MC_CH + 3) / 4);
#pragma unroll
    for (int kk = 0; kk < MC_CH / 4; ++kk) {
      if (kk >= nk) break;
      const double* row = cur + (4 * kk + k) * LDB + i;
      const double wv = wb[cb][w][4 * kk + k];
      double v[NB];
#pragma unroll
      for (int r = 0; r < NB; ++r) v[r] = row[16 * r];
#pragma unroll
      for (int r = 0; r < NB; ++r) {
        const double av = v[r] * wv;
#pragma unroll
        for (int j = 0; j <= r; ++j)
          acc[r * (r + 1) / 2 + j] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, v[j], acc[r * (r + 1) / 2 + j], 0, 0, 0);
      }
    }
    if (ch + 1 < nch) store(cb ^ 1);
    __syncthreads();
  }
  if (!live) return;
  double* out = A.TNT + D.tnt_off + (int64_t)c * A.tnt_cstride;
  double* dout = A.d + D.d_off + (int64_t)c * A.d_cstride;
#pragma unroll
  for (int r = 0; r < NB; ++r)
#pragma unroll
    for (int j = 0; j <= r; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 16 * r + k + 4 * q, col = 16 * j + i;
        const double v = acc[r * (r + 1) / 2 + j][q];
        if (row < m && col <= row) {  // lower element only: exact symmetry
          out[(int64_t)row * m + col] = v;
          out[(int64_t)col * m + row] = v;
        } else if (row == m && col < m) {
          dout[col] = v;
        }
      }
}

// d_c = T^T (r / N_c): grid (n_sys, ceil(m_max / 64)).
__global__ __launch_bounds__(256) void k_white_tnr(WhiteTntArgs A) {
  __shared__ double red[4][64];
  __shared__ double sb[3][GS_WHITE_MAX_BK + 1];
  const int64_t sys = blockIdx.x;
  const int p = (int)(sys / A.n_chain), c = (int)(sys % A.n_chain);
  const gs_tnt_desc D = A.tdesc[p];
  const gs_white_desc W = A.wdesc[p];
  stage_white(A, W, A.x_per_sys ? sys : (int64_t)c, sb[0], sb[1], sb[2]);
  const int w = gs_wave_id(), l = threadIdx.x & 63;
  const int m = (int)D.m;
  const int j = blockIdx.y * 64 + l;
  double s = 0.0;
  if (j < m) {
    const double* Tp = A.T + D.T_off;
    const double* s2 = A.sigma2 + D.toa_off;
    const int32_t* bk = A.bk + D.toa_off;
    const double* r = A.r + D.toa_off;
    for (int64_t t = w; t < D.n_toa; t += 4) {
      const int kb = bk[t];
      const double N = sb[0][kb] * (s2[t] + sb[1][kb]) + sb[2][kb];
      s = fma(Tp[t * m + j], r[t] / N, s);
    }
  }
  red[w][l] = s;
  __syncthreads();
  if (w == 0 && j < m) A.d[D.d_off + (int64_t)c * A.d_cstride + j] = red[0][l] + red[1][l] + red[2][l] + red[3][l];
}


// ECORR operands with white noise sampled (gs_ecorr_epoch_sums): the epoch columns of T
// are quantisation indicators, so TNT[e, j] = sum over epoch e's TOAs of u_t T[t, j] / N_t
// -- a segmented sum of a few TOAs per epoch instead of the n_toa x m x m SYRK.  One
// workgroup per (16 epochs, ES_CH chains): the group's u_t / N_t are computed once per
// chain into LDS, then one thread per (epoch, reordered column) loads each T[t, j] ONCE
// for all ES_CH chains (T is shared; only the weights differ per chain); column dcol
// carries d_e = sum u_t r_t / N_t, j = 0 also Dg[e] = sum u_t^2 / N_t.
constexpr int ES_EPB = 16;    // epochs per workgroup
constexpr int ES_MAXQ = 256;  // TOA entries staged per workgroup (larger groups fall back)
constexpr int ES_CH = 8;      // chains per workgroup
__global__ __launch_bounds__(256) void k_ecorr_epoch_sums(EcorrSumArgs A) {
  __shared__ double sb[ES_CH][3][GS_WHITE_MAX_BK + 1];
  __shared__ double wq[ES_CH][ES_MAXQ];
  __shared__ int tq[ES_MAXQ];
  const int tid = threadIdx.x;
  const int c0 = blockIdx.y * ES_CH;
  const int nch = min(ES_CH, A.n_chain - c0);
  const gs_white_desc W = A.w.wdesc[0];
  // white parameters of the workgroup's chains (stage_white for ES_CH chains at once)
  for (int i = tid; i < ES_CH * W.n_bk; i += 256) {
    const int ci = i / W.n_bk, k = i % W.n_bk;
    sb[ci][0][k] = 1.0;
    sb[ci][1][k] = 0.0;
    sb[ci][2][k] = 0.0;
  }
  __syncthreads();
  for (int i = tid; i < nch * W.n_w; i += 256) {
    const int ci = i / W.n_w;
    const int64_t o = W.w_off + i % W.n_w;
    const int k = A.w.wbk[o], kind = A.w.wkind[o];
    double e = 1.0, t = 0.0, q = 0.0;
    apply_white(kind, A.w.x[(int64_t)(c0 + ci) * A.w.ldx + A.w.wcol[o]], e, t, q);
    if (kind == GS_WHITE_EFAC) sb[ci][0][k] = e;
    else if (kind == GS_WHITE_TNEQUAD) sb[ci][2][k] = q;
    else sb[ci][1][k] = t;
  }
  __syncthreads();
  const int e_lo = blockIdx.x * ES_EPB;
  const int e_hi = min(A.ne, e_lo + ES_EPB);
  const int q_lo = A.eptr[e_lo], q_hi = A.eptr[e_hi];
  const bool staged = q_hi - q_lo <= ES_MAXQ;
  // u_t / N_t of chain ci for TOA entry q
  auto weight = [&](int ci, int q, int t) {
    const int kb = A.w.bk[t];
    return A.eu[q] / (sb[ci][0][kb] * (A.w.sigma2[t] + sb[ci][1][kb]) + sb[ci][2][kb]);
  };
  if (staged) {
    for (int q = q_lo + tid; q < q_hi; q += 256) tq[q - q_lo] = A.etoa[q];
    __syncthreads();
    for (int i = tid; i < nch * (q_hi - q_lo); i += 256) {
      const int ci = i / (q_hi - q_lo), qq = i % (q_hi - q_lo);
      wq[ci][qq] = weight(ci, q_lo + qq, tq[qq]);
    }
  }
  __syncthreads();
  const int m = A.w.m_max;
  for (int idx = tid; idx < (e_hi - e_lo) * A.kb; idx += 256) {
    const int e = e_lo + idx / A.kb, j = idx % A.kb;
    const int cj = A.colmap[j];
    double acc[ES_CH], dg[ES_CH];
#pragma unroll
    for (int ci = 0; ci < ES_CH; ++ci) acc[ci] = dg[ci] = 0.0;
    for (int q = A.eptr[e]; q < A.eptr[e + 1]; ++q) {
      const int t = staged ? tq[q - q_lo] : A.etoa[q];
      const double v = (cj >= 0) ? A.w.T[(int64_t)t * m + cj] : ((j == A.dcol) ? A.w.r[t] : 0.0);
      const double u = A.eu[q];
#pragma unroll
      for (int ci = 0; ci < ES_CH; ++ci) {
        if (ci < nch) {
          const double wgt = staged ? wq[ci][q - q_lo] : weight(ci, q, t);
          acc[ci] = fma(v, wgt, acc[ci]);
          dg[ci] = fma(u, wgt, dg[ci]);
        }
      }
    }
#pragma unroll
    for (int ci = 0; ci < ES_CH; ++ci) {
      if (ci < nch) {
        A.Bx[((int64_t)(c0 + ci) * A.ne + e) * A.kb + j] = acc[ci];
        if (j == 0) A.Dg[(int64_t)(c0 + ci) * A.ne + e] = dg[ci];
      }
    }
  }
}

}  // namespace

int launch_ecorr_epoch_sums(hipStream_t s, const EcorrSumArgs& a) {
  hipLaunchKernelGGL(k_ecorr_epoch_sums,
                     dim3((unsigned)((a.ne + ES_EPB - 1) / ES_EPB), (unsigned)((a.n_chain + ES_CH - 1) / ES_CH)),
                     dim3(256), 0, s, a);
  return 0;
}

int launch_white_mh(hipStream_t s, const WhiteMhArgs& a) {
  dim3 grid((unsigned)((a.n_chain + MH_WPB - 1) / MH_WPB), (unsigned)a.n_psr);
  hipLaunchKernelGGL(k_white_mh, grid, dim3(64 * MH_WPB), 0, s, a);
  return 0;
}

int launch_white_resid(hipStream_t s, const WhiteResidArgs& a) {
  if (!getenv("GS_RESID_VALU")) {
    dim3 g((unsigned)((a.n_toa_max + 63) / 64), (unsigned)a.n_psr, (unsigned)((a.n_chain + 15) / 16));
    hipLaunchKernelGGL(k_white_resid_mfma, g, dim3(256), 0, s, a);
    return 0;
  }
  dim3 grid((unsigned)((a.n_toa_max + 255) / 256), (unsigned)a.n_psr,
            (unsigned)((a.n_chain + RES_CT - 1) / RES_CT));
  hipLaunchKernelGGL(k_white_resid, grid, dim3(256), 0, s, a);
  return 0;
}

template <int NB>
static void launch_syrk(hipStream_t s, const WhiteTntArgs& a, int64_t n_sys) {
  static bool attr = false;  // > 64 KB of dynamic LDS needs the opt-in (NB = 16)
  const size_t lds = (size_t)2 * (SY_TC * sy_ld(NB) + SY_TC) * sizeof(double);
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_white_syrk<NB>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL(k_white_syrk<NB>, dim3((unsigned)(((n_sys + 7) / 8) * 8)), dim3(64 * SY_WAVES), lds, s, a);
}

template <int NB>
static void launch_syrk_mc(hipStream_t s, const WhiteTntArgs& a) {
  static bool attr = false;
  const size_t lds = (size_t)2 * MC_CH * 16 * NB * sizeof(double);
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_white_syrk_mc<NB>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL(k_white_syrk_mc<NB>, dim3((unsigned)((a.n_chain + MC_WAVES - 1) / MC_WAVES), (unsigned)a.n_psr),
                     dim3(64 * MC_WAVES), lds, s, a);
}

int launch_white_tnt(hipStream_t s, const WhiteTntArgs& a) {
  const int nb = (a.m_max + 15) / 16;
  const int64_t n_sys = (int64_t)a.n_psr * a.n_chain;
  // one-pass batched SYRK for m + 1 <= 256 (block count of the r-augmented T)
  const int nba = (a.m_max + 1 + 15) / 16;
  if (nba <= 6 && !getenv("GS_SYRK_PAIRED")) {  // small m: chains share the T chunks
    switch (nba) {
      case 1: launch_syrk_mc<1>(s, a); break;
      case 2: launch_syrk_mc<2>(s, a); break;
      case 3: launch_syrk_mc<3>(s, a); break;
      case 4: launch_syrk_mc<4>(s, a); break;
      case 5: launch_syrk_mc<5>(s, a); break;
      default: launch_syrk_mc<6>(s, a); break;
    }
    return 0;
  }
  if (nba <= 16) {
    switch (nba) {
      case 1: launch_syrk<1>(s, a, n_sys); break;
      case 2: launch_syrk<2>(s, a, n_sys); break;
      case 3: launch_syrk<3>(s, a, n_sys); break;
      case 4: launch_syrk<4>(s, a, n_sys); break;
      case 5: launch_syrk<5>(s, a, n_sys); break;
      case 6: launch_syrk<6>(s, a, n_sys); break;
      case 7: launch_syrk<7>(s, a, n_sys); break;
      case 8: launch_syrk<8>(s, a, n_sys); break;
      case 9: launch_syrk<9>(s, a, n_sys); break;
      case 10: launch_syrk<10>(s, a, n_sys); break;
      case 11: launch_syrk<11>(s, a, n_sys); break;
      case 12: launch_syrk<12>(s, a, n_sys); break;
      case 13: launch_syrk<13>(s, a, n_sys); break;
      case 14: launch_syrk<14>(s, a, n_sys); break;
      case 15: launch_syrk<15>(s, a, n_sys); break;
      default: launch_syrk<16>(s, a, n_sys); break;
    }
    return 0;
  }
  hipLaunchKernelGGL(k_white_tnt, dim3((unsigned)n_sys, (unsigned)(nb * (nb + 1) / 2)), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_white_tnr, dim3((unsigned)n_sys, (unsigned)((a.m_max + 63) / 64)), dim3(256), 0, s, a);
  return 0;
}
