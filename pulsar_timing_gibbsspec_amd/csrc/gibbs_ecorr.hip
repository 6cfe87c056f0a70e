// Basis-ECORR block: the epoch columns of a basis-ECORR signal have a
// DIAGONAL block in TNT (every TOA belongs to at most one epoch), so Sigma = TNT +
// diag(phiinv) is reduced to the [timing model | free spectrum] columns R by eliminating
// the epochs first:
//     a_e = TNT_ee + 1/phi_e,  Sigma_R' = TNT_RR - B^T diag(1/a) B,  d_R' = d_R - B^T (d_E / a)
// (B = TNT[E, R]).  k_ecorr_schur forms Sigma_R', d_R' and the scalars of the
// marginalised likelihood for every chain's ECORR values; the existing prefix / lnlike /
// b-draw kernels then run on the R system, and k_ecorr_bdraw_e draws the epochs
// b_E | b_R ~ N((d_E - B b_R) / a, 1/a).  The Metropolis block is
// PulsarBlockGibbs.update_ecorr_params (pulsar_gibbs.py:409-486) on
// get_lnlikelihood_fullmarg (:569-610): k_ecorr_propose / k_ecorr_accept bracket one
// batched likelihood evaluation per step.
#include <algorithm>

#include "gibbs_internal.h"
#include "gibbs_tile.h"

namespace {

typedef double gs_d4_t __attribute__((ext_vector_type(4)));

// 4-chain workgroups (one wavefront per chain), at least 2 waves per SIMD (<= 256 VGPRs), 3 for
// k_ecorr_prefix with the shared chunks (<= 168 VGPRs: NB = 5 fits with 3 spilled): independent
// workgroups per CU whose epoch loops and epilogues overlap.  Measured (r05o, 4096 chains, NB = 5,
// likelihood mode): shared 0.1269 ms (8-wave workgroups, register-staged chunks) -> 0.1249 (8 waves,
// LDS-DMA chunks) -> 0.1238 (4 waves) -> 0.1200 (4 waves, 3 per SIMD); per-chain operands 0.169 ->
// 0.154 (8 waves, LDS-DMA double buffer) -> 0.146 (4 waves)
#ifndef GS_EC_WAVES
#define GS_EC_WAVES 4
#endif
constexpr int EC_WAVES = GS_EC_WAVES;  // chains per workgroup (one wavefront each)
#ifndef GS_EC_MINW
#define GS_EC_MINW 2
#endif
#ifndef GS_EC_MINW_SH
#define GS_EC_MINW_SH 3  // k_ecorr_prefix with the shared chunks
#endif
#ifndef GS_EC_MINW_INC
#define GS_EC_MINW_INC 2  // the incremental Metropolis step
#endif
constexpr int EC_CH = 32;    // epochs per LDS chunk
// per-chain operands (k_ecorr_prefix<.., PC = true>) staged by LDS-DMA, double-buffered 8-epoch
// chunks (1) or through registers, one 16-epoch chunk at a time (0)
#ifndef GS_EC_PCDMA
#define GS_EC_PCDMA 1
#endif
constexpr int EC_PCH = GS_EC_PCDMA ? 8 : 16;  // epochs per per-chain chunk
// LDS buffers per wave of the per-wave DMA path: chunk i + NBUF - 1 is issued while chunk i is
// multiplied (an 8-epoch chunk is only 2 k-steps = 30 MFMAs, ~1.9k cycles, against the L2 / HBM latency)
#ifndef GS_EC_NBUF
#define GS_EC_NBUF 2  // 3 measured no faster (r05z: the chunk latency is hidden at 2)
#endif
constexpr int EC_NBUF = GS_EC_NBUF;
static_assert(EC_NBUF >= 2 && EC_NBUF <= 4, "GS_EC_NBUF in 2..4");
// shared [B | d_E] chunks (one copy per workgroup) staged by LDS-DMA (1) or through registers (0)
#ifndef GS_EC_GLDS
#define GS_EC_GLDS 1
#endif
typedef __attribute__((address_space(3))) void* gs_ec_lds_vptr;
// s_waitcnt immediate waiting for vmcnt <= n only (gfx9 layout: vmcnt[3:0] + [15:14], expcnt[6:4],
// lgkmcnt[11:8] left at their maxima)
constexpr int ec_vmcnt(int n) { return (n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8); }
// LDS-DMA of ROWS rows of LDB doubles (row-major, stride LDB) starting at row e0 of src into the
// contiguous LDS block dst: wave-instructions k = wv, wv + nw, ... of the copy (lane-linear, 16-byte
// units when src is 16-byte aligned, else 4-byte units); rows at or past ne re-read row ne - 1, so
// every lane loads and the per-wave instruction count is fixed (finite data; callers weight those
// rows by 0).  Returns nothing to registers: the data is in LDS once vmcnt has drained.
template <int LDB, int ROWS>
__device__ __forceinline__ void ec_dma_rows(const double* src, int e0, int ne, double* dst, int wv, int nw, int l,
                                            bool w16) {
  if (w16) {
    constexpr int NI = ROWS * LDB / 128;
    for (int k = wv; k < NI; k += nw) {
      const int lin = 2 * (64 * k + l);
      const int e = min(e0 + lin / LDB, ne - 1);
      __builtin_amdgcn_global_load_lds((const void*)(src + (int64_t)e * LDB + lin % LDB), (gs_ec_lds_vptr)(dst + 128 * k),
                                       16, 0, 0);
    }
  } else {
    constexpr int NI = ROWS * LDB / 32;
    for (int k = wv; k < NI; k += nw) {
      const int lin = 64 * k + l;  // 4-byte unit of the block
      const int e = min(e0 + lin / (2 * LDB), ne - 1);
      __builtin_amdgcn_global_load_lds(
          (const void*)(reinterpret_cast<const float*>(src + (int64_t)e * LDB) + lin % (2 * LDB)),
          (gs_ec_lds_vptr)(reinterpret_cast<float*>(dst) + 64 * k), 4, 0, 0);
    }
  }
}

__device__ __forceinline__ double ec_wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// the wave sum as a wave-uniform value in an SGPR pair (readfirstlane): kept across the
// 256-VGPR epilogue of k_ecorr_prefix<5> without holding (or spilling) a VGPR pair
__device__ __forceinline__ double ec_wave_sum_u(double v) {
  v = ec_wave_sum(v);
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(u & 0xffffffffull));
  const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(u >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// 1/phi_k and log phi_k of backend k from log10_ecorr (phi = 10**(2 x), get_phiinv = 1/phi)
__device__ __forceinline__ void ec_phi(double x, double& inv, double& lg) {
  const double ph = pow(10.0, 2.0 * x);
  inv = 1.0 / ph;
  lg = gs_log_lnl(ph);
}

// Batched ECORR Schur complement, one wavefront per chain, EC_WAVES chains per
// workgroup sharing every LDS chunk of Bx = [B | d_E] (EC_CH epochs x 16 NB columns).
// Per 4-epoch step a lane loads NB values of its epoch row, scales them by the chain's
// 1/a_e and issues NB (NB + 1) / 2 v_mfma_f64_16x16x4f64 into the lower tiles of
// [B | d_E]^T diag(1/a) [B | d_E]: rows < mR give B^T W B, row mR gives B^T W d_E and
// (mR, mR) gives sum d_E^2 / a.  Roofline: fp64 MFMA, 2 ne (16 NB)^2 / 2 flop per chain,
// Bx read once per workgroup from L2.
// NP > 1 (NB >= 7, m_R > 96): the NT accumulator tiles (4 f64 registers each: 36 tiles at
// NB = 8 would need 288 VGPRs and spilled ~1.8k) are split over NP launches, launch PART
// keeping tiles t with t % NP == PART; each launch streams Bx again.
template <int NB, int NP = 1, int PART = 0>
__global__ __launch_bounds__(64 * EC_WAVES, GS_EC_MINW) void k_ecorr_schur(EcorrSchurArgs A) {
  extern __shared__ double lds[];
  __shared__ double wb[2][EC_WAVES][EC_CH];
  __shared__ double sinv[EC_WAVES][GS_WHITE_MAX_BK + 1], slog[EC_WAVES][GS_WHITE_MAX_BK + 1];
  constexpr int LDB = 16 * NB;
  constexpr int NT = NB * (NB + 1) / 2;
  const int tid = threadIdx.x, l = tid & 63, i = l & 15, k = l >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = blockIdx.x * EC_WAVES + w;
  const bool live = c < A.n_chain;
  const int ne = A.ne, mR = A.mR;
  if (l < A.n_bk) {
    double inv = 0.0, lg = 0.0;
    if (live) ec_phi(A.x[(int64_t)c * A.ldx + A.xcol[l]], inv, lg);
    sinv[w][l] = inv;
    slog[w][l] = lg;
  }
  __syncthreads();

  constexpr int NTP = (NT - PART + NP - 1) / NP;  // tiles of this part
  gs_d4_t acc[NTP];
#pragma unroll
  for (int t = 0; t < NTP; ++t) acc[t] = gs_d4_t{0.0, 0.0, 0.0, 0.0};
  double sla = 0.0, slp = 0.0;

  constexpr int LPT = EC_CH * LDB / (64 * EC_WAVES);  // chunk elements per thread
  double reg[GS_EC_GLDS ? 1 : LPT];
  int kreg = -1;
  double dreg = 0.0;
  const bool bx16 = (reinterpret_cast<uintptr_t>(A.Bx) & 15) == 0;  // uniform
  auto load = [&](int e0, int buf) {
    if constexpr (GS_EC_GLDS) {
      // straight into LDS buffer buf (its last reads ended at the previous barrier); waited by
      // the vmcnt(0) the weights' loads below take in store() and the barrier after it
      if (ne > 0) ec_dma_rows<LDB, EC_CH>(A.Bx, e0, ne, lds + buf * (EC_CH * LDB), w, EC_WAVES, l, bx16);
    } else {
#pragma unroll
      for (int q = 0; q < LPT; ++q) {
        const int idx = tid + 64 * EC_WAVES * q;
        const int e = e0 + idx / LDB;
        reg[q] = (e < ne) ? A.Bx[(int64_t)e0 * LDB + idx] : 0.0;
      }
    }
    kreg = -1;
    if (l < EC_CH && live && e0 + l < ne) {
      kreg = A.ebk[e0 + l];
      dreg = A.Dg[e0 + l];
    }
  };
  // the weights are formed here, after the chunk's MFMAs: using the loaded ebk / Dg inside load()
  // made the whole chunk prefetch wait (vmcnt(0)) before the MFMAs
  auto store = [&](int buf) {
    if constexpr (!GS_EC_GLDS) {
      double* dst = lds + buf * (EC_CH * LDB);
#pragma unroll
      for (int q = 0; q < LPT; ++q) dst[tid + 64 * EC_WAVES * q] = reg[q];
    }
    double wv = 0.0;
    if (kreg >= 0) {
      const double a = dreg + sinv[w][kreg];
      wv = 1.0 / a;
      sla += gs_log_lnl(a);
      slp += slog[w][kreg];
    }
    if (l < EC_CH) wb[buf][w][l] = wv;
  };

  const int nch = (ne + EC_CH - 1) / EC_CH;
  load(0, 0);
  store(0);
  if constexpr (GS_EC_GLDS) gs_wait_dma();
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    const int cb = ch & 1;
    if (ch + 1 < nch) load((ch + 1) * EC_CH, cb ^ 1);
    __builtin_amdgcn_sched_barrier(0);
    const double* cur = lds + cb * (EC_CH * LDB);
    const int nk = min(EC_CH / 4, (ne - ch * EC_CH + 3) / 4);  // k-steps holding epochs (uniform)
#pragma unroll
    for (int kk = 0; kk < EC_CH / 4; ++kk) {
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
        for (int j = 0; j <= r; ++j) {
          const int t = r * (r + 1) / 2 + j;
          if (t % NP == PART) acc[t / NP] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, v[j], acc[t / NP], 0, 0, 0);
        }
      }
    }
    if (ch + 1 < nch) store(cb ^ 1);
    if constexpr (GS_EC_GLDS) gs_wait_dma();  // the next chunk's DMA complete before the barrier
    __syncthreads();
  }
  sla = ec_wave_sum(sla);
  slp = ec_wave_sum(slp);
  if (!live) return;

  double* out = A.TNT + (int64_t)c * mR * mR;
  double* dout = A.d + (int64_t)c * mR;
#pragma unroll
  for (int r = 0; r < NB; ++r) {
#pragma unroll
    for (int j = 0; j <= r; ++j) {
      if ((r * (r + 1) / 2 + j) % NP != PART) continue;
      const gs_d4_t v4 = acc[(r * (r + 1) / 2 + j) / NP];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 16 * r + k + 4 * q, col = 16 * j + i;
        const double v = v4[q];
        if (row < mR && col <= row) {  // lower triangle only: exact symmetry
          const double s = A.A[(int64_t)row * mR + col] - v;
          out[(int64_t)row * mR + col] = s;
          out[(int64_t)col * mR + row] = s;
        } else if (row == mR && col < mR) {
          dout[col] = A.dR[col] - v;
        } else if (row == mR && col == mR) {
          A.aux[(int64_t)c * 4 + 1] = v;
        }
      }
    }
  }
  if (PART == 0 && l == 0) {
    A.aux[(int64_t)c * 4 + 0] = sla;
    A.aux[(int64_t)c * 4 + 2] = slp;
    A.aux[(int64_t)c * 4 + 3] = 0.0;
  }
}


// Fused ECORR Schur complement + fixed-prior prefix.  Bx / Ap columns are ordered
// [M (nM <= 16, padded to 16) | F (NF) | d | pad]: Ap = TNT of that ordering with phiinv_M on
// the M diagonal, d as row/column 16 + NF, (d, d) = 0 and 1 on every padded diagonal.
// Accumulated tiles are the UPPER ones, (j, r) for j <= r (block row M first), so the
// C layout of every off-diagonal tile is directly the B operand of a left product.
// Epilogue per wavefront, all in registers: T = Ap - P (the accumulators start at Ap); tile_elim (DPP column
// elimination, gibbs_tile.h) factors T_MM = U^T U -> V = U^-1 = L_M^-T; W_r = V^T T_0r,
// S_jr = T_jr - W_j^T W_r (4 MFMA each).
//   LNL = false: G_r = V W_r and S are written into the model block (gs_prefix layout) that
//                gs_lnlike_marg / gs_bdraw_sys read;
//   LNL = true:  the marginalised likelihood directly: phiinv_F is added to the S diagonal
//                and S (F block + the d row/column) is factored by an upper tile Cholesky
//                (tile_elim on the diagonal tiles, 4-MFMA TRSM and updates); after the last
//                F pivot the eliminated (d, d) entry is -(d^T Sigma^-1 d) of the whole
//                system (Ap_dd = 0), so no solve is needed and nothing per chain but lnl
//                goes to HBM.
// INC (likelihood mode, GS_EC_PCDMA): one Metropolis step from the chain's stored state instead of
// the full epoch SYRK.  A step moves ONE backend's ECORR parameter, so only that backend's epochs
// change weight: T(x') = T(x) - sum_{e in b} (1/a'_e - 1/a_e) [B | d_E]_e^T [B | d_E]_e, with T(x) =
// Ap - P(x) read from tbuf[tidx[c]] (lane layout of the accumulator tiles) and T(x') written to the
// other slot for k_ecorr_accept to adopt (tidx ^= 1) when the step is accepted.  Epochs are grouped by
// backend (eoff[k] .. eoff[k + 1]), so the loop covers one backend's rows: half the MFMAs with two
// backends.  Per-wave staging as the per-chain path (each chain's backend differs).
template <int NB, bool LNL, bool PC, bool INC = false>
__global__ __launch_bounds__(64 * EC_WAVES, INC ? GS_EC_MINW_INC : (PC ? GS_EC_MINW : GS_EC_MINW_SH)) void k_ecorr_prefix(
    EcorrPrefixArgs A) {
  static_assert(!INC || (LNL && GS_EC_PCDMA), "the incremental step is a likelihood-mode, LDS-DMA kernel");
  extern __shared__ double lds[];
  __shared__ double wb[2][EC_WAVES][EC_CH];
  __shared__ double sinv[EC_WAVES][GS_WHITE_MAX_BK + 1], slog[EC_WAVES][GS_WHITE_MAX_BK + 1];
  __shared__ double Ls[EC_WAVES][16 * 17];
  constexpr int LDB = 16 * NB;
  constexpr int NF = 20 * (NB - 2);  // 20, 40, 60 <-> NB = 3, 4, 5
  constexpr int NTF = NB - 1;        // tile rows of the F + d block
  constexpr int NT = 1 + 2 * NTF + NTF * (NTF - 1) / 2;
  const int tid = threadIdx.x, l = tid & 63, c = l & 15, q = l >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ch_id = blockIdx.x * EC_WAVES + w;
  const bool live = ch_id < A.n_chain;
  const int ne = A.ne, nM = A.nM;
  if (l < A.n_bk) {
    double inv = 0.0, lg = 0.0;
    if (live) ec_phi(A.x[(int64_t)ch_id * A.ldx + A.xcol[l]], inv, lg);
    sinv[w][l] = inv;
    slog[w][l] = lg;
  }
  __syncthreads();

  // tile slots: 0 = (0,0); r = (0,r) for r = 1..NTF; (j,r), 1 <= j <= r: NB + tix(j-1, r-1)
  auto ts = [](int j, int r) { return NB + gtile::tix(j - 1, r - 1, NTF); };
  // The accumulators start at Ap and the MFMAs subtract (weights negated): T = Ap - P comes
  // out of the epoch loop with no epilogue loads (loaded after the loop, the 60 Ap doubles sat
  // beside the 60 accumulated ones and spilled).
  const double* Apc = A.Ap + (int64_t)(live ? ch_id : 0) * A.ap_cs;
  auto Aq = [&](int r0, int c0, int s) { return Apc[(int64_t)(r0 + 4 * s + q) * LDB + c0 + c]; };
  gs_d4_t acc[NT];
  // (GS_EC_PROBE_INC_NOLOAD / _NOSTORE: cost-attribution builds only, wrong results)
#ifdef GS_EC_PROBE_INC_NOLOAD
  if constexpr (false) {
#else
  if constexpr (INC) {
#endif
    const int tc = live ? A.tidx[ch_id] : 0;
    const double* tb = A.tbuf + ((int64_t)tc * A.n_chain + (live ? ch_id : 0)) * (NT * 256);
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int s = 0; s < 4; ++s) acc[t][s] = live ? tb[(4 * t + s) * 64 + l] : 0.0;
  } else {
#pragma unroll
    for (int s = 0; s < 4; ++s) acc[0][s] = live ? Aq(0, 0, s) : 0.0;
#pragma unroll
    for (int r = 1; r < NB; ++r)
#pragma unroll
      for (int s = 0; s < 4; ++s) acc[r][s] = live ? Aq(0, 16 * r, s) : 0.0;
#pragma unroll
    for (int jj = 1; jj < NB; ++jj)
#pragma unroll
      for (int r = jj; r < NB; ++r)
#pragma unroll
        for (int s = 0; s < 4; ++s) acc[ts(jj, r)][s] = live ? Aq(16 * jj, 16 * r, s) : 0.0;
  }
  double sla = 0.0, slp = 0.0;
  constexpr int LPT = EC_CH * LDB / (64 * EC_WAVES);  // chunk elements per thread
  double reg[GS_EC_GLDS ? 1 : LPT];
  int kreg = -1;
  double dreg = 0.0;
  const bool bx16 = (reinterpret_cast<uintptr_t>(A.Bx) & 15) == 0;  // uniform
  auto load = [&](int e0, int buf) {
    if constexpr (GS_EC_GLDS) {
      // straight into LDS buffer buf (its last reads ended at the previous barrier); waited by
      // the vmcnt(0) the weights' loads below take in store() and the barrier after it
      if (ne > 0) ec_dma_rows<LDB, EC_CH>(A.Bx, e0, ne, lds + buf * (EC_CH * LDB), w, EC_WAVES, l, bx16);
    } else {
#pragma unroll
      for (int u = 0; u < LPT; ++u) {
        const int idx = tid + 64 * EC_WAVES * u;
        const int e = e0 + idx / LDB;
        reg[u] = (e < ne) ? A.Bx[(int64_t)e0 * LDB + idx] : 0.0;
      }
    }
    kreg = -1;
    if (l < EC_CH && live && e0 + l < ne) {
      kreg = A.ebk[e0 + l];
      dreg = A.Dg[e0 + l];
    }
  };
  // the weights are formed here, after the chunk's MFMAs: using the loaded ebk / Dg inside load()
  // made the whole chunk prefetch wait (vmcnt(0)) before the MFMAs
  auto store = [&](int buf) {
    if constexpr (!GS_EC_GLDS) {
      double* dst = lds + buf * (EC_CH * LDB);
#pragma unroll
      for (int u = 0; u < LPT; ++u) dst[tid + 64 * EC_WAVES * u] = reg[u];
    }
    double wv = 0.0;
    if (kreg >= 0) {
      const double a = dreg + sinv[w][kreg];
      wv = 1.0 / a;
      sla += gs_log_lnl(a);
      slp += slog[w][kreg];
    }
    if (l < EC_CH) wb[buf][w][l] = wv;
  };
  if constexpr (PC || INC) {
    // per-chain [B | d_E] (white noise sampled: TNT differs per chain): no sharing across
    // waves; each wavefront stages chunks of its own rows in its slice of the dynamic LDS
    if (!live) return;  // no workgroup barriers below
    const double* Bc = A.Bx + (int64_t)ch_id * A.bx_cs;
    const double* Dc = A.Dg + (int64_t)ch_id * A.dg_cs;
    constexpr int PCH = EC_PCH;
    auto kstep = [&](const double* buf, const double* wrow, int kk) {
      const double* row = buf + (4 * kk + q) * LDB + c;
      const double wk = -wrow[4 * kk + q];
      double v[NB];
#pragma unroll
      for (int r = 0; r < NB; ++r) v[r] = row[16 * r];
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const double av = v[j] * wk;
#pragma unroll
        for (int r = j; r < NB; ++r) {
          const int t = (j == 0) ? r : ts(j, r);
          acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, v[r], acc[t], 0, 0, 0);
        }
      }
    };
    if constexpr (GS_EC_PCDMA) {
      // LDS-DMA: the rows of chunk i + NBUF - 1 go global -> LDS (lane-linear, NB wave-instructions
      // of 16-byte units, or 4 NB of 4-byte units when the chain's rows are not 16-byte aligned)
      // while chunk i is multiplied; a chunk's rows past the range end e_hi re-read row e_hi - 1, so
      // every chunk issues the same instruction count (the vmcnt waits below count them) and those
      // rows have weight 0.  The weights of a 64-epoch segment are computed by its lanes at the
      // segment's first chunk (the only ordinary loads of the loop; their wait also covers the DMA).
      constexpr int CHD = PCH * LDB;
      double* bufs = lds + (int64_t)w * (EC_NBUF * CHD + 64);
      double* wsl = bufs + EC_NBUF * CHD;
      const bool w16 = (reinterpret_cast<uintptr_t>(Bc) & 15) == 0;  // uniform
      // epoch range [e_lo, e_hi): all epochs, or (INC) the moved backend's
      int e_lo = 0, e_hi = ne;
      double s_new = 0.0, s_old = 0.0;  // INC: 1/phi of the moved backend at the proposal / the state
      if constexpr (INC) {
        const int col = (int)A.prop[(int64_t)ch_id * 4];
        const unsigned long long mk = __ballot(l < A.n_bk && A.xcol[l < A.n_bk ? l : 0] == col);
        const int k = mk ? (int)__builtin_ctzll(mk) : -1;
        if (k >= 0) {
          e_lo = __builtin_amdgcn_readfirstlane(A.eoff[k]);
          e_hi = __builtin_amdgcn_readfirstlane(A.eoff[k + 1]);
          s_new = sinv[w][k];
          double lg;
          ec_phi(A.xold[(int64_t)ch_id * A.ldx + col], s_old, lg);
        } else {
          e_hi = 0;  // nothing moved: T(x') = T(x)
        }
        // sum log a and sum log phi_E over every epoch at the proposal
        for (int e = l; e < ne; e += 64) {
          const int kb = A.ebk[e];
          sla += gs_log_lnl(Dc[e] + sinv[w][kb]);
          slp += slog[w][kb];
        }
      }
      auto dma = [&](int e0, double* dst) { ec_dma_rows<LDB, PCH>(Bc, e0, e_hi, dst, 0, 1, l, w16); };
      constexpr int WAIT0 = ec_vmcnt(0);
      const int nch = (e_hi - e_lo + PCH - 1) / PCH;
      // the accumulators' Ap loads land here: otherwise the loop's first MFMA waits vmcnt(0) (the
      // waitcnt pass merges the loop entry into every iteration) and no DMA overlaps the math
      __builtin_amdgcn_s_waitcnt(WAIT0);
      // chunks 0 .. NBUF - 2 in flight before the loop (no rows: nothing to read)
#pragma unroll
      for (int j = 0; j < EC_NBUF - 1; ++j)
        if (j < nch) dma(e_lo + j * PCH, bufs + j * CHD);
      // s_waitcnt immediates: chunk i has landed once at most n chunks issued after it are pending
      auto wait_chunks = [&](int n) {  // n uniform, 0 .. NBUF - 2
        if (w16) {
          if (n >= 2) __builtin_amdgcn_s_waitcnt(ec_vmcnt(2 * NB));
          else if (n == 1) __builtin_amdgcn_s_waitcnt(ec_vmcnt(NB));
          else __builtin_amdgcn_s_waitcnt(WAIT0);
        } else {
          if (n >= 2) __builtin_amdgcn_s_waitcnt(ec_vmcnt(8 * NB));
          else if (n == 1) __builtin_amdgcn_s_waitcnt(ec_vmcnt(4 * NB));
          else __builtin_amdgcn_s_waitcnt(WAIT0);
        }
      };
      for (int i = 0; i < nch; ++i) {
        const int e0 = e_lo + i * PCH, er = i * PCH;
        if ((er & 63) == 0) {
          double wv = 0.0;
          if (e0 + l < e_hi) {
            const int e = e0 + l;
            if constexpr (INC) {
              const double dg = Dc[e];
              wv = 1.0 / (dg + s_new) - 1.0 / (dg + s_old);
            } else {
              const int kb = A.ebk[e];
              const double a = Dc[e] + sinv[w][kb];
              wv = 1.0 / a;
              sla += gs_log_lnl(a);
              slp += slog[w][kb];
            }
          }
          wsl[l] = wv;
        }
        __builtin_amdgcn_sched_barrier(0);
        const int ia = i + EC_NBUF - 1;  // the chunk issued now (its buffer's reads ended with chunk i - 1)
        if (ia < nch) dma(e0 + (EC_NBUF - 1) * PCH, bufs + (ia % EC_NBUF) * CHD);
        wait_chunks(min(EC_NBUF - 1, nch - 1 - i));
        __builtin_amdgcn_sched_barrier(0);
        wave_lds_sync();
        const double* cur = bufs + (i % EC_NBUF) * CHD;
        const int nk = min(PCH / 4, (e_hi - e0 + 3) / 4);
#pragma unroll
        for (int kk = 0; kk < PCH / 4; ++kk) {
          if (kk >= nk) break;
          kstep(cur, wsl + (er & 63), kk);
        }
      }
    } else {
      // register-staged: all of a chunk's loads in flight at once, 1/a by lanes 0..PCH-1
      constexpr int PL = PCH * LDB / 64;  // doubles per lane per chunk
      double* buf = lds + (int64_t)w * (PCH * LDB + PCH);
      double* wsl = buf + PCH * LDB;
      for (int e0 = 0; e0 < ne; e0 += PCH) {
        double rg[PL];
#pragma unroll
        for (int u = 0; u < PL; ++u) {
          const int idx = l + 64 * u;
          rg[u] = (e0 + idx / LDB < ne) ? Bc[(int64_t)e0 * LDB + idx] : 0.0;
        }
        double wv = 0.0;
        if (l < PCH && e0 + l < ne) {
          const int e = e0 + l;
          const int kb = A.ebk[e];
          const double a = Dc[e] + sinv[w][kb];
          wv = 1.0 / a;
          sla += gs_log_lnl(a);
          slp += slog[w][kb];
        }
        wave_lds_sync();  // previous chunk's LDS reads are done before the overwrite
#pragma unroll
        for (int u = 0; u < PL; ++u) buf[l + 64 * u] = rg[u];
        if (l < PCH) wsl[l] = wv;
        wave_lds_sync();
        const int nk = min(PCH / 4, (ne - e0 + 3) / 4);
#pragma unroll
        for (int kk = 0; kk < PCH / 4; ++kk) {
          if (kk >= nk) break;
          kstep(buf, wsl, kk);
        }
      }
    }
  } else {
  const int nch = (ne + EC_CH - 1) / EC_CH;
  load(0, 0);
  store(0);
  if constexpr (GS_EC_GLDS) gs_wait_dma();
  __syncthreads();
  for (int chk = 0; chk < nch; ++chk) {
    const int cb = chk & 1;
    if (chk + 1 < nch) load((chk + 1) * EC_CH, cb ^ 1);
    __builtin_amdgcn_sched_barrier(0);
    const double* cur = lds + cb * (EC_CH * LDB);
    const int nk = min(EC_CH / 4, (ne - chk * EC_CH + 3) / 4);  // k-steps holding epochs (uniform)
#pragma unroll
    for (int kk = 0; kk < EC_CH / 4; ++kk) {
      if (kk >= nk) break;
      const double* row = cur + (4 * kk + q) * LDB + c;
      const double wv = -wb[cb][w][4 * kk + q];
      double v[NB];
#pragma unroll
      for (int r = 0; r < NB; ++r) v[r] = row[16 * r];
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const double av = v[j] * wv;
#pragma unroll
        for (int r = j; r < NB; ++r) {
          const int t = (j == 0) ? r : ts(j, r);
          acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, v[r], acc[t], 0, 0, 0);
        }
      }
    }
    if (chk + 1 < nch) store(cb ^ 1);
    if constexpr (GS_EC_GLDS) gs_wait_dma();  // the next chunk's DMA complete before the barrier
    __syncthreads();
  }
  }
#ifdef GS_EC_PROBE_INC_NOSTORE
  if (A.tbuf && live && !INC) {
#else
  if (A.tbuf && live) {
#endif
    // T = Ap - P of this evaluation into the chain's state slot (INC: the proposal's slot)
    const int tc = A.tidx[ch_id] ^ (INC ? 1 : 0);
    double* tb = A.tbuf + ((int64_t)tc * A.n_chain + ch_id) * (NT * 256);
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int s = 0; s < 4; ++s) tb[(4 * t + s) * 64 + l] = acc[t][s];
  }
  sla = ec_wave_sum_u(sla);
  slp = ec_wave_sum_u(slp);
  if (!live) return;  // no workgroup barriers below

  constexpr int LD_D = NF % 16;            // d's position in the last F tile
  double pdd = 0.0;                        // sum d_E^2 / a = P_dd = -T_dd (Ap_dd = 0)
#pragma unroll
  for (int s = 0; s < 4; ++s)
    if (c == LD_D && 4 * s + q == LD_D) pdd = -acc[ts(NTF, NTF)][s];
  pdd = ec_wave_sum_u(pdd);
  // T_MM = U^T U: V = U^-1 = L_M^-T (upper), L_M^-1 = V^T
  gs_d4_t V, Ecol = acc[0];
  double rsd;
  tile_elim<16>(Ecol, V, rsd, q, c);
#pragma unroll
  for (int s = 0; s < 4; ++s) V[s] *= rsd;
  int fail = 0;
  {
    const bool bad = (q == 0) && (c < nM) && !(rsd > 0.0 && rsd < INFINITY);
    const unsigned long long m = __ballot(bad);
    if (m) fail = __builtin_ctzll(m) + 1;
  }
  double ldl = (q == 0 && c < nM) ? -gs_log_lnl(rsd) : 0.0;  // sum log diag L_M
  ldl = ec_wave_sum_u(ldl);

  // W_r = L_M^-1 T_0r = V^T T_0r;  S_jr = T_jr - W_j^T W_r
  gs_d4_t W[NB];
#pragma unroll
  for (int r = 1; r < NB; ++r) W[r] = gtile::mfma_tn(gs_d4_t{0.0, 0.0, 0.0, 0.0}, V, acc[r]);
#pragma unroll
  for (int j = 1; j < NB; ++j)
#pragma unroll
    for (int r = j; r < NB; ++r) {
      const int t = ts(j, r);
#pragma unroll
      for (int s = 0; s < 4; ++s) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(-W[j][s], W[r][s], acc[t], 0, 0, 0);
    }

  if constexpr (LNL) {
    // + phiinv_F on the diagonal, then the upper tile Cholesky of the F block
    const double* ph = A.phiinv_F + (int64_t)ch_id * NF;
#pragma unroll
    for (int K = 1; K < NB; ++K)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int i = 16 * (K - 1) + c;
        if (4 * s + q == c && i < NF) acc[ts(K, K)][s] += ph[i];
      }
    double ldS = 0.0, quad = 0.0;
#pragma unroll
    for (int K = 1; K < NB; ++K) {
      gs_d4_t Vk, Ak = acc[ts(K, K)];
      double rk;
      if (K < NTF) {
        tile_elim<16>(Ak, Vk, rk, q, c);
      } else {
        // KMAX = LD_D + 1: tile_elim applies a step's column operation only when a later
        // row remains, so the d row must be in range for the last F pivot to reach it
        tile_elim<LD_D + 1>(Ak, Vk, rk, q, c);
        // column-eliminated (d, d) entry = -(d^T Sigma^-1 d) of the whole system
#pragma unroll
        for (int s = 0; s < 4; ++s)
          if (c == LD_D && 4 * s + q == LD_D) quad = -Ak[s];
      }
      const int lim = (K < NTF) ? 16 : LD_D;
      const bool badk = (q == 0) && (c < lim) && !(rk > 0.0 && rk < INFINITY);
      const unsigned long long mk = __ballot(badk);
      if (mk && fail == 0) fail = 16 * K + __builtin_ctzll(mk) + 1;
      ldS += (q == 0 && c < lim) ? -2.0 * gs_log_lnl(rk) : 0.0;
#pragma unroll
      for (int s = 0; s < 4; ++s) Vk[s] *= rk;
      // U_KJ = V_K^T T_KJ (J > K), then T_IJ -= U_KI^T U_KJ (K < I <= J)
#pragma unroll
      for (int J = K + 1; J < NB; ++J) acc[ts(K, J)] = gtile::mfma_tn(gs_d4_t{0.0, 0.0, 0.0, 0.0}, Vk, acc[ts(K, J)]);
#pragma unroll
      for (int I = K + 1; I < NB; ++I)
#pragma unroll
        for (int J = I; J < NB; ++J)
#pragma unroll
          for (int s = 0; s < 4; ++s)
            acc[ts(I, J)] = __builtin_amdgcn_mfma_f64_16x16x4f64(-acc[ts(K, I)][s], acc[ts(K, J)][s], acc[ts(I, J)], 0, 0, 0);
    }
    ldS = ec_wave_sum_u(ldS);
    quad = ec_wave_sum_u(quad);
    double lph = (l < NF) ? gs_log_lnl(ph[l]) : 0.0;
    lph = ec_wave_sum_u(lph);
    if (l == 0) {
      // in gs_ecorr_accept's convention: lnl + (aux1 - aux0 - aux2) / 2, with aux1 = 0 here
      A.lnl[ch_id] = 0.5 * (quad - 2.0 * ldl - ldS + lph);
      double* ax = A.aux + (int64_t)ch_id * 4;
      ax[0] = sla;
      ax[1] = 0.0;
      ax[2] = slp;
      ax[3] = pdd;
      if (A.info) A.info[ch_id] = fail;
    }
    return;
  } else {
    const gs_d4_t Vt = gtile::transpose(V, Ls[w], q, c);  // C layout of V^T
    const int NMX = A.NMX, ldw = NF + 1;
    double* mb = A.model + (int64_t)ch_id * A.mstride;
    double* S0 = mb;
    double* dF = S0 + (int64_t)NF * ldw;
    double* Gm = dF + NF;
    double* hm = Gm + (int64_t)NMX * ldw;
    double* Rm = hm + NMX;
    double* am = Rm + (int64_t)NMX * NMX;
    double e2 = 0.0;  // |L_M^-1 d_M|^2: column d of W
#pragma unroll
    for (int r = 1; r < NB; ++r) {
      if (r == NTF && c == LD_D)
#pragma unroll
        for (int s = 0; s < 4; ++s) e2 += W[r][s] * W[r][s];
      // G_r = L_M^-T W_r = V W_r = (V^T)^T W_r
      const gs_d4_t G = gtile::mfma_tn(gs_d4_t{0.0, 0.0, 0.0, 0.0}, Vt, W[r]);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int mr = 4 * s + q, col = 16 * (r - 1) + c;
        if (mr < nM && col <= NF) {  // G's column NF is zero padding (k_prefix layout); h = L^-T e
          Gm[(int64_t)mr * ldw + col] = (col < NF) ? G[s] : 0.0;
          if (col == NF) hm[mr] = G[s];
        }
      }
    }
    e2 = ec_wave_sum_u(e2);
    // S0 (rows < NF, cols <= NF, column NF = dF) from the upper tiles
#pragma unroll
    for (int j = 1; j < NB; ++j)
#pragma unroll
      for (int r = j; r < NB; ++r) {
        const int t = ts(j, r);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int row = 16 * (j - 1) + 4 * s + q, col = 16 * (r - 1) + c;
          if (row > col) continue;
          const double v = acc[t][s];
          if (row < NF && col <= NF) S0[(int64_t)row * ldw + col] = v;
          if (col < NF && row != col) S0[(int64_t)col * ldw + row] = v;
          if (col == NF && row < NF) dF[row] = v;
        }
      }
    // R = L_M^-T = V (upper), zero beyond nM
    for (int idx = l; idx < NMX * NMX; idx += 64) Rm[idx] = 0.0;
    gtile::lds_fence();
#pragma unroll
    for (int s = 0; s < 4; ++s)
      if (4 * s + q < nM && c < nM) Rm[(4 * s + q) * NMX + c] = V[s];
    for (int64_t qq = (am - mb) + 2 + l; qq < A.mstride; qq += 64) mb[qq] = 0.0;
    if (l == 0) {
      am[0] = ldl;
      am[1] = e2;
      double* ax = A.aux + (int64_t)ch_id * 4;
      ax[0] = sla;
      ax[1] = pdd;
      ax[2] = slp;
      ax[3] = 0.0;
      if (A.info) A.info[ch_id] = fail;
    }
  }
}

// One Metropolis proposal per chain (pulsar_gibbs.py:458-462): scale, one ECORR parameter
// uniformly, q[par] += randn * (0.05 n_e) * scale.  xq = x with the jump applied;
// prop[c] = {x column, log U, inside prior, proposed value}.  Only the ECORR columns of xq
// are written (the rest of the row is never read).
__device__ __forceinline__ void ecorr_propose_one(const EcorrMhArgs& A, int c, int step) {
  double sc, z, u;
  int p;
  if (A.inj) {
    const double* q = A.inj + ((int64_t)step * A.n_chain + c) * 4;
    sc = q[0];
    p = (int)q[1];
    z = q[2];
    u = q[3];
  } else {
    const long long sw = gs_sweep(A.sweep, A.sweep_dev), gc = A.chain_base + c;
    const uint32_t s3 = 3u * (uint32_t)step;
    double u1, u2, v1, v2, u4;
    gs_uniform2(gs_counter(s3, sw, gc, 0, GS_EV_ECORR), A.key, u1, u2);
    gs_uniform2(gs_counter(s3 + 1, sw, gc, 0, GS_EV_ECORR), A.key, v1, v2);
    gs_uniform2(gs_counter(s3 + 2, sw, gc, 0, GS_EV_ECORR), A.key, u, u4);
    sc = gs_mh_scale(u1);
    p = min((int)(u2 * A.n_e), A.n_e - 1);
    z = sqrt(-2.0 * log(1.0 - v1)) * cospi(2.0 * v2);
  }
  const double* xr = A.x + (int64_t)c * A.ldx;
  double* qr = A.xq + (int64_t)c * A.ldx;
  // the likelihood kernels read only the ECORR columns of xq
  for (int j = 0; j < A.n_e; ++j) qr[A.ecol[j]] = xr[A.ecol[j]];
  const int col = A.ecol[p];
  const double qv = gs_add_rn(xr[col], gs_mul_rn(gs_mul_rn(z, 0.05 * A.n_e), sc));  // numpy's rounding (no fma)
  qr[col] = qv;
  double* pr = A.prop + (int64_t)c * 4;
  pr[0] = (double)col;
  pr[1] = log(u);
  pr[2] = (qv >= A.emin[p] && qv <= A.emax[p]) ? 1.0 : 0.0;  // Uniform prior (:613-617)
  pr[3] = qv;
}

__global__ __launch_bounds__(256) void k_ecorr_propose(EcorrMhArgs A) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= A.n_chain) return;
  ecorr_propose_one(A, c, A.step);
}

// Metropolis decision (pulsar_gibbs.py:465-472), optionally followed by the next proposal: lnL = lnl_R + (sum d_E^2/a - sum log a -
// sum log phi_E) / 2 (the chain-independent constants cancel); -inf when a factor was not
// positive definite or the proposal left the prior.  init: only record lnL0 at x.
__global__ __launch_bounds__(256) void k_ecorr_accept(EcorrMhArgs A) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= A.n_chain) return;
  const double* ax = A.aux + (int64_t)c * 4;
  const bool pd = !(A.info && A.info[c]) && !(A.pinfo && A.pinfo[c]);
  const double l1 = pd ? A.lnl[c] + 0.5 * (ax[1] - ax[0] - ax[2]) : -INFINITY;
  if (A.init) {
    A.lnl0[c] = l1;
  } else {
    const double* pr = A.prop + (int64_t)c * 4;
    const double diff = (pr[2] != 0.0) ? l1 - A.lnl0[c] : -INFINITY;
    if (A.q_rec)
      for (int j = 0; j < A.n_e; ++j) A.q_rec[(int64_t)c * A.n_e + j] = A.xq[(int64_t)c * A.ldx + A.ecol[j]];
    if (diff > pr[1]) {
      A.x[(int64_t)c * A.ldx + (int)pr[0]] = pr[3];
      A.lnl0[c] = l1;
      if (A.n_acc) A.n_acc[c] += 1;
      if (A.tidx) A.tidx[c] ^= 1;  // the proposal's stored T becomes the chain's state
    }
  }
  // gs_ecorr_accept_propose: the next step's proposal from the updated state, same thread
  // (one launch per Metropolis step instead of two)
  if (A.next_step >= 0) ecorr_propose_one(A, c, A.next_step);
}

// b_E | b_R and the scatter of b_R into b's original column order.  Grid (EB_BLK(ne) +
// ceil(mR / 256), n_chain): the first EB_BLK workgroups hold 64 epochs each, FOUR lanes per
// epoch splitting the Bx row's columns t = sub, sub + 4, ... (each load instruction touches
// 16 rows x 32 contiguous bytes instead of 64 rows x 8 bytes with a lane per epoch; the
// per-chain Bx of the white + ECORR path streams from HBM), partial sums combined over the
// quad; the remaining workgroups scatter b_R (one thread per column).
constexpr int EB_EPB = 64;    // epochs per workgroup (4 lanes each)
constexpr int EB_MAXC = 128;  // Bx columns (16 NB, NB <= 6 -> 96)
__host__ __device__ constexpr int eb_blk(int ne) { return (ne + EB_EPB - 1) / EB_EPB; }

// CH chains per workgroup: with a shared Bx (bx_cs = 0) every Bx row load serves CH chains'
// b_R (CH = 8); per-chain Bx uses CH = 1.
template <int CH>
__global__ __launch_bounds__(256) void k_ecorr_bdraw_e(EcorrBArgs A) {
  const int c0 = blockIdx.y * CH;
  const int nch = min(CH, A.n_chain - c0);
  const int neb = eb_blk(A.ne);
  if ((int)blockIdx.x >= neb) {
    const int j = ((int)blockIdx.x - neb) * 256 + threadIdx.x;
    for (int ci = 0; ci < nch; ++ci) {
      const int c = c0 + ci;
      if (A.chain_mask && !A.chain_mask[c]) continue;  // gate (pulsar_gibbs.py:697-698)
      if (j < A.mR) A.b[(int64_t)c * A.ldb + A.rcol[j]] = A.bR[(int64_t)c * A.ldbR + j];
    }
    return;
  }
  // b_R in Bx column order (0 on skipped columns) staged once per workgroup, so the
  // column loop has one global load per step and no dependent jmap -> b_R gather
  __shared__ double wb[CH][EB_MAXC];
  for (int i = threadIdx.x; i < nch * A.ldbx; i += 256) {
    const int ci = i / A.ldbx, t = i % A.ldbx;
    const int jr = A.jmap[t];
    wb[ci][t] = (jr >= 0) ? A.bR[(int64_t)(c0 + ci) * A.ldbR + jr] : 0.0;
  }
  __syncthreads();
  const int e = (int)blockIdx.x * EB_EPB + (threadIdx.x >> 2), sub = threadIdx.x & 3;
  const bool ok = e < A.ne;  // uniform over each quad
  const double* row = A.Bx + (int64_t)c0 * A.bx_cs + (int64_t)(ok ? e : 0) * A.ldbx;
  double s[CH];
#pragma unroll
  for (int ci = 0; ci < CH; ++ci) s[ci] = 0.0;
  if (ok) {
#pragma unroll 4
    for (int t = sub; t < A.ldbx; t += 4) {
      const double v = row[t];
#pragma unroll
      for (int ci = 0; ci < CH; ++ci) s[ci] = fma(-v, wb[ci][t], s[ci]);
    }
  }
#pragma unroll
  for (int ci = 0; ci < CH; ++ci) {
    s[ci] += __shfl_xor(s[ci], 1);
    s[ci] += __shfl_xor(s[ci], 2);
  }
  if (!ok || sub != 0) return;
  const double dE = row[A.dcol];
#pragma unroll
  for (int ci = 0; ci < CH; ++ci) {
    const int c = c0 + ci;
    if (ci >= nch) break;
    if (A.chain_mask && !A.chain_mask[c]) continue;
    double inv, lg;
    ec_phi(A.x[(int64_t)c * A.ldx + A.xcol[A.ebk[e]]], inv, lg);
    const double a = A.Dg[(int64_t)c * A.dg_cs + e] + inv;
    double z;
    if (A.z) {
      z = A.z[(int64_t)c * A.m + A.ecid[e]];
    } else {
      double n1, n2;
      gs_normal2(gs_counter((uint32_t)(e >> 1), gs_sweep(A.sweep, A.sweep_dev), A.chain_base + c, 0, A.event),
                 A.key, n1, n2);
      z = (e & 1) ? n2 : n1;
    }
    A.b[(int64_t)c * A.ldb + A.ecid[e]] = (dE + s[ci]) / a + z / sqrt(a);
  }
}

template <int NB, int NP, int PART>
void launch_schur_part(hipStream_t s, const EcorrSchurArgs& a) {
  static bool attr = false;
  const size_t lds = (size_t)2 * EC_CH * 16 * NB * sizeof(double);
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_ecorr_schur<NB, NP, PART>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL((k_ecorr_schur<NB, NP, PART>), dim3((unsigned)((a.n_chain + EC_WAVES - 1) / EC_WAVES)),
                     dim3(64 * EC_WAVES), lds, s, a);
}

template <int NB>
void launch_schur_nb(hipStream_t s, const EcorrSchurArgs& a) {
  if constexpr (NB >= 7) {
    launch_schur_part<NB, 2, 0>(s, a);
    launch_schur_part<NB, 2, 1>(s, a);
  } else {
    launch_schur_part<NB, 1, 0>(s, a);
  }
}

template <int NB, bool LNL, bool PC, bool INC = false>
void launch_prefix_nbp(hipStream_t s, const EcorrPrefixArgs& a) {
  static bool attr = false;
  const size_t lds = (PC || INC) ? (size_t)EC_WAVES *
                               (GS_EC_PCDMA ? EC_NBUF * EC_PCH * 16 * NB + 64 : EC_PCH * 16 * NB + EC_PCH) *
                               sizeof(double)
                        : (size_t)2 * EC_CH * 16 * NB * sizeof(double);
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_ecorr_prefix<NB, LNL, PC, INC>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL((k_ecorr_prefix<NB, LNL, PC, INC>), dim3((unsigned)((a.n_chain + EC_WAVES - 1) / EC_WAVES)),
                     dim3(64 * EC_WAVES), lds, s, a);
}

template <int NB, bool LNL>
void launch_prefix_nb(hipStream_t s, const EcorrPrefixArgs& a) {
  if constexpr (LNL) {
    if (a.xold) {  // incremental Metropolis step (shared or per-chain operands alike)
      launch_prefix_nbp<NB, true, false, true>(s, a);
      return;
    }
  }
  if (a.bx_cs) launch_prefix_nbp<NB, LNL, true>(s, a);
  else launch_prefix_nbp<NB, LNL, false>(s, a);
}

// per-chain [B | d_E], Dg, Ap from per-chain TNT / d (white noise sampled)
__global__ __launch_bounds__(256) void k_ecorr_gather(EcorrGatherArgs A) {
  const int c = blockIdx.y;
  const int kb = A.kb, ne = A.ne, m = A.m;
  const double* T = A.TNT + (int64_t)c * A.tnt_cstride;
  const double* dv = A.d + (int64_t)c * A.d_cstride;
  const int64_t nB = (int64_t)ne * kb, nA = (int64_t)kb * kb;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nB + nA + ne; i += (int64_t)gridDim.x * 256) {
    if (i < nB) {
      const int e = (int)(i / kb), j = (int)(i % kb);
      const int cj = A.colmap[j];
      const int ce = A.ecid[e];
      A.Bx[(int64_t)c * nB + i] = (cj >= 0) ? T[(int64_t)ce * m + cj] : ((cj == -2) ? dv[ce] : 0.0);
    } else if (i < nB + nA) {
      const int64_t k = i - nB;
      const int r = (int)(k / kb), j = (int)(k % kb);
      const int cr = A.colmap[r], cj = A.colmap[j];
      double v;
      if (cr >= 0 && cj >= 0) {
        v = T[(int64_t)cr * m + cj];
        if (r == j && r < 16) v += A.phm[r];
      } else if (cr == -2 && cj >= 0) {
        v = dv[cj];
      } else if (cj == -2 && cr >= 0) {
        v = dv[cr];
      } else {
        v = (r == j && cr == -1) ? 1.0 : 0.0;
      }
      A.Ap[(int64_t)c * nA + k] = v;
    } else {
      const int e = (int)(i - nB - nA);
      const int ce = A.ecid[e];
      A.Dg[(int64_t)c * ne + e] = T[(int64_t)ce * m + ce];
    }
  }
}

}  // namespace

int launch_ecorr_prefix(hipStream_t s, const EcorrPrefixArgs& a) {
  const bool lnl = a.lnl != nullptr;
  switch (a.ldbx / 16) {
    case 3: lnl ? launch_prefix_nb<3, true>(s, a) : launch_prefix_nb<3, false>(s, a); break;
    case 4: lnl ? launch_prefix_nb<4, true>(s, a) : launch_prefix_nb<4, false>(s, a); break;
    case 5: lnl ? launch_prefix_nb<5, true>(s, a) : launch_prefix_nb<5, false>(s, a); break;
    default: return 1;
  }
  return 0;
}

bool ecorr_nb_supported(int nb) { return nb >= 1 && nb <= 8; }  // NB 7, 8: two tile halves

int launch_ecorr_schur(hipStream_t s, const EcorrSchurArgs& a) {
  switch (a.ldbx / 16) {
    case 1: launch_schur_nb<1>(s, a); break;
    case 2: launch_schur_nb<2>(s, a); break;
    case 3: launch_schur_nb<3>(s, a); break;
    case 4: launch_schur_nb<4>(s, a); break;
    case 5: launch_schur_nb<5>(s, a); break;
    case 6: launch_schur_nb<6>(s, a); break;
    case 7: launch_schur_nb<7>(s, a); break;
    case 8: launch_schur_nb<8>(s, a); break;
    default: return 1;
  }
  return 0;
}

int launch_ecorr_propose(hipStream_t s, const EcorrMhArgs& a) {
  hipLaunchKernelGGL(k_ecorr_propose, dim3((unsigned)((a.n_chain + 255) / 256)), dim3(256), 0, s, a);
  return 0;
}

int launch_ecorr_accept(hipStream_t s, const EcorrMhArgs& a) {
  hipLaunchKernelGGL(k_ecorr_accept, dim3((unsigned)((a.n_chain + 255) / 256)), dim3(256), 0, s, a);
  return 0;
}

int launch_ecorr_gather(hipStream_t s, const EcorrGatherArgs& a) {
  const int64_t n = (int64_t)a.ne * a.kb + (int64_t)a.kb * a.kb + a.ne;
  hipLaunchKernelGGL(k_ecorr_gather, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 64), (unsigned)a.n_chain),
                     dim3(256), 0, s, a);
  return 0;
}

int launch_ecorr_bdraw_e(hipStream_t s, const EcorrBArgs& a) {
  const unsigned gx = (unsigned)(eb_blk(a.ne) + (a.mR + 255) / 256);
  if (a.bx_cs == 0)  // shared Bx: 8 chains per workgroup
    hipLaunchKernelGGL(k_ecorr_bdraw_e<8>, dim3(gx, (unsigned)((a.n_chain + 7) / 8)), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(k_ecorr_bdraw_e<1>, dim3(gx, (unsigned)a.n_chain), dim3(256), 0, s, a);
  return 0;
}
