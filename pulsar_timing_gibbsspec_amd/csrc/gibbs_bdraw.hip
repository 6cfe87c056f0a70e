// b|rho conditional and the fused free-spectrum sweep (gfx950, fp64).
//
// Algorithm: Sigma = TNT + diag(phiinv) is factorised with the
// fixed-prior columns (timing model, phiinv constant) first.  That prefix of
// the Cholesky does not change between sweeps, so it is done once per model by
// gs_prefix; each sweep only factorises the NF x NF Schur block
// S = S0 + diag(phiinv_F) (NF = 2 n_f <= 64), one wavefront per system:
//
//   lane i owns row i of the SYMMETRIC trailing matrix in registers a[0..NF-1].
//   Right-looking step k: pivot broadcast by v_readlane, lanes > k scale their
//   a[k] into L[i][k], every lane > k applies a[j] -= L[i][k] L[j][k] for
//   j > k with L[j][k] broadcast from lane j.  Because the update is applied to
//   the whole symmetric trailing block, lane i ends up holding row i of L
//   (a[j<i]) AND, unscaled, column i of L (a[j>i] = L[j][i] L[i][i]), so both
//   triangular solves are lane-local AXPYs on a broadcast scalar: no LDS, no
//   shuffles, no barriers.
//
// Reference: PulsarBlockGibbs.update_b pulsar_gibbs.py:489-520 (SVD draw);
// the draw law is identical (b ~ N(Sigma^-1 d, Sigma^-1)); with injected normals
// rotated by the oracle (z' = L^T U S^-1/2 z) the samples coincide.
#include <cmath>

#include "gibbs_common.h"
#include "gibbs_internal.h"
#include "gibbs_tile.h"
#include "gibbs_tile2.h"

#ifndef GS_SWEEP_MINW
#define GS_SWEEP_MINW 2
#endif

#define GS_BCAST_READLANE 0
#define GS_BCAST_LDS 1
#define GS_BCAST_BATCH 2
#define GS_BCAST_TILE 3

// min waves per SIMD (launch bounds) of the tile variant: 3 (<= 168 VGPRs).  Round 2 measured 3
// slower than 2 (3.05 vs 2.85 ms per launch: 35 spilled VGPRs, 54 spilled SGPRs at 207 VGPRs).
// Round 3 (r03f, MI355X, NF = 60, 4096 chains, interleaved A/B): with the tiled model block (no
// SGPR spills, 196 VGPRs) and z_F / the previous b parked in LDS (186 VGPRs) the 3-wave build
// spills 13 VGPRs, all outside the sweep's inner body, and runs 2.235 vs 2.281-2.287 ms per
// launch.  The run-time-NF instantiations with 4-5 tile rows keep 2 (24 / 84 spills at 3).
#ifndef GS_TILE_MINW
#define GS_TILE_MINW 3
#endif
#define GS_MINW(bc, nfc, ntc) \
  (((bc) == GS_BCAST_TILE || (nfc) == 0) ? (((nfc) == 0 && (ntc) >= 4) ? 2 : GS_TILE_MINW) : GS_SWEEP_MINW)

// per-wave LDS scratch (doubles) of each factorisation variant
#define GS_SCR_DOUBLES(bc, nf) ((bc) == GS_BCAST_TILE ? gs_tile_scr(nf) : 64)

#ifndef GS_BCAST_CHUNK
#define GS_BCAST_CHUNK 8
#endif

namespace {

// An SGPR copy of a compile-time index the compiler cannot see through: keeps
// the per-step lane masks (lane == k, lane > k) from being CSE'd across the
// fully unrolled factorisation and held live (3 x NF 64-bit masks -> SGPR spills).
__device__ __forceinline__ int opaque(int v) {
  asm volatile("" : "+s"(v));
  return v;
}

struct ModelLds {
  const double* S0;  // NF x (NF+1)
  const double* dF;  // NF
  const double* G;   // NMX x (NF+1)
  const double* h;   // NMX
  const double* R;   // NMX x NMX
};

template <bool FX>
__device__ __forceinline__ ModelTiled model_tiled_view(const double* base, int NF, int NMX) {
  ModelTiled m;
  m.S = base;
  m.fixt = FX;  // == model_tiled_fix(NMX): the launcher picks the instantiation
  if (FX) {
    m.G = base + model_tiled_g_offset(NF);
    m.R = base + model_tiled_r_offset(NF, NMX);
    m.h = base + model_tiled_h_offset(NF, NMX);
  } else {  // row-major G | h | R after S'
    m.G = base + model_tiled_g_offset(NF);
    m.h = m.G + (int64_t)NMX * (NF + 1);
    m.R = m.h + NMX;
  }
  return m;
}
// The view of a block staged with the pulsar's own layout (FX: the batch's NMX <= 16, all tiled);
// returns the NMX the tile core indexes the block with.
template <bool FX>
__device__ __forceinline__ ModelTiled model_tiled_view_psr(const double* base, int NF, int NMX, int nM, int& NMXe) {
  if (FX) {
    NMXe = NMX;
    return model_tiled_view<true>(base, NF, NMX);
  }
  NMXe = model_tiled_layout(NMX, nM);
  return model_tiled_fix(NMXe) ? model_tiled_view<true>(base, NF, NMXe) : model_tiled_view<false>(base, NF, NMX);
}

__device__ __forceinline__ ModelLds model_view(const double* base, int NF, int NMX) {
  ModelLds m;
  m.S0 = base;
  m.dF = m.S0 + NF * (NF + 1);
  m.G = m.dF + NF;
  m.h = m.G + NMX * (NF + 1);
  m.R = m.h + NMX;
  return m;
}

// One b|rho draw for the wavefront's system.  Inputs per lane: phinv (lane < NF),
// zF (lane < NF), zM (lane < nM).  Outputs: bF (lane < NF), bM (lane < nM).
// Returns the 1-based index of the first non-positive pivot (0 = ok), uniform.
template <int NF, int BC>
__device__ __forceinline__ int bdraw_wave(const ModelLds& M, int NMX, int nM, int lane,
                                          double phinv, double zF, double zM, double& bF,
                                          double& bM, double* __restrict__ scr) {
  const bool act = lane < NF;
  const int row = act ? lane : 0;
  double a[NF];
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    const double v = act ? M.S0[row * (NF + 1) + j] : 0.0;
    a[j] = (opaque(j) == lane) ? v + phinv : v;
  }
  // ---- right-looking Cholesky, symmetric trailing update
  double dinv = 0.0;
#pragma unroll
  for (int k = 0; k < NF; ++k) {
    const int kk = opaque(k);
    const double piv = rdlane(a[k], k);
    const double rs = rsqrt(piv);
    dinv = (lane == kk) ? rs : dinv;
    const double lk = a[k] * rs;
    const bool below = lane > kk;
    const double f = below ? lk : 0.0;
    a[k] = below ? lk : a[k];
    if constexpr (BC == GS_BCAST_READLANE) {
#pragma unroll
      for (int j = k + 1; j < NF; ++j) {
        a[j] = fma(-f, rdlane(a[k], j), a[j]);
        // bound the broadcasts in flight (each holds 2 SGPRs until its FMA)
        if (((j - k) % GS_BCAST_CHUNK) == 0) __builtin_amdgcn_sched_barrier(0);
      }
    } else if constexpr (BC == GS_BCAST_BATCH) {
      // batches of GS_BCAST_CHUNK broadcasts into distinct SGPR pairs, then the
      // FMAs: the readlane -> SGPR-read wait states overlap instead of a s_nop
      // per pair.  Constant trip counts so the inner loops unroll before k's.
#pragma unroll
      for (int j0 = 0; j0 < NF; j0 += GS_BCAST_CHUNK) {
        if (j0 + GS_BCAST_CHUNK - 1 > k) {
          double l[GS_BCAST_CHUNK];
#pragma unroll
          for (int q = 0; q < GS_BCAST_CHUNK; ++q)
            if (j0 + q > k && j0 + q < NF) l[q] = rdlane(a[k], j0 + q);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int q = 0; q < GS_BCAST_CHUNK; ++q)
            if (j0 + q > k && j0 + q < NF) a[j0 + q] = fma(-f, l[q], a[j0 + q]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    } else {
      // column k through the wave's LDS slot: one ds_write_b64 per lane, then
      // same-address (broadcast) ds_read_b128 pairs; DS ops of a wave are in order.
      scr[lane] = f;
      wave_lds_sync();
#pragma unroll
      for (int j = (k + 1) & ~1; j < NF; j += 2) {
        const double2 v = *reinterpret_cast<const double2*>(scr + j);
        if (j > k) a[j] = fma(-f, v.x, a[j]);
        a[j + 1] = fma(-f, v.y, a[j + 1]);
        if ((((j - k) >> 1) % (GS_BCAST_CHUNK / 2)) == 0) __builtin_amdgcn_sched_barrier(0);
      }
      wave_lds_sync();
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  // first non-positive pivot: lane k's dinv = rsqrt(pivot k) is NaN/inf/<=0
  const unsigned long long badm = __ballot(act && !(dinv > 0.0 && dinv < __builtin_inf()));
  const int fail = badm ? (__ffsll((long long)badm)) : 0;
  // ---- forward solve L y = dF (column AXPY)
  double r = act ? M.dF[row] : 0.0;
#pragma unroll
  for (int k = 0; k < NF; ++k) {
    const int kk = opaque(k);
    const double yk = rdlane(r * dinv, k);
    r = (lane == kk) ? yk : ((lane > kk) ? fma(-a[k], yk, r) : r);
  }
  // ---- back solve L^T x = y + zF; lane i < k holds L[k][i] L[i][i] in a[k]
  const double w = r + zF;
  double acc = 0.0, gacc = 0.0;
  const bool actm = lane < nM;
  const int mrow = actm ? lane : 0;
#pragma unroll
  for (int k = NF - 1; k >= 0; --k) {
    const int kk = opaque(k);
    const double xk = rdlane((w - dinv * acc) * dinv, k);
    bF = (lane == kk) ? xk : bF;
    acc = (lane < kk) ? fma(a[k], xk, acc) : acc;
    gacc = fma(actm ? M.G[mrow * (NF + 1) + k] : 0.0, xk, gacc);
  }
  // ---- fixed-prior block: x_M = h + R z_M - G x_F
  double v = actm ? M.h[mrow] - gacc : 0.0;
  for (int j = 0; j < nM; ++j) {
    const double zj = rdlane(zM, j);
    v = fma(actm ? M.R[mrow * NMX + j] : 0.0, zj, v);
  }
  if (actm) bM = v;
  return fail;
}

// One b|rho draw with the variant BC (tile MFMA or lane-row broadcast).  NFC > 0: the
// fixed-NF instantiations (20 / 40 / 60, every variant); NFC == 0: any even NF < 16 NTC at
// run time (tile variant only).
// LNLD (tile variant only): also leave gs_lnlike_marg's y and pivots in scr (lnl_terms).
template <int NFC, int NTC, int BC, bool PR = false, bool LNLD = false, typename ModelT>
__device__ __forceinline__ int bdraw_sys(const ModelT& M, int NMX, int nM, int lane, double phinv,
                                         double zF, double zM, double& bF, double& bM, double* scr, int NF) {
  constexpr int L = LNLD ? 2 : 0;
  if constexpr (NFC == 0)
    return bdraw_tile_n<NTC, L, PR>(M, NMX, nM, lane, phinv, zF, zM, bF, bM, scr, NF);
  else if constexpr (BC == GS_BCAST_TILE)
    return bdraw_tile<NFC, L, PR>(M, NMX, nM, lane, phinv, zF, zM, bF, bM, scr);
  else {
    static_assert(!LNLD, "the likelihood terms come with the tile variant only");
    return bdraw_wave<NFC, BC>(M, NMX, nM, lane, phinv, zF, zM, bF, bM, scr);
  }
}

// Copy a pulsar's model block into LDS (whole workgroup), 16 bytes per lane and access: model
// blocks are a 16-byte multiple of doubles (model_stride_doubles) at 16-byte aligned offsets.
// GS_STAGE_GLDS: by LDS-DMA (global_load_lds_dwordx4: no VGPR round trip, no ds_write), each
// wave-instruction filling 1 KB of the block lane-linearly.
#ifndef GS_STAGE_GLDS
#define GS_STAGE_GLDS 1
#endif
typedef __attribute__((address_space(3))) void* gs_lds_vptr;
__device__ __forceinline__ void stage_model(double* lds, const double* g, int64_t n) {
  const int n2 = (int)(n >> 1);
#if GS_STAGE_GLDS
  const int wave = gs_wave_id(), lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  for (int base = wave * 64; base < n2; base += nw * 64) {
    if (base + lane < n2)
      __builtin_amdgcn_global_load_lds((const void*)(g + 2 * (base + lane)), (gs_lds_vptr)(lds + 2 * base), 16, 0,
                                       0);
  }
  gs_wait_dma();
#else
  const double2* __restrict__ g2 = reinterpret_cast<const double2*>(g);
  double2* l2 = reinterpret_cast<double2*>(lds);
#pragma unroll 4
  for (int i = threadIdx.x; i < n2; i += blockDim.x) l2[i] = g2[i];
#endif
  __syncthreads();
}

// The fused sweep's model block in the register-tile layout (gibbs_tile.h ModelTiled,
// gibbs_internal.h model_tiled_*), built in LDS once per launch from the row-major block in
// global memory (L2): one double per thread and step, amortised over the launch's sweeps.
// Values are copied (or negated, G) exactly, so the draws are bit-identical to the row-major path.
#ifndef GS_SWEEP_TILED
#define GS_SWEEP_TILED 1
#endif
// NMX: the batch's fixed-column count (the row-major block's strides); the LDS layout is the
// pulsar's own, model_tiled_layout(NMX, nM).
__device__ void stage_model_tiled(double* __restrict__ L, const double* __restrict__ g, int NF, int NMX, int nM) {
  const int NML = model_tiled_layout(NMX, nM);
  const int NT = model_tiled_nt(NF), LD = NF + 1, nP = model_tiled_np(NML);
  const bool fixt = model_tiled_fix(NML);
  const int oG = (int)model_tiled_g_offset(NF), n = (int)model_tiled_doubles(NF, NMX);
  const int oR = fixt ? (int)model_tiled_r_offset(NF, NML) : n, oH = fixt ? (int)model_tiled_h_offset(NF, NML) : n;
  const double* S0 = g;  // NF x (NF + 1), column NF = dF
  const double* G = g + NF * LD + NF;
  const double* h = G + NMX * LD;
  const double* R = h + NMX;
  for (int idx = threadIdx.x; idx < n; idx += blockDim.x) {
    const int l = idx & 63, s = (idx >> 6) & 3, q = l >> 4, c = l & 15;
    double v = 0.0;
    if (idx < oG) {  // S': tile (I, J), I <= J, row-major over the upper triangle of tiles
      int t = idx >> 8, I = 0;
      while (t >= NT - I) t -= NT - I++;
      const int J = I + t, r = 16 * I + 4 * s + q, col = 16 * J + c;
      if (r < NF && col < NF)
        v = S0[r * LD + col];
      else if (r < NF && col == NF)
        v = S0[r * LD + NF];  // dF on the augmented column ...
      else if (r == NF && col < NF)
        v = S0[col * LD + NF];  // ... and row
      else if (r == col)
        v = 1.0;  // identity padding (the augmented pivot too)
    } else if (!fixt) {  // row-major G | h | R, copied as they are
      const int k = idx - oG;
      if (k < NMX * LD + NMX + NMX * NMX) v = G[k];
    } else if (idx < oR) {  // G' = -G: chunk P (rows 16 P + c), tile column J
      const int k = idx - oG, P = k / (NT * 256), J = (k >> 8) % NT;
      const int row = 16 * P + c, f = 16 * J + 4 * s + q;
      if (row < nM && f < NF) v = -G[row * LD + f];
    } else if (idx < oH) {  // R': chunk pair (P, Q >= P)
      int t = (idx - oR) >> 8, P = 0;
      while (t >= nP - P) t -= nP - P++;
      const int Q = P + t, row = 16 * P + c, mm = 16 * Q + 4 * s + q;
      if (row < nM && mm < nM) v = R[row * NMX + mm];
    } else {
      const int k = idx - oH;
      if (k < NML) v = h[k];
    }
    L[idx] = v;
  }
  __syncthreads();
}

// ------------------------------------------------------------ batched b draw, wide timing model
// 64 < nM <= 128 fixed-prior columns (NF <= 64): the model block (R alone is up to 128 KB) is
// read from global memory / L2, z_M rows 64.. come from Philox slot 64 + lane (or injected),
// and rows >= 64 of x_M are stored by the factorisation routine itself.
template <int NTC, int WPB>
__global__ __launch_bounds__(64 * WPB, 2) void k_bdraw_wide(BdrawArgs A) {
  extern __shared__ double lds[];
  const int NF = A.NF;
  const int wave = gs_wave_id(), lane = threadIdx.x & 63;
  const int nb = (A.n_chain + WPB - 1) / WPB;
  const int p = blockIdx.x / nb;
  const int c = (blockIdx.x % nb) * WPB + wave;
  if (c >= A.n_chain) return;
  const int64_t sys = (int64_t)p * A.n_chain + c;
  if (A.chain_mask && A.chain_mask[A.mask_per_sys ? sys : (int64_t)c] == 0) return;
  const ModelLds M = model_view(A.model + (A.model_per_sys ? sys : (int64_t)p) * A.mstride, NF, A.NMX);
  const int nM = __builtin_amdgcn_readfirstlane(A.nm[p]);  // uniform: SGPR
  const int32_t* mrow = A.midx + (int64_t)p * A.NMX;
  const int fi = lane < NF ? A.fidx[p * NF + lane] : 0;
  const int mi = lane < nM ? mrow[lane] : 0;
  const int mia = 64 + lane < nM ? mrow[64 + lane] : 0;
  const double phinv = lane < NF ? A.phiinv_F[(A.phi_per_chain ? (int64_t)c : sys) * NF + lane] : 0.0;
  double zF = 0.0, zM = 0.0, zMa = 0.0;
  if (A.z) {
    zF = lane < NF ? A.z[sys * A.ldb + fi] : 0.0;
    zM = lane < nM ? A.z[sys * A.ldb + mi] : 0.0;
    zMa = 64 + lane < nM ? A.z[sys * A.ldb + mia] : 0.0;
  } else {
    const long long sw = gs_sweep(A.sweep, A.sweep_dev);
    gs_normal2(gs_counter(lane, sw, A.chain_base + c, p + A.psr_base, A.event), A.key, zF, zM);
    double unused;
    gs_normal2(gs_counter(64 + lane, sw, A.chain_base + c, p + A.psr_base, A.event), A.key, zMa, unused);
  }
  double bF = 0.0, bM = 0.0;
  double* scr = lds + wave * gs_tile_scr(NF);
  double* brow = A.b + sys * A.ldb;
  const int fail = bdraw_tile_wide<NTC>(M, A.NMX, nM, lane, phinv, zF, zM, zMa, bF, bM, scr, NF, brow, mrow);
  if (!fail) {  // non-PD Sigma: the previous b stays (wave-uniform)
    if (lane < NF) brow[fi] = bF;
    if (lane < nM) brow[mi] = bM;
  } else if (A.fail_count && lane == 0) {
    A.fail_count[sys] += 1;
  }
  if (A.info && lane == 0) A.info[sys] = fail;
}

// ------------------------------------------------------------ batched b draw
// Issue priorities in k_bdraw / k_bdraw_tiled: on since the 4-group loop made its waves long-lived
// (r03l: CURN k_bdraw 0.535/0.526 vs 0.549/0.535 ms, CURN + red 0.540/0.540 vs 0.554/0.551; round 2's
// one-draw waves lost 25 % with them)
#ifndef GS_BDRAW_PR
#define GS_BDRAW_PR true
#endif
// Chain groups per workgroup (shared model: staged once for all of them).  Measured on MI355X
// (r03h, CURN line, 2048 chains x 45 pulsars, k_bdraw per launch): 1 -> 0.563-0.570 ms, 4 -> 0.545,
// 8 -> 0.566 (fewer, longer workgroups: the last round of the grid runs part-empty).
#ifndef GS_BDRAW_LOOP
#define GS_BDRAW_LOOP 4
#endif
// Shared model converted to the register-tile layout by each workgroup from global memory
// (stage_model_tiled) -- measured slower in k_bdraw (0.873 ms at loop 1, 0.631-0.661 at loop 4/8):
// unlike the fused sweep, one launch draws too few systems per workgroup to amortise the conversion.
#ifndef GS_BDRAW_TILED
#define GS_BDRAW_TILED 0
#endif
// k_bdraw_tiled's persistent ranges in XCD-major order (1) or in workgroup order (0).  Measured on
// MI355X (r05b, interleaved A/B, 2048 chains x 45 pulsars): XCD-major was SLOWER -- CURN 4.01e6 vs
// 4.11-4.12e6 chain-it/s, curn_plred 1.75e6 vs 1.78e6 -- although it fetches each pulsar's block
// into one or two XCDs' L2 instead of eight: the draw is issue bound, and a contiguous run of
// pulsars per XCD loads the XCDs unevenly (the per-pulsar cost varies with the timing model).  Off.
#ifndef GS_BDRAW_XCD
#define GS_BDRAW_XCD 0
#endif
// lnl[sys] of k_lnlike_marg from the two factorisation terms (gs_ctx_set_bdraw_lnl)
__device__ __forceinline__ void bdraw_lnl_store(const BdrawArgs& A, int p, int64_t sys, int NF, int lane, double phinv,
                                                int fail, double yy, double lp) {
  double lph = lane < NF ? gs_log_lnl(phinv) : 0.0;  // phinv > 0 (lnl_terms)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) lph += __shfl_xor(lph, o);
  if (lane == 0) {
    const double* aux = A.lnl_model + (int64_t)p * A.lnl_mstride + model_aux_offset(NF, A.NMX);
    A.lnl[sys] = fail ? -__builtin_inf() : 0.5 * (aux[1] + yy - 2.0 * aux[0] - lp) + 0.5 * lph;
  }
}

// one (pulsar p, chain c) system of k_bdraw.  LNLD: also lnl[sys] = gs_lnlike_marg's value at the
// same phiinv (bit-identical: the same factorisation and accumulation, the model constants from the
// row-major block A.lnl_model) -- the PTA hyper block's lnL_p seed for the next sweep -- for the
// systems the gate skips as well (likelihood mode on the already staged block: no second launch).
template <int NFC, int NTC, int BC, bool LNLD = false, typename ModelT>
__device__ __forceinline__ void bdraw_item(const BdrawArgs& A, const ModelT& M, int p, int c, int NF, int nM, int fi,
                                           int mi, double* scr, int lane, int NMXe = -1) {
  if (NMXe < 0) NMXe = A.NMX;  // the NMX the block is indexed with (model_tiled_view_psr)
  const int64_t sys = (int64_t)p * A.n_chain + c;
  const bool shut = A.chain_mask && A.chain_mask[A.mask_per_sys ? sys : (int64_t)c] == 0;  // gate closed: keep b
  if constexpr (!LNLD) {
    if (shut) return;
  }
  const double phinv = lane < NF ? A.phiinv_F[(A.phi_per_chain ? (int64_t)c : sys) * NF + lane] : 0.0;
  if constexpr (LNLD) {
    if (shut) {  // no draw, but the lnL at this phiinv all the same (likelihood mode: no solves)
      double yy = 0.0, lp = 0.0;
      int fail;
      if constexpr (NFC == 0)
        fail = bdraw_tile_n<NTC, 1, GS_BDRAW_PR>(M, NMXe, nM, lane, phinv, 0.0, 0.0, yy, lp, scr, NF);
      else
        fail = bdraw_tile<NFC, 1, GS_BDRAW_PR>(M, NMXe, nM, lane, phinv, 0.0, 0.0, yy, lp, scr);
      bdraw_lnl_store(A, p, sys, NF, lane, phinv, fail, yy, lp);
      return;
    }
  }
  double zF = 0.0, zM = 0.0;
  if (A.z) {
    zF = lane < NF ? A.z[sys * A.ldb + fi] : 0.0;
    zM = lane < nM ? A.z[sys * A.ldb + mi] : 0.0;
  } else {
    gs_normal2(gs_counter(lane, gs_sweep(A.sweep, A.sweep_dev), A.chain_base + c, p + A.psr_base, A.event), A.key, zF,
               zM);
  }
  double bF = 0.0, bM = 0.0;
  const int fail = bdraw_sys<NFC, NTC, BC, GS_BDRAW_PR, LNLD>(M, NMXe, nM, lane, phinv, zF, zM, bF, bM, scr, NF);
  if (!fail) {  // non-PD Sigma: the previous b stays (wave-uniform)
    if (lane < NF) A.b[sys * A.ldb + fi] = bF;
    if (lane < nM) A.b[sys * A.ldb + mi] = bM;
  } else if (A.fail_count && lane == 0) {
    A.fail_count[sys] += 1;
  }
  if (A.info && lane == 0) A.info[sys] = fail;
  if constexpr (LNLD) {
    double yy, lp;
    lnl_terms(scr, lane, NF, yy, lp);
    bdraw_lnl_store(A, p, sys, NF, lane, phinv, fail, yy, lp);
  }
}

template <int NFC, int NTC, int WPB, int BC>
__global__ __launch_bounds__(64 * WPB, GS_MINW(BC, NFC, NTC)) void k_bdraw(BdrawArgs A) {
  extern __shared__ double lds[];
  const int NF = NFC ? NFC : A.NF;
  const int wave = gs_wave_id(), lane = threadIdx.x & 63;
  const int nb = (A.n_chain + WPB - 1) / WPB;
  if (A.model_per_sys) {
    // per-system models (white-noise runs, TNT differs per chain): read from global memory (L2)
    const int p = blockIdx.x / nb;
    const int c = (blockIdx.x % nb) * WPB + wave;
    if (c >= A.n_chain) return;
    const int nM = __builtin_amdgcn_readfirstlane(A.nm[p]);  // uniform: SGPR
    const int fi = lane < NF ? A.fidx[p * NF + lane] : 0;
    const int mi = lane < nM ? A.midx[p * A.NMX + lane] : 0;
    const int64_t sys = (int64_t)p * A.n_chain + c;
    bdraw_item<NFC, NTC, BC>(A, model_view(A.model + sys * A.mstride, NF, A.NMX), p, c, NF, nM, fi, mi,
                             lds + wave * GS_SCR_DOUBLES(BC, NF), lane);
    return;
  }
  // shared pulsar model: staged once per workgroup for GS_BDRAW_LOOP chain groups of the pulsar
  const int nbl = (nb + GS_BDRAW_LOOP - 1) / GS_BDRAW_LOOP;
  const int p = blockIdx.x / nbl;
  const int g0 = (blockIdx.x % nbl) * GS_BDRAW_LOOP;
  const int nM = __builtin_amdgcn_readfirstlane(A.nm[p]);  // uniform: SGPR
  const int fi = lane < NF ? A.fidx[p * NF + lane] : 0;
  const int mi = lane < nM ? A.midx[p * A.NMX + lane] : 0;
  constexpr bool TL = GS_BDRAW_TILED && (BC == GS_BCAST_TILE || NFC == 0);
  using ModelT = typename std::conditional<TL, ModelTiled, ModelLds>::type;
  ModelT M;
  int64_t mlds;
  int NMXe = A.NMX;
  if constexpr (TL) {
    stage_model_tiled(lds, A.model + (int64_t)p * A.mstride, NF, A.NMX, nM);
    mlds = model_tiled_doubles(NF, A.NMX);
    M = model_tiled_view_psr<false>(lds, NF, A.NMX, nM, NMXe);
  } else {
    stage_model(lds, A.model + (int64_t)p * A.mstride, A.mstride);
    mlds = A.mstride;
    M = model_view(lds, NF, A.NMX);
  }
  double* scr = lds + mlds + wave * GS_SCR_DOUBLES(BC, NF);
#pragma unroll 1
  for (int r = 0; r < GS_BDRAW_LOOP; ++r) {
    const int c = (g0 + r) * WPB + wave;
    if (c >= A.n_chain) break;
    bdraw_item<NFC, NTC, BC>(A, M, p, c, NF, nM, fi, mi, scr, lane, NMXe);
  }
}

// ------------------------------------------------------------ tiled shared models (gs_bdraw_tiled)
// Register-tile copies of n_psr shared model blocks (one workgroup per pulsar, the fused sweep's
// stage_model_tiled writing to global memory), once per white-noise state.
__global__ void k_model_tile(const double* __restrict__ model, int64_t mstride, int NF, int NMX,
                             const int32_t* __restrict__ nm, double* __restrict__ tiled, int64_t tstride) {
  const int p = blockIdx.x;
  stage_model_tiled(tiled + p * tstride, model + p * mstride, NF, NMX, nm[p]);
}

// k_bdraw on precomputed tiled blocks: each workgroup DMA-stages its pulsar's tile-layout block
// (30.8 KB at NF = 60, nm = 16, against 40.5 KB row-major) for GS_BDRAW_LOOP chain groups, and
// the draw loads its tiles lane-linearly (tile variant only).
template <int NFC, int NTC, int WPB, bool FX, bool LNLD>
__global__ __launch_bounds__(64 * WPB, GS_MINW(GS_BCAST_TILE, NFC, NTC)) void k_bdraw_tiled(BdrawArgs A) {
  extern __shared__ double lds[];
  const int NF = NFC ? NFC : A.NF;
  const int wave = gs_wave_id(), lane = threadIdx.x & 63;
  const int nb = (A.n_chain + WPB - 1) / WPB;
  double* scr = lds + A.mstride + wave * gs_tile_scr(NF);
  if (A.persist) {
    // one round of workgroups (A.persist = CUs x resident workgroups per CU), workgroup w taking the
    // (pulsar, chain group) items [w n / G, (w + 1) n / G) in pulsar-major order: every workgroup
    // draws the same number of groups, restaging the model only where its range crosses a pulsar
    const int64_t n_items = (int64_t)A.n_psr * nb;
    // GS_BDRAW_XCD (off): XCD-major ranges -- workgroups are dealt round-robin over the 8 XCDs
    // (blocks b and b + 8 share one, MI355X_MICROARCH.md), so the workgroups of one XCD would take
    // one contiguous run of items
    int64_t w = blockIdx.x;
    if (GS_BDRAW_XCD && (A.persist & 7) == 0) w = (w & 7) * (A.persist >> 3) + (w >> 3);
    const int64_t lo = w * n_items / A.persist, hi = (w + 1) * n_items / A.persist;
    int cur = -1, nM = 0, fi = 0, mi = 0, NMXe = A.NMX;
    ModelTiled M;
#pragma unroll 1
    for (int64_t it = lo; it < hi; ++it) {
      const int p = (int)(it / nb), grp = (int)(it % nb);
      if (p != cur) {  // uniform over the workgroup
        if (cur >= 0) __syncthreads();  // every wave is done with the previous block
        stage_model(lds, A.model + (int64_t)p * A.mstride, A.mstride);
        cur = p;
        nM = __builtin_amdgcn_readfirstlane(A.nm[p]);
        fi = lane < NF ? A.fidx[p * NF + lane] : 0;
        mi = lane < nM ? A.midx[p * A.NMX + lane] : 0;
        M = model_tiled_view_psr<FX>(lds, NF, A.NMX, nM, NMXe);
      }
      const int c = grp * WPB + wave;
      if (c < A.n_chain) bdraw_item<NFC, NTC, GS_BCAST_TILE, LNLD>(A, M, p, c, NF, nM, fi, mi, scr, lane, NMXe);
    }
    return;
  }
  const int nbl = (nb + GS_BDRAW_LOOP - 1) / GS_BDRAW_LOOP;
  const int p = blockIdx.x / nbl;
  const int g0 = (blockIdx.x % nbl) * GS_BDRAW_LOOP;
  const int nM = __builtin_amdgcn_readfirstlane(A.nm[p]);  // uniform: SGPR
  const int fi = lane < NF ? A.fidx[p * NF + lane] : 0;
  const int mi = lane < nM ? A.midx[p * A.NMX + lane] : 0;
  stage_model(lds, A.model + (int64_t)p * A.mstride, A.mstride);
  int NMXe;
  const ModelTiled M = model_tiled_view_psr<FX>(lds, NF, A.NMX, nM, NMXe);
#pragma unroll 1
  for (int r = 0; r < GS_BDRAW_LOOP; ++r) {
    const int c = (g0 + r) * WPB + wave;
    if (c >= A.n_chain) break;
    bdraw_item<NFC, NTC, GS_BCAST_TILE, LNLD>(A, M, p, c, NF, nM, fi, mi, scr, lane, NMXe);
  }
}

// ------------------------------------------------------------ b draws, two chains per wave
// gs_bdraw_tiled at NF = 60 without the lnL output (GS_OPT_SWEEP_SCHED = 3, or the cost model where the
// pairs fill 2 waves per SIMD): each wave draws chains c, c + 1 of one pulsar together
// (gibbs_tile2.h bdraw_tile_pair60: both chains' diagonal eliminations in one paired register set),
// bit-identical to bdraw_item's draws -- same normals (counters per chain), same tile core per chain; a
// shut chain (chain_mask) has its draw discarded and nothing written, as bdraw_item skips it.  Pulsars
// whose fixed block is row-major (nM > 16) run bdraw_item for each chain in turn.  Persistent ranges
// of (pulsar, group of 2 WPB chains) items as k_bdraw_tiled; n_chain is even.
constexpr int GS_BPAIR_SCR = 2 * gs_tile_scr(60) + 128;  // per wave: the chains' scratches + z_M slots
// cost of a row-major pulsar's item (paired items = 10).  Measured on the 45-pulsar curn array (r06g2/3,
// every chain drawing): 0.474 ms per launch at 13, 0.441-0.445 at 15, 0.461-0.464 at 18, against
// 0.444-0.445 for k_bdraw_tiled and 0.554 unweighted (r06s)
#ifndef GS_BPAIR_RM_COST
#define GS_BPAIR_RM_COST 15
#endif

template <int WPB>
__global__ __launch_bounds__(64 * WPB, 2) void k_bdraw_pair(BdrawArgs A) {
  extern __shared__ double lds[];
  constexpr int NF = 60, CPB = 2 * WPB;
  const int wave = gs_wave_id(), lane = threadIdx.x & 63;
  const int nb = (A.n_chain + CPB - 1) / CPB;
  double* wl = lds + A.mstride + (int64_t)wave * GS_BPAIR_SCR;
  double* const scr[2] = {wl, wl + gs_tile_scr(60)};
  double* zmslot = wl + 2 * gs_tile_scr(60);
  // persistent ranges weighted by cost: an item of a pulsar whose fixed block is row-major (drawn one
  // chain at a time) costs GS_BPAIR_RM_COST / 10 of a paired one, so the workgroups covering such
  // pulsars take fewer items (without the weights they ran ~1.3x longer than the rest, r06s)
  const int64_t G = A.persist ? A.persist : (int64_t)gridDim.x;
  auto cost = [&](int q) -> int {
    if (!A.persist) return 1;  // one item per workgroup
    const int nq = __builtin_amdgcn_readfirstlane(A.nm[q]);
    return model_tiled_fix(model_tiled_layout(A.NMX, nq)) ? 10 : GS_BPAIR_RM_COST;
  };
  int64_t tot = 0;
#pragma unroll 1
  for (int q = 0; q < A.n_psr; ++q) tot += (int64_t)nb * cost(q);
  const int64_t c_lo = blockIdx.x * tot / G, c_hi = (blockIdx.x + 1) * tot / G;
  int cur = -1, nM = 0, fi = 0, mi = 0, NMXe = A.NMX;
  ModelTiled M;
  int64_t P0 = 0;
#pragma unroll 1
  for (int p = 0; p < A.n_psr && P0 < c_hi; ++p) {
    const int cp = cost(p);
    const int64_t P1 = P0 + (int64_t)nb * cp;
    // items grp with start P0 + grp cp in [c_lo, c_hi)
    const int g0 = c_lo > P0 ? (int)((c_lo - P0 + cp - 1) / cp) : 0;
    const int g1 = P1 > c_lo ? (int)min((int64_t)nb, (c_hi - P0 + cp - 1) / cp) : 0;
    P0 = P1;
#pragma unroll 1
  for (int grp = g0; grp < g1; ++grp) {
    if (p != cur) {  // uniform over the workgroup
      if (cur >= 0) __syncthreads();
      stage_model(lds, A.model + (int64_t)p * A.mstride, A.mstride);
      cur = p;
      nM = __builtin_amdgcn_readfirstlane(A.nm[p]);
      fi = lane < NF ? A.fidx[p * NF + lane] : 0;
      mi = lane < nM ? A.midx[p * A.NMX + lane] : 0;
      M = model_tiled_view_psr<false>(lds, NF, A.NMX, nM, NMXe);
    }
    const int c0 = grp * CPB + 2 * wave;
    if (c0 >= A.n_chain) continue;
    if (!M.fixt) {  // row-major fixed block (nM > 16): one chain at a time
      bdraw_item<60, 0, GS_BCAST_TILE, false>(A, M, p, c0, NF, nM, fi, mi, scr[0], lane, NMXe);
      bdraw_item<60, 0, GS_BCAST_TILE, false>(A, M, p, c0 + 1, NF, nM, fi, mi, scr[0], lane, NMXe);
      continue;
    }
    const int64_t sys0 = (int64_t)p * A.n_chain + c0;
    bool shut[2];
    double phinv[2], zF[2], zM[2];
#pragma unroll
    for (int ch = 0; ch < 2; ++ch) {
      const int64_t sys = sys0 + ch;
      const int c = c0 + ch;
      shut[ch] = A.chain_mask && A.chain_mask[A.mask_per_sys ? sys : (int64_t)c] == 0;
    }
    if (shut[0] && shut[1]) continue;
#pragma unroll
    for (int ch = 0; ch < 2; ++ch) {
      const int64_t sys = sys0 + ch;
      const int c = c0 + ch;
      // a shut chain draws on a unit prior (its draw is discarded): no read of its phiinv row
      phinv[ch] = shut[ch] ? (lane < NF ? 1.0 : 0.0)
                           : (lane < NF ? A.phiinv_F[(A.phi_per_chain ? (int64_t)c : sys) * NF + lane] : 0.0);
      if (A.z) {
        zF[ch] = lane < NF ? A.z[sys * A.ldb + fi] : 0.0;
        zM[ch] = lane < nM ? A.z[sys * A.ldb + mi] : 0.0;
      } else {
        gs_normal2(gs_counter(lane, gs_sweep(A.sweep, A.sweep_dev), A.chain_base + c, p + A.psr_base, A.event), A.key,
                   zF[ch], zM[ch]);
      }
    }
    double bF[2], bM[2];
    int f[2];
    bdraw_tile_pair60<GS_BDRAW_PR>(M, NMXe, nM, lane, phinv, zF, zM, bF, bM, scr, zmslot, f);
#pragma unroll
    for (int ch = 0; ch < 2; ++ch) {
      if (shut[ch]) continue;
      const int64_t sys = sys0 + ch;
      if (!f[ch]) {  // non-PD Sigma: the previous b stays (wave-uniform)
        if (lane < NF) A.b[sys * A.ldb + fi] = bF[ch];
        if (lane < nM) A.b[sys * A.ldb + mi] = bM[ch];
      } else if (A.fail_count && lane == 0) {
        A.fail_count[sys] += 1;
      }
      if (A.info && lane == 0) A.info[sys] = f[ch];
    }
  }
  }
}

// ------------------------------------------------------------ marginalised likelihood
//  get_lnlikelihood_fullmarg pulsar_gibbs.py:569-610, phiinv-dependent part:
//   lnl = 1/2 (d^T Sigma^-1 d - log det Sigma) + 1/2 sum_F log phiinv_F
// with the prefix: d^T Sigma^-1 d = |e|^2 + |y|^2, log det Sigma = 2 sum log diag L_M +
// log det S; |y|^2 and log det S come out of the augmented tile factorisation.  The
// model constants -1/2 (log det N + r^T N^-1 r) - 1/2 sum_M log phi_M are the caller's.
// A shared model block is staged once per workgroup for GS_BDRAW_LOOP chain groups (as k_bdraw):
// staging it for every WPB chains cost more than the factorisations (0.61 ms per configs[3]-shaped
// launch, 92k systems; r04).
template <int NFC, int NTC, int WPB>
__device__ __forceinline__ void lnlike_item(const LnlArgs& A, const double* mb, int p, int c, double* scr, int lane) {
  const int NF = NFC ? NFC : A.NF;
  const int64_t sys = (int64_t)p * A.n_chain + c;
  const ModelLds M = model_view(mb, NF, A.NMX);
  const double phinv = lane < NF ? A.phiinv_F[sys * NF + lane] : 1.0;
  double yy = 0.0, ldS = 0.0;
  int fail;
  if constexpr (NFC == 0)
    fail = bdraw_tile_n<NTC, true>(M, A.NMX, A.nm[p], lane, phinv, 0.0, 0.0, yy, ldS, scr, NF);
  else
    fail = bdraw_tile<NFC, true>(M, A.NMX, A.nm[p], lane, phinv, 0.0, 0.0, yy, ldS, scr);
  double lph = lane < NF ? gs_log_lnl(phinv) : 0.0;  // phinv > 0 (lnl_terms)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) lph += __shfl_xor(lph, o);
  const int64_t ao = model_aux_offset(NF, A.NMX);
  const double lm = mb[ao], ee = mb[ao + 1];
  if (lane == 0) {
    A.lnl[sys] = fail ? -__builtin_inf() : 0.5 * (ee + yy - 2.0 * lm - ldS) + 0.5 * lph;
    if (A.info) A.info[sys] = fail;
  }
}

template <int NFC, int NTC, int WPB>
__global__ __launch_bounds__(64 * WPB, 2) void k_lnlike_marg(LnlArgs A) {
  extern __shared__ double lds[];
  const int wave = gs_wave_id(), lane = threadIdx.x & 63;
  const int nb = (A.n_chain + WPB - 1) / WPB;
  const bool in_lds = !A.model_per_sys && !A.model_global;
  double* scr = lds + (in_lds ? A.mstride : 0) + wave * gs_tile_scr(NFC ? NFC : A.NF);
  if (!in_lds) {
    const int p = blockIdx.x / nb;
    const int c = (blockIdx.x % nb) * WPB + wave;
    if (c >= A.n_chain || (A.skip && A.skip[c])) return;
    const int64_t sys = (int64_t)p * A.n_chain + c;
    lnlike_item<NFC, NTC, WPB>(A, A.model + (A.model_per_sys ? sys : (int64_t)p) * A.mstride, p, c, scr, lane);
    return;
  }
  const int nbl = (nb + GS_BDRAW_LOOP - 1) / GS_BDRAW_LOOP;
  const int p = blockIdx.x / nbl;
  const int g0 = (blockIdx.x % nbl) * GS_BDRAW_LOOP;
  constexpr int PER = GS_BDRAW_LOOP * WPB;  // chains per workgroup
  __shared__ int sel[PER];
  if (A.skip) {
    // gs_lnlike_marg_gated: workgroup j of pulsar p takes the chains of rank [PER j, PER j + PER)
    // among those with skip[c] == 0 (a block-wide ballot scan of skip), so the model is staged only
    // by workgroups with work and every wave of them draws.  Workgroups past the count return.
    __shared__ int wcnt[WPB];
    __shared__ int base_s;
    const int want0 = (blockIdx.x % nbl) * PER;
    if (threadIdx.x < PER) sel[threadIdx.x] = -1;
    if (threadIdx.x == 0) base_s = 0;
    __syncthreads();
    for (int c0 = 0; c0 < A.n_chain; c0 += 64 * WPB) {
      const int c = c0 + (int)threadIdx.x;
      const bool todo = c < A.n_chain && A.skip[c] == 0;
      const unsigned long long m = __ballot(todo);
      if (lane == 0) wcnt[wave] = __popcll(m);
      __syncthreads();
      int rank = base_s;
      for (int w = 0; w < wave; ++w) rank += wcnt[w];
      rank += __popcll(m & ((1ull << lane) - 1ull));
      if (todo && rank >= want0 && rank < want0 + PER) sel[rank - want0] = c;
      __syncthreads();
      if (threadIdx.x == 0)
        for (int w = 0; w < WPB; ++w) base_s += wcnt[w];
      __syncthreads();
      if (base_s >= want0 + PER) break;
    }
    if (sel[0] < 0) return;
  }
  stage_model(lds, A.model + (int64_t)p * A.mstride, A.mstride);
#pragma unroll 1
  for (int r = 0; r < GS_BDRAW_LOOP; ++r) {
    const int c = A.skip ? sel[r * WPB + wave] : (g0 + r) * WPB + wave;
    if (c < 0 || c >= A.n_chain) break;
    lnlike_item<NFC, NTC, WPB>(A, lds, p, c, scr, lane);
  }
}

// ------------------------------------------------------------ PTA red hyper-parameter MH
// PTABlockGibbs.update_hyper_params with redsample='mh' (pta_gibbs.py:278-340), the reference's
// default: `nsteps` single-parameter Metropolis steps per chain on the summed marginalised
// likelihood get_lnlikelihood (:577-621).  A step moves one red parameter of ONE pulsar p, so
// only lnL_p changes: diff = lnL_p(q) - lnL_p(x) (the reference's full sums (lnlike1 + lnprior1)
// - (lnlike0 + lnprior0) differ from it only by rounding: the other pulsars' terms and the
// uniform prior constants cancel), and a proposal outside its prior box is rejected without a
// likelihood (the reference evaluates it first and can die in cho_factor on the overflowed phi).
// One wavefront per chain (one per workgroup), the chain's x row and lnL_p of every pulsar in LDS,
// the pulsar's model block read from global memory (all blocks ~2 MB: L2-resident), the
// likelihood from the augmented tile factorisation of gs_lnlike_marg (same arithmetic, so
// lnl_p seeded by gs_lnlike_marg and the in-kernel values agree exactly).
// Proposal (pta_gibbs.py:322-328): scale = choice(sizes, p), par = choice(hind), q[par] +=
// randn * (0.05 len(hind)) * scale; accept if diff > log(rand).  Philox event GS_EV_HYPER,
// slots 3 s .. 3 s + 2 of step s: (u_scale, u_par), (Box-Muller pair), (u_acc, -).

// GS_HY_W = 2: two waves per chain, wave w taking the steps whose pulsar p has p % 2 == w (a step
// changes only pulsar p's parameters and lnL_p, so the two subsequences are independent and each
// keeps the reference's step order): 4096 waves for 2048 chains instead of 2048, at <= 168 VGPRs
// (7 spilled).  Measured (power-law MH line, tools/gpu_ab_mh.sh ALT=w2): the launch alone 0.148 ->
// 0.144 ms, the sweep 1.154 -> 1.172 ms -- off by default.
#ifndef GS_HY_W
#define GS_HY_W 1
#endif
__device__ __forceinline__ void hy_sync() {
  if constexpr (GS_HY_W == 1)
    wave_lds_sync();
  else
    __syncthreads();
}

template <int NFC, int NTC>
__global__ __launch_bounds__(64 * GS_HY_W, GS_HY_W == 1 ? 2 : 3) void k_hyper_mh(HyperMhArgs A) {
  extern __shared__ double lds[];
  const int NF = NFC ? NFC : A.NF;
  const int n_f = NF / 2;
  const int lane = threadIdx.x & 63;
  const int wv = GS_HY_W == 1 ? 0 : gs_wave_id();
  const int c = blockIdx.x;
  double* xs = lds;              // the chain's x row
  double* Ls = lds + A.ldx;      // lnL_p of every pulsar at x
  // The proposals do not depend on the chain state: lane l draws step s0 + l's (scale, parameter,
  // normal, log u) for 64 steps at once into the chain's step table (3 Philox blocks per lane in
  // parallel instead of 3 wave-uniform blocks on the critical path of every step).
  double* stab = lds + ((A.ldx + A.n_psr + 1) & ~1);
  double* scr = stab + 4 * 64 + wv * gs_tile_scr(NF);
  double* xg = A.x + (int64_t)c * A.ldx;
  for (int i = threadIdx.x; i < A.ldx; i += 64 * GS_HY_W) xs[i] = xg[i];
  for (int p = threadIdx.x; p < A.n_psr; p += 64 * GS_HY_W) Ls[p] = A.lnl_p[(int64_t)p * A.n_chain + c];
  hy_sync();
  const bool act = lane < NF;
  const int kf = act ? (lane >> 1) : 0;
  // the common spectrum is fixed during the block (only red parameters move)
  const double gw = act ? pow(10.0, 2.0 * xs[A.gw_col[kf]]) : 0.0;
  const double sig = 0.05 * A.n_h;  // sigmas = 0.05 * len(hind)
  const long long chain = A.chain_base + c;
  const long long sw = gs_sweep(A.sweep, A.sweep_dev);
  int nacc = 0;
  for (int s0 = 0; s0 < A.nsteps; s0 += 64) {
    const int ns = min(64, A.nsteps - s0);
    if (wv == 0 && lane < ns) {
      const int st = s0 + lane;
      double sc, z, u;
      int j;
      if (A.inj) {
        const double* q = A.inj + ((int64_t)st * A.n_chain + c) * 4;
        sc = q[0];
        j = min(max((int)q[1], 0), A.n_h - 1);  // the host validates; never index out of range
        z = q[2];
        u = q[3];
      } else {
        double u1, u2, v1, v2, u4;
        gs_uniform2(gs_counter(3u * st, sw, chain, 0, GS_EV_HYPER), A.key, u1, u2);
        gs_normal2(gs_counter(3u * st + 1, sw, chain, 0, GS_EV_HYPER), A.key, v1, v2);
        gs_uniform2(gs_counter(3u * st + 2, sw, chain, 0, GS_EV_HYPER), A.key, u, u4);
        sc = gs_mh_scale(u1);
        j = min((int)(u2 * A.n_h), A.n_h - 1);
        z = v1;
      }
      stab[4 * lane] = sc;
      stab[4 * lane + 1] = (double)j;
      stab[4 * lane + 2] = z;
      stab[4 * lane + 3] = log(u);
    }
    hy_sync();
    for (int i = 0; i < ns; ++i) {
      const int st = s0 + i;
      const int j = __builtin_amdgcn_readfirstlane((int)stab[4 * i + 1]);
      const int col = A.hcol[j], p = A.hpsr[j];
      if (p < 0) continue;  // a pulsar of another rank (pulsar-sharded run): its steps are applied there
      if (GS_HY_W > 1 && p % GS_HY_W != wv) continue;  // the other wave's pulsar
      const double sc = stab[4 * i], z = stab[4 * i + 2], lu = stab[4 * i + 3];
      // q[par] += randn * sigmas * scale, rounded as numpy does (no fma contraction)
      const double xq = gs_add_rn(xs[col], gs_mul_rn(gs_mul_rn(z, sig), sc));
      bool accepted = false;
      if (xq >= A.hlo[j] && xq <= A.hhi[j]) {  // uniform prior: -inf outside (:298, :624-628)
        double red;
        if (A.red_kind == 0) {  // free spectrum: phi_red = 10^(2 rho_red)
          const int rc = A.red_col[p * n_f + kf];
          red = pow(10.0, 2.0 * (rc == col ? xq : xs[rc]));
        } else {                // power law: log phi_red = (a log10_A + c) + g gamma
          const int ca = A.pl_col[2 * p], cg = A.pl_col[2 * p + 1];
          const double la = ca == col ? xq : xs[ca], ga = cg == col ? xq : xs[cg];
          const double* L = A.lnphi + (int64_t)p * 3 * n_f;
          red = exp(gs_add_rn(gs_add_rn(gs_mul_rn(L[n_f + kf], la), L[kf]), gs_mul_rn(L[2 * n_f + kf], ga)));
        }
        const double phinv = act ? 1.0 / (gw + red) : 1.0;
        const double* mb = A.model + (int64_t)p * A.mstride;
        const ModelLds M = model_view(mb, NF, A.NMX);
        double yy = 0.0, ldS = 0.0;
        int fail;
        if constexpr (NFC == 0)
          fail = bdraw_tile_n<NTC, true>(M, A.NMX, A.nm[p], lane, phinv, 0.0, 0.0, yy, ldS, scr, NF);
        else
          fail = bdraw_tile<NFC, true>(M, A.NMX, A.nm[p], lane, phinv, 0.0, 0.0, yy, ldS, scr);
        double lph = act ? gs_log_lnl(phinv) : 0.0;  // as gs_lnlike_marg (bit-identical seeds)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) lph += __shfl_xor(lph, o);
        const int64_t ao = model_aux_offset(NF, A.NMX);
        const double L1 = fail ? -__builtin_inf() : 0.5 * (mb[ao + 1] + yy - 2.0 * mb[ao] - ldS) + 0.5 * lph;
        const double diff = L1 - Ls[p];
        if (diff > lu) {
          accepted = true;
          ++nacc;
          if (lane == 0) {
            xs[col] = xq;
            Ls[p] = L1;
          }
        }
        wave_lds_sync();
      }
      if (A.q_rec && lane == 0) {
        double* qr = A.q_rec + ((int64_t)st * A.n_chain + c) * 3;
        qr[0] = (double)j;
        qr[1] = xq;
        qr[2] = accepted ? 1.0 : 0.0;
      }
    }
    hy_sync();  // the next 64 steps rewrite the table
  }
  for (int i = threadIdx.x; i < A.ldx; i += 64 * GS_HY_W) xg[i] = xs[i];
  for (int p = threadIdx.x; p < A.n_psr; p += 64 * GS_HY_W) A.lnl_p[(int64_t)p * A.n_chain + c] = Ls[p];
  if constexpr (GS_HY_W > 1) {
    __shared__ int nac[GS_HY_W];
    if (lane == 0) nac[wv] = nacc;
    __syncthreads();
    if (threadIdx.x == 0)
      for (int w = 1; w < GS_HY_W; ++w) nacc += nac[w];
  }
  if (A.n_acc && threadIdx.x == 0) A.n_acc[c] = nacc;
}

// ------------------------------------------------------------ fused sweep
// GS_RNG_MERGE (off): one Philox block per lane per sweep for the rho uniforms and the normals.
// Measured on MI355X (r05d/r05e, interleaved A/B, 4096 chains, 300 launches): 2.078-2.086 ms per
// launch merged vs 2.042-2.049 with the two blocks -- the crossbar redistribution and the pair kept
// for Box-Muller raise the 12-wave kernel's spills 6 -> 19-26 VGPRs, which costs more than the 2.0 %
// the rho uniforms' Philox pass takes (profiles/r05b).
#ifndef GS_RNG_MERGE
#define GS_RNG_MERGE 0
#endif
#ifndef GS_RHO_EXP
#define GS_RHO_EXP 0
#endif
// FX: the tiled model block's fixed-prior part in tiles (nm <= 16, k_sweep_freespec) or row-major
// (k_sweep_freespec_rm): a compile-time choice, so each kernel carries only its own fixed-block
// code (both in one kernel cost the headline 7 more spilled VGPRs, +1.2 %, r03j).
template <int NFC, int NTC, int WPB, int BC, bool FX>
__device__ __forceinline__ void sweep_freespec_body(const SweepArgs& A) {
  extern __shared__ double lds[];
  const int NF = NFC ? NFC : A.NF;
  const int NFR = NF / 2;
  const int wave = gs_wave_id(), lane = threadIdx.x & 63;
  // tile variant: the model block in the register-tile layout (stage_model_tiled); the lane-row
  // broadcast variants read the row-major block
  constexpr bool TL = GS_SWEEP_TILED && (BC == GS_BCAST_TILE || NFC == 0);
  // BAL (12-wave workgroups = 3 waves on each SIMD of a CU, tile variant): 16 chains per
  // workgroup, waves 0..11 own chains 0..11 and each trio (waves 3e, 3e+1, 3e+2) runs chain 12 + e
  // in thirds of the sweeps, handed from wave to wave through LDS -- every wave draws 4/3 chains,
  // so 4096 chains fill the 3072 wave slots of a 3-waves/SIMD launch in one round instead of a
  // full round plus a third of a round at 1 wave/SIMD.
  constexpr bool BAL = TL && WPB == 12;
  constexpr int CPB = BAL ? 16 : WPB;  // chains per workgroup
  constexpr int NTRIO = BAL ? 4 : 1;
  const int nb = (A.n_chain + CPB - 1) / CPB;
  const int p = blockIdx.x / nb;
  const int cblk = (blockIdx.x % nb) * CPB;
  const int c_own = cblk + wave;
  const int nM = __builtin_amdgcn_readfirstlane(A.nm[p]);  // uniform: SGPR
  int64_t mlds;
  if constexpr (BAL) {  // hand-off flags (the staging's barrier orders this before any use)
    if (threadIdx.x < NTRIO)
      reinterpret_cast<int*>(lds + model_tiled_doubles(NF, A.NMX) + WPB * (GS_SCR_DOUBLES(BC, NF) + 128 + 256) +
                             NTRIO * 256)[threadIdx.x] = 0;
  }
  if constexpr (TL) {
    stage_model_tiled(lds, A.model + (int64_t)p * A.mstride, NF, A.NMX, nM);
    mlds = model_tiled_doubles(NF, A.NMX);
  } else {
    stage_model(lds, A.model + (int64_t)p * A.mstride, A.mstride);
    mlds = A.mstride;
  }
  if (c_own >= A.n_chain) return;  // (then no extra chain either: 12 + e > wave)
  using ModelT = typename std::conditional<TL, ModelTiled, ModelLds>::type;
  ModelT M;
  int NMXe = A.NMX;  // the NMX the staged block is indexed with (its own layout, model_tiled_view_psr)
  if constexpr (TL) {
    M = model_tiled_view_psr<FX>(lds, NF, A.NMX, nM, NMXe);
  } else {
    M = model_view(lds, NF, A.NMX);
  }
  const int64_t n_sys = (int64_t)A.n_psr * A.n_chain;
  const bool act = lane < NF, actm = lane < nM;
  const int kf = act ? (lane >> 1) : 0;  // frequency of this lane
  const int fi = act ? A.fidx[p * NF + lane] : 0;
  const int mi = actm ? A.midx[p * A.NMX + lane] : 0;
  double* scr = lds + mlds + wave * GS_SCR_DOUBLES(BC, NF);
  double* bsave = lds + mlds + WPB * GS_SCR_DOUBLES(BC, NF) + wave * 128;  // previous b (failed draws)
  // BAL: the wave's parked own-chain state (x, bF, bM, fail) while it runs the extra chain, and
  // the trio's hand-off slot of the extra chain (+ its progress flag), after the save slots
  double* park = lds + mlds + WPB * (GS_SCR_DOUBLES(BC, NF) + 128) + wave * 256;
  double* hand = lds + mlds + WPB * (GS_SCR_DOUBLES(BC, NF) + 128 + 256) + (wave / 3) * 256;
  int* hflag =
      reinterpret_cast<int*>(lds + mlds + WPB * (GS_SCR_DOUBLES(BC, NF) + 128 + 256) + NTRIO * 256) + wave / 3;
  GS_PH_INIT(scr)
#ifdef GS_STATIC_PRIO
  // A/B knob: half of the workgroups (one of the two co-resident waves of a SIMD) at priority 1
  if (blockIdx.x & 1) __builtin_amdgcn_s_setprio(1);
#endif

  const double rhomin = A.rhomin, rhomax = A.rhomax;
  const double irhomin = 1.0 / rhomin, irhomax = 1.0 / rhomax;
  const int64_t xr_step = n_sys * NFR;
  const int64_t br_step = (A.brec_nc == 0 ? n_sys : (int64_t)A.n_psr * A.brec_nc) * A.ldb;
  // segments (uniform per wave): chain, sweep range, where the state comes from / goes to
  // (0 global state arrays, 1 the wave's park slot, 2 the trio's hand-off slot)
  const int S = A.n_sweeps, s1 = S / 3, s2 = 2 * S / 3, t = wave % 3;
  const int c_ext = cblk + 12 + wave / 3;
  const bool ext = BAL && c_ext < A.n_chain;
  const int nseg = ext ? (t == 0 ? 2 : 3) : 1;
#pragma unroll 1
  for (int seg = 0; seg < nseg; ++seg) {
    int c = c_own, sw_a = 0, sw_b = S, src = 0, dst = 0, need = 0;
    if (ext) {
      if (t == 0) {  // extra [0, s1) -> hand-off, then own [0, S)
        if (seg == 0) { c = c_ext; sw_b = s1; dst = 2; }
      } else {       // own [0, sN) -> park, extra [sN, sN') from / to hand-off, own [sN, S) from park
        const int sa = t == 1 ? s1 : s2, sb = t == 1 ? s2 : S;
        if (seg == 0) { sw_b = sa; dst = 1; }
        if (seg == 1) { c = c_ext; sw_a = sa; sw_b = sb; src = 2; dst = t == 1 ? 2 : 0; need = t; }
        if (seg == 2) { sw_a = sa; src = 1; }
      }
    }
    const int64_t sys = (int64_t)p * A.n_chain + c;
    const long long gchain = A.chain_base + c;
    double x = 0.0, bF = 0.0, bM = 0.0;
    int fail = 0;
    // dead (wave-uniform): the hand-off of the extra chain did not arrive in time, or arrived
    // poisoned by an earlier dead third -- the segment's sweeps are skipped, nothing stale is
    // recorded or stored, and the chain ends with info = -1 (the host raises on it)
    bool dead = false;
    if (src == 0) {
      x = act ? A.x_state[sys * NFR + kf] : 0.0;
      bF = act ? A.b_state[sys * A.ldb + fi] : 0.0;
      bM = actm ? A.b_state[sys * A.ldb + mi] : 0.0;
    } else {
      double* slot = src == 1 ? park : hand;
      if (src == 2) {
        // wait for the trio's previous third of the extra chain (its waves are co-resident: same
        // workgroup); bounded, so a logic error cannot hang the device -- and on expiry the chain
        // is marked failed instead of continuing from a stale slot
        const int limit = A.dbg_handoff ? (1 << 16) : (1 << 24);
        int spins = 0;
        while (__hip_atomic_load(hflag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < need) {
          __builtin_amdgcn_s_sleep(2);
          if (++spins > limit) {
            dead = true;
            break;
          }
        }
      }
      if (!dead) {
        gtile::lds_fence();
        x = slot[lane];
        bF = slot[64 + lane];
        bM = slot[128 + lane];
        fail = (int)slot[192];
        dead = fail < 0;
      }
    }
    if (dead) sw_b = sw_a;
    // record pointers of this lane, advanced by one sweep's rows per iteration: x rows of every
    // system; b rows of every system, or of the first brec_nc chains of each pulsar, compact
    double* xrp = (A.x_rec && act && !(lane & 1)) ? A.x_rec + sw_a * xr_step + sys * NFR + kf : nullptr;
    const bool brec = A.b_rec && (A.brec_nc == 0 || c < A.brec_nc);
    const int64_t brow0 = A.brec_nc == 0 ? sys : (int64_t)p * A.brec_nc + c;
    double* bFp = (brec && act) ? A.b_rec + sw_a * br_step + brow0 * A.ldb + fi : nullptr;
    double* bMp = (brec && actm) ? A.b_rec + sw_a * br_step + brow0 * A.ldb + mi : nullptr;
  // Merged RNG (production draws: nothing injected): ONE Philox block per lane per sweep feeds both
  // the rho|b uniforms and the b|rho normals.  Lane l < npair turns its two 53-bit uniforms into the
  // Box-Muller pair (normals 2l, 2l+1 of [z_F | z_M]); lane npair + j lends its two uniforms to
  // frequencies 2j, 2j+1 of the rho draw; the values reach their consumer lanes through the LDS
  // crossbar (ds_bpermute, no VALU).  One Philox pass per sweep instead of two (the separate rho
  // uniforms cost 2.0 % of the headline launch, profiles/r05b); falls back to the two-block scheme
  // when the lanes do not suffice (NF + nM + NF / 2 > 128).
  const int npair = (NF + nM + 1) >> 1;
  const bool mrg = GS_RNG_MERGE && !A.u_inj && !A.z_inj && npair + ((NFR + 1) >> 1) <= 64;
#pragma unroll 1
  for (int sw = sw_a; sw < sw_b; ++sw) {
    const long long ii = A.it0 + sw;
    const int64_t rec = (int64_t)sw * n_sys + sys;
    GS_PH_BEGIN
    // record-before-update (pulsar_gibbs.py:658-659)
    if (xrp) *xrp = x;
    if (bFp) *bFp = bF;
    if (bMp) *bMp = bM;
    xrp = xrp ? xrp + xr_step : nullptr;
    bFp = bFp ? bFp + br_step : nullptr;
    bMp = bMp ? bMp + br_step : nullptr;
    // pass 0: first b draw from xs at global sweep 0 (pulsar_gibbs.py:661-662);
    // pass 1: rho|b then the gated b draw.  One bdraw_wave call site.
#pragma unroll 1
    for (int pass = (ii == 0) ? 0 : 1; pass < 2; ++pass) {
      const double* zinj = A.z0_inj;
      int ev = GS_EV_B0;
      double phinv = 0.0;
      int64_t zrow = sys;
      if (pass == 1) {
        if constexpr (GS_RHO_PRIO > 0) __builtin_amdgcn_s_setprio(GS_RHO_PRIO);
        // rho|b analytic (pulsar_gibbs.py:208-216, 236)
        const double partner = __shfl_xor(bF, 1);
        const double be = (lane & 1) ? partner : bF, bo = (lane & 1) ? bF : partner;
        // tau = (b_sin^2 + b_cos^2) / 2 rounded as numpy (pulsar_gibbs.py:208-209): no fma contraction
        const double tau = gs_add_rn(gs_mul_rn(be, be), gs_mul_rn(bo, bo)) / 2;
        double U;
        if (A.u_inj) {
          U = act ? A.u_inj[rec * NFR + kf] : 0.5;
        } else if (mrg) {
          double mu1, mu2;
          gs_uniform2(gs_counter(lane, ii, gchain, p + A.psr_base, GS_EV_B), A.key, mu1, mu2);
          const int src = npair + (kf >> 1);
          const double ua = gtile::bcast_lane_bp(mu1, src), ub = gtile::bcast_lane_bp(mu2, src);
          U = (kf & 1) ? ub : ua;
          // the pair waits for Box-Muller in the wave's save slot (free until the draw), not in
          // 4 VGPRs across the rho step (26 spilled VGPRs that way)
          bsave[lane] = mu1;
          bsave[64 + lane] = mu2;
        } else {
          double u2;
#ifdef GS_PROBE_NO_RHO_PHILOX  // cost attribution only (wrong draws): the rho uniform without Philox
          U = 0.25 + 0.5 * __builtin_amdgcn_fract(tau * 1e3);
          (void)u2;
#else
          gs_uniform2(gs_counter(kf, ii, gchain, p + A.psr_base, GS_EV_RHO), A.key, U, u2);
#endif
        }
#if GS_FAST_MATH
        // the reference's expressions with its divisions by the prior bounds as products with
        // their reciprocals, tau / den and den / tau by v_rcp_f64 + two Newton steps, and
        // the short log (gibbs_common.h): ~2 ulp per value, ~150 fewer VALU per draw
        const double t1 = tau * irhomax;
        const double arg = t1 - tau * irhomin;
#else
        const double t1 = tau / rhomax;
        const double arg = t1 - (tau / rhomin);
#endif
        // 1 - exp(arg) rounds to exactly 1 for arg < -37.5: skip the exp when every
        // lane is there (the usual case, tau >> rhomin)
        double hi = 1.0;
#if GS_FAST_MATH && GS_RHO_EXP
        if (__ballot(act && !(arg < -40.0))) hi = 1 - gs_exp_neg(arg);  // arg <= 0 (rhomin < rhomax)
#else
        if (__ballot(act && !(arg < -40.0))) hi = 1 - exp(arg);
#endif
        const double eta = 0.0 + hi * U;
#if GS_FAST_MATH
#ifdef GS_PROBE_NO_RHO_LOG  // cost attribution only (wrong draws)
        const double den = t1 + eta;
#else
        const double den = t1 - gs_log_pos(1 - eta);
#endif
        const double rho = tau * rcp_nr2(den);
        const double xnew = act ? gs_log_pos(rho) * 0x1.bcb7b1526e50ep-3 : 0.0;  // 0.5 log10 rho
        // phiinv = 1/rho = den / tau
        phinv = act ? den * rcp_nr2(tau) : 0.0;
#else
        const double den = t1 - log(1 - eta);
        const double rho = tau / den;
        const double xnew = act ? 0.5 * log10(rho) : 0.0;
        // phiinv of the new rho: 1/rho (rcp + two Newton steps) instead of the
        // reference's 1/10**(2 x) round trip through log10 (equal to a few ulp)
        phinv = act ? rcp_nr2(rho) : 0.0;
#endif
        // gate: all(xnew != x_old[-1])  (pulsar_gibbs.py:697)
        const double xlast = rdlane(x, NF - 1);
        const bool same = act && (xnew == xlast);
        const bool gate = __ballot(same) == 0ull;
        x = xnew;
        if constexpr (GS_RHO_PRIO > 0) __builtin_amdgcn_s_setprio(GS_BASE_PRIO);
        if (!gate) break;
        zinj = A.z_inj;
        ev = GS_EV_B;
        zrow = rec;
      }
      GS_PH(6)
      double zF, zM;
      if (zinj) {
        zF = act ? zinj[zrow * A.ldb + fi] : 0.0;
        zM = actm ? zinj[zrow * A.ldb + mi] : 0.0;
      } else {
#ifdef GS_PROBE_NO_NORMALS  // cost attribution only (wrong draws): no Philox + Box-Muller pass
        zF = __builtin_amdgcn_fract(x * 7.0) - 0.5;
        zM = __builtin_amdgcn_fract(x * 3.0) - 0.5;
#else
        if (mrg && pass == 1) {
          // normal j of [z_F | z_M] is component j & 1 of lane j >> 1's pair
          double n1, n2;
          gtile::lds_fence();
          gs_box_muller(bsave[lane], bsave[64 + lane], n1, n2);
          gtile::lds_fence();
          const int sf = lane >> 1, sm = (NF + lane) >> 1;
          const double f1 = gtile::bcast_lane_bp(n1, sf), f2 = gtile::bcast_lane_bp(n2, sf);
          const double m1 = gtile::bcast_lane_bp(n1, sm), m2 = gtile::bcast_lane_bp(n2, sm);
          zF = (lane & 1) ? f2 : f1;
          zM = ((NF + lane) & 1) ? m2 : m1;
        } else {
          gs_normal2(gs_counter(lane, ii, gchain, p + A.psr_base, ev), A.key, zF, zM);
        }
#endif
      }
      if (pass == 0) phinv = act ? 1.0 / pow(10.0, 2.0 * x) : 0.0;  // first draw from xs
      GS_PH(7)
      // a failed factorisation (non-PD Sigma, wave-uniform) keeps the previous b: no NaN ever
      // enters the state (the reference's LinAlgError branch, pulsar_gibbs.py:507-516).  The
      // previous b waits in the wave's LDS save slot, not in 4 VGPRs across the draw.
      bsave[lane] = bF;
      bsave[64 + lane] = bM;
      const int f = bdraw_sys<NFC, NTC, BC, true>(M, NMXe, nM, lane, phinv, zF, zM, bF, bM, scr, NF);
      if (f) {
        gtile::lds_fence();
        bF = bsave[lane];
        bM = bsave[64 + lane];
        if (!fail) fail = f;
        if (A.fail_count && lane == 0) A.fail_count[sys] += 1;
      }
    }
  }
    if (dst == 0) {
      if (!dead) {
        if (act && !(lane & 1)) A.x_state[sys * NFR + kf] = x;
        if (act) A.b_state[sys * A.ldb + fi] = bF;
        if (actm) A.b_state[sys * A.ldb + mi] = bM;
      }
      if (A.info && lane == 0) A.info[sys] = dead ? -1 : fail;
    } else {
      double* slot = dst == 1 ? park : hand;
      gtile::lds_fence();
      slot[lane] = x;
      slot[64 + lane] = bF;
      slot[128 + lane] = bM;
      if (lane == 0) slot[192] = dead ? -1.0 : (double)fail;
      gtile::lds_fence();
      // (GS_OPT_DEBUG_HANDOFF: workgroup 0's first trio never publishes its first third, so the
      // test sees the wait expire)
      const bool skip = A.dbg_handoff && blockIdx.x == 0 && wave == 0;
      if (dst == 2 && !skip) __hip_atomic_store(hflag, t + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  GS_PH_FLUSH(scr)
}

template <int NFC, int NTC, int WPB, int BC>
__global__ __launch_bounds__(64 * WPB, GS_MINW(BC, NFC, NTC)) void k_sweep_freespec(SweepArgs A) {
  sweep_freespec_body<NFC, NTC, WPB, BC, true>(A);
}
template <int NFC, int NTC, int WPB, int BC>
__global__ __launch_bounds__(64 * WPB, GS_MINW(BC, NFC, NTC)) void k_sweep_freespec_rm(SweepArgs A) {
  sweep_freespec_body<NFC, NTC, WPB, BC, false>(A);
}

// ------------------------------------------------------------ fused sweep, two chains per wave
// GS_OPT_SWEEP_SCHED = 3 (and the cost model's choice where it applies, launch_sweep_freespec): the
// same sweep as sweep_freespec_body for NF = 60 on the tiled model block (nm <= 16) with device Philox,
// each wavefront running chains c, c + 1 side by side and drawing their b together
// (gibbs_tile2.h bdraw_tile_pair60).  Every draw, uniform and record is the one-chain kernel's bit for
// bit: the Philox counters are per chain, a chain whose gate is shut has its (computed) draw discarded
// exactly where the one-chain kernel skips it, and a failed factorisation keeps that chain's b.
// 2 waves per SIMD (both chains' tiles: ~200 VGPRs): 4096 chains are 2048 waves, one round.
constexpr int GS_PAIR_SCR = 2 * gs_tile_scr(60) + 256 + 128 + 128;
// GS_PAIR_WPB: waves (chain pairs) per workgroup
#ifndef GS_PAIR_WPB
#define GS_PAIR_WPB 4
#endif
// GS_PAIR_RHO_PRIO: issue priority of the pair kernel's rho step (the one-chain kernels: GS_RHO_PRIO = 0).
// Measured on the headline (r06x, 4 interleaved reps): 1.915-1.927 ms per launch at 1 against
// 1.928-1.938 at 0 and 1.931-1.943 at 2
#ifndef GS_PAIR_RHO_PRIO
#define GS_PAIR_RHO_PRIO 1
#endif
// GS_PAIR_RHO_MERGE: both chains' rho steps in one pass over the wave (30 frequencies each)
#ifndef GS_PAIR_RHO_MERGE
#define GS_PAIR_RHO_MERGE 1
#endif  // per wave: 2 scratches, b save, z_M, x park

template <int WPB>
__global__ __launch_bounds__(64 * WPB, 2) void k_sweep_pair(SweepArgs A) {
  extern __shared__ double lds[];
  constexpr int NF = 60, NFR = 30;
  const int wave = gs_wave_id(), lane = threadIdx.x & 63;
  constexpr int CPB = 2 * WPB;
  const int nb = (A.n_chain + CPB - 1) / CPB;
  const int p = blockIdx.x / nb;
  const int cA = (blockIdx.x % nb) * CPB + 2 * wave;  // chains cA, cA + 1 (n_chain is even)
  const int nM = __builtin_amdgcn_readfirstlane(A.nm[p]);
  stage_model_tiled(lds, A.model + (int64_t)p * A.mstride, NF, A.NMX, nM);
  const int64_t mlds = model_tiled_doubles(NF, A.NMX);
  if (cA >= A.n_chain) return;
  int NMXe = A.NMX;
  const ModelTiled M = model_tiled_view_psr<true>(lds, NF, A.NMX, nM, NMXe);
  const int64_t n_sys = (int64_t)A.n_psr * A.n_chain;
  const bool act = lane < NF, actm = lane < nM;
  const int kf = act ? (lane >> 1) : 0;
  const int fi = act ? A.fidx[p * NF + lane] : 0;
  const int mi = actm ? A.midx[p * A.NMX + lane] : 0;
  double* wl = lds + mlds + (int64_t)wave * GS_PAIR_SCR;
  double* const scr[2] = {wl, wl + gs_tile_scr(60)};
  double* bsave = wl + 2 * gs_tile_scr(60);  // [2][128]: the chains' previous b (failed or shut draws)
  double* zmslot = bsave + 256;              // [2][64]: the chains' z_M during the draw
  double* xpark = zmslot + 128;              // [2][64]: the chains' x during the draw (not in VGPRs)

  const double irhomin = 1.0 / A.rhomin, irhomax = 1.0 / A.rhomax;
  const int64_t xr_step = n_sys * NFR;
  const int64_t br_step = (A.brec_nc == 0 ? n_sys : (int64_t)A.n_psr * A.brec_nc) * A.ldb;
  const int S = A.n_sweeps;
  int64_t sys[2];
  long long gchain[2];
  double x[2], bF[2], bM[2];
  int fail[2] = {0, 0};
  // record targets: per-lane 32/64-bit offsets from the uniform record bases (-1: this lane records
  // nothing), advanced by one sweep's rows per iteration
  int xro[2], bFo[2], bMo[2];
#pragma unroll
  for (int ch = 0; ch < 2; ++ch) {
    const int c = cA + ch;
    sys[ch] = (int64_t)p * A.n_chain + c;
    gchain[ch] = A.chain_base + c;
    x[ch] = act ? A.x_state[sys[ch] * NFR + kf] : 0.0;
    bF[ch] = act ? A.b_state[sys[ch] * A.ldb + fi] : 0.0;
    bM[ch] = actm ? A.b_state[sys[ch] * A.ldb + mi] : 0.0;
    xro[ch] = (A.x_rec && act && !(lane & 1)) ? (int)(sys[ch] * NFR + kf) : -1;
    const bool brec = A.b_rec && (A.brec_nc == 0 || c < A.brec_nc);
    const int64_t brow0 = A.brec_nc == 0 ? sys[ch] : (int64_t)p * A.brec_nc + c;
    bFo[ch] = (brec && act) ? (int)(brow0 * A.ldb + fi) : -1;
    bMo[ch] = (brec && actm) ? (int)(brow0 * A.ldb + mi) : -1;
  }
#pragma unroll 1
  for (int sw = 0; sw < S; ++sw) {
    const long long ii = A.it0 + sw;
#pragma unroll
    for (int ch = 0; ch < 2; ++ch) {  // record-before-update (pulsar_gibbs.py:658-659)
      if (xro[ch] >= 0) A.x_rec[sw * xr_step + xro[ch]] = x[ch];
      if (bFo[ch] >= 0) A.b_rec[sw * br_step + bFo[ch]] = bF[ch];
      if (bMo[ch] >= 0) A.b_rec[sw * br_step + bMo[ch]] = bM[ch];
    }
#pragma unroll 1
    for (int pass = (ii == 0) ? 0 : 1; pass < 2; ++pass) {
      int ev = GS_EV_B0;
      double phinv[2] = {0.0, 0.0};
      bool draw[2] = {true, true};
      if (pass == 1) {
        if constexpr (GS_PAIR_RHO_PRIO > 0) __builtin_amdgcn_s_setprio(GS_PAIR_RHO_PRIO);
#if GS_PAIR_RHO_MERGE
        {
          // rho|b analytic (pulsar_gibbs.py:208-216, 236), as sweep_freespec_body, for both chains in
          // one pass: lane 32 h + k computes frequency k of chain h (the one-chain layout has each
          // frequency on two lanes), same operations and Philox counter per (chain, k)
          const int h = lane >> 5, k = lane & 31;
          const bool am = k < NFR;
          double tau2[2];
#pragma unroll
          for (int ch = 0; ch < 2; ++ch) {
            const double partner = __shfl_xor(bF[ch], 1);
            const double be = (lane & 1) ? partner : bF[ch], bo = (lane & 1) ? bF[ch] : partner;
            tau2[ch] = gs_add_rn(gs_mul_rn(be, be), gs_mul_rn(bo, bo)) / 2;
          }
          const int src = am ? 2 * k : 0;
          const double ta = gtile::bcast_lane_bp(tau2[0], src), tb = gtile::bcast_lane_bp(tau2[1], src);
          const double tau = h ? tb : ta;
          double U, u2;
          gs_uniform2(gs_counter(k, ii, h ? gchain[1] : gchain[0], p + A.psr_base, GS_EV_RHO), A.key, U, u2);
#if GS_FAST_MATH
          const double t1 = tau * irhomax;
          const double arg = t1 - tau * irhomin;
#else
          const double t1 = tau / A.rhomax;
          const double arg = t1 - (tau / A.rhomin);
#endif
          // (1 - exp(arg) is exactly 1 where the skip applies, so one ballot over both chains draws
          // the same values as a ballot per chain)
          double hi = 1.0;
#if GS_FAST_MATH && GS_RHO_EXP
          if (__ballot(am && !(arg < -40.0))) hi = 1 - gs_exp_neg(arg);
#else
          if (__ballot(am && !(arg < -40.0))) hi = 1 - exp(arg);
#endif
          const double eta = 0.0 + hi * U;
#if GS_FAST_MATH
          const double den = t1 - gs_log_pos(1 - eta);
          const double rho = tau * rcp_nr2(den);
          const double xnew = am ? gs_log_pos(rho) * 0x1.bcb7b1526e50ep-3 : 0.0;
          const double phm = am ? den * rcp_nr2(tau) : 0.0;
#else
          const double den = t1 - log(1 - eta);
          const double rho = tau / den;
          const double xnew = am ? 0.5 * log10(rho) : 0.0;
          const double phm = am ? rcp_nr2(rho) : 0.0;
#endif
          // gate: all(xnew != x_old[-1])  (pulsar_gibbs.py:697), per chain
          const double xl0 = rdlane(x[0], NF - 1), xl1 = rdlane(x[1], NF - 1);
          const unsigned long long same = __ballot(am && (xnew == (h ? xl1 : xl0)));
          draw[0] = (same & 0xffffffffull) == 0ull;
          draw[1] = (same >> 32) == 0ull;
          // back to the one-chain layout: lane l of chain ch holds frequency l >> 1
#pragma unroll
          for (int ch = 0; ch < 2; ++ch) {
            const int from = 32 * ch + (act ? (lane >> 1) : 0);
            const double xv = gtile::bcast_lane_bp(xnew, from), pv = gtile::bcast_lane_bp(phm, from);
            x[ch] = act ? xv : 0.0;
            phinv[ch] = act ? pv : 0.0;
          }
        }
#else
#pragma unroll
        for (int ch = 0; ch < 2; ++ch) {
          // rho|b analytic (pulsar_gibbs.py:208-216, 236), as sweep_freespec_body
          const double partner = __shfl_xor(bF[ch], 1);
          const double be = (lane & 1) ? partner : bF[ch], bo = (lane & 1) ? bF[ch] : partner;
          const double tau = gs_add_rn(gs_mul_rn(be, be), gs_mul_rn(bo, bo)) / 2;
          double U, u2;
          gs_uniform2(gs_counter(kf, ii, gchain[ch], p + A.psr_base, GS_EV_RHO), A.key, U, u2);
#if GS_FAST_MATH
          const double t1 = tau * irhomax;
          const double arg = t1 - tau * irhomin;
#else
          const double t1 = tau / A.rhomax;
          const double arg = t1 - (tau / A.rhomin);
#endif
          double hi = 1.0;
#if GS_FAST_MATH && GS_RHO_EXP
          if (__ballot(act && !(arg < -40.0))) hi = 1 - gs_exp_neg(arg);
#else
          if (__ballot(act && !(arg < -40.0))) hi = 1 - exp(arg);
#endif
          const double eta = 0.0 + hi * U;
#if GS_FAST_MATH
          const double den = t1 - gs_log_pos(1 - eta);
          const double rho = tau * rcp_nr2(den);
          const double xnew = act ? gs_log_pos(rho) * 0x1.bcb7b1526e50ep-3 : 0.0;
          phinv[ch] = act ? den * rcp_nr2(tau) : 0.0;
#else
          const double den = t1 - log(1 - eta);
          const double rho = tau / den;
          const double xnew = act ? 0.5 * log10(rho) : 0.0;
          phinv[ch] = act ? rcp_nr2(rho) : 0.0;
#endif
          // gate: all(xnew != x_old[-1])  (pulsar_gibbs.py:697)
          const double xlast = rdlane(x[ch], NF - 1);
          draw[ch] = __ballot(act && (xnew == xlast)) == 0ull;
          x[ch] = xnew;
        }
#endif
        if constexpr (GS_PAIR_RHO_PRIO > 0) __builtin_amdgcn_s_setprio(GS_BASE_PRIO);
        if (!draw[0] && !draw[1]) break;
        ev = GS_EV_B;
      }
      double zF[2], zM[2];
#pragma unroll
      for (int ch = 0; ch < 2; ++ch) {
#ifdef GS_PROBE_NO_NORMALS  // cost attribution only (wrong draws): no Philox + Box-Muller pass
        zF[ch] = __builtin_amdgcn_fract(x[ch] * 7.0) - 0.5;
        zM[ch] = __builtin_amdgcn_fract(x[ch] * 3.0) - 0.5;
#else
        gs_normal2(gs_counter(lane, ii, gchain[ch], p + A.psr_base, ev), A.key, zF[ch], zM[ch]);
#endif
        if (pass == 0) phinv[ch] = act ? 1.0 / pow(10.0, 2.0 * x[ch]) : 0.0;  // first draw from xs
        // the previous b waits in the wave's save slot (a failed or shut draw keeps it)
        bsave[128 * ch + lane] = bF[ch];
        bsave[128 * ch + 64 + lane] = bM[ch];
        xpark[64 * ch + lane] = x[ch];
      }
      int f[2];
      bdraw_tile_pair60<true>(M, NMXe, nM, lane, phinv, zF, zM, bF, bM, scr, zmslot, f);
      gtile::lds_fence();
#pragma unroll
      for (int ch = 0; ch < 2; ++ch) {
        x[ch] = xpark[64 * ch + lane];
        const bool keep = !draw[ch] || f[ch];
        if (keep) {
          gtile::lds_fence();
          bF[ch] = bsave[128 * ch + lane];
          bM[ch] = bsave[128 * ch + 64 + lane];
        }
        if (draw[ch] && f[ch]) {
          if (!fail[ch]) fail[ch] = f[ch];
          if (A.fail_count && lane == 0) A.fail_count[sys[ch]] += 1;
        }
      }
    }
  }
#pragma unroll
  for (int ch = 0; ch < 2; ++ch) {
    if (act && !(lane & 1)) A.x_state[sys[ch] * NFR + kf] = x[ch];
    if (act) A.b_state[sys[ch] * A.ldb + fi] = bF[ch];
    if (actm) A.b_state[sys[ch] * A.ldb + mi] = bM[ch];
    if (A.info && lane == 0) A.info[sys[ch]] = fail[ch];
  }
}

// ------------------------------------------------------------ rho|b analytic
__global__ void k_rho_analytic(RhoArgs A) {
  const int64_t n_sys = (int64_t)A.n_psr * A.n_chain;
  const int NFR = A.NF / 2;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_sys * NFR) return;
  const int64_t sys = t / NFR;
  const int k = (int)(t % NFR);
  const int p = (int)(sys / A.n_chain), c = (int)(sys % A.n_chain);
  const double bs = A.b[sys * A.ldb + A.fidx[p * A.NF + 2 * k]];
  const double bc = A.b[sys * A.ldb + A.fidx[p * A.NF + 2 * k + 1]];
  const double tau = gs_add_rn(gs_mul_rn(bs, bs), gs_mul_rn(bc, bc)) / 2;  // numpy's rounding
  double U;
  if (A.u) {
    U = A.u[sys * NFR + k];
  } else {
    double u2;
    gs_uniform2(gs_counter(k, gs_sweep(A.sweep, A.sweep_dev), A.chain_base + c, p + A.psr_base, GS_EV_RHO), A.key, U, u2);
  }
  const double hi = 1 - exp((tau / A.rhomax) - (tau / A.rhomin));
  const double eta = 0.0 + hi * U;
  const double rho = tau / ((tau / A.rhomax) - log(1 - eta));
  A.x[sys * A.ldx + k] = 0.5 * log10(rho);
}

#ifdef GS_PHASE_PROF
extern "C" int gs_debug_phase_cycles(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(gs_phase_cyc), sizeof(unsigned long long) * 8) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(gs_phase_cyc), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

// Fixed NF in {20, 40, 60}: every broadcast variant; any other even NF <= 64: the tile
// variant with NF at run time, one instantiation per tile count NT = NF / 16 + 1.
// dynamic LDS above 64 KB (nm up to 64: model blocks up to 95 KB) needs the kernel attribute
template <typename K>
int set_lds(K kernel, size_t lds) {
  return hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
         hipSuccess;
}
#define GS_LAUNCH(KERNEL, NFC, NTC, BC, ARGS)                                              \
  if (lds > 65536 && set_lds(KERNEL<NFC, NTC, WPB, BC>, lds)) return 2;                     \
  hipLaunchKernelGGL((KERNEL<NFC, NTC, WPB, BC>), grid, dim3(64 * WPB), lds, s, ARGS);     \
  return 0;
#define GS_NF_CASES(KERNEL, ARGS)                                                       \
  switch (NF * 4 + bc) {                                                                \
    case 80: GS_LAUNCH(KERNEL, 20, 0, 0, ARGS)                                          \
    case 81: GS_LAUNCH(KERNEL, 20, 0, 1, ARGS)                                          \
    case 82: GS_LAUNCH(KERNEL, 20, 0, 2, ARGS)                                          \
    case 83: GS_LAUNCH(KERNEL, 20, 0, 3, ARGS)                                          \
    case 160: GS_LAUNCH(KERNEL, 40, 0, 0, ARGS)                                         \
    case 161: GS_LAUNCH(KERNEL, 40, 0, 1, ARGS)                                         \
    case 162: GS_LAUNCH(KERNEL, 40, 0, 2, ARGS)                                         \
    case 163: GS_LAUNCH(KERNEL, 40, 0, 3, ARGS)                                         \
    case 240: GS_LAUNCH(KERNEL, 60, 0, 0, ARGS)                                         \
    case 241: GS_LAUNCH(KERNEL, 60, 0, 1, ARGS)                                         \
    case 242: GS_LAUNCH(KERNEL, 60, 0, 2, ARGS)                                         \
    case 243: GS_LAUNCH(KERNEL, 60, 0, 3, ARGS)                                         \
    default: break;                                                                     \
  }                                                                                     \
  if (NF <= 0 || NF > 64 || (NF & 1)) return 1;                                         \
  switch (NF / 16 + 1) {                                                                \
    case 1: GS_LAUNCH(KERNEL, 0, 1, 3, ARGS)                                            \
    case 2: GS_LAUNCH(KERNEL, 0, 2, 3, ARGS)                                            \
    case 3: GS_LAUNCH(KERNEL, 0, 3, 3, ARGS)                                            \
    case 4: GS_LAUNCH(KERNEL, 0, 4, 3, ARGS)                                            \
    default: GS_LAUNCH(KERNEL, 0, 5, 3, ARGS)                                           \
  }

template <int WPB>
int dispatch_nf_sweep(int NF, int bc, dim3 grid, size_t lds, hipStream_t s, const SweepArgs& a) {
  if (model_tiled_fix(a.NMX)) {
    GS_NF_CASES(k_sweep_freespec, a)
  } else {
    GS_NF_CASES(k_sweep_freespec_rm, a)
  }
}

template <int WPB>
int dispatch_nf_bdraw(int NF, int bc, dim3 grid, size_t lds, hipStream_t s, const BdrawArgs& a) {
  GS_NF_CASES(k_bdraw, a)
}

}  // namespace

int launch_lnlike_marg(hipStream_t s, const LnlArgs& a) {
  constexpr int WPB = GS_SWEEP_WPB;
  const int nb = (a.n_chain + WPB - 1) / WPB;
  const bool in_lds = !a.model_per_sys && !a.model_global;
  dim3 grid((unsigned)(a.n_psr * (in_lds ? (nb + GS_BDRAW_LOOP - 1) / GS_BDRAW_LOOP : nb)));
  const size_t lds = ((size_t)(a.model_per_sys || a.model_global ? 0 : a.mstride) + gs_tile_scr(a.NF) * WPB) *
                     sizeof(double);
  // a shared model block staged in LDS: above 64 KB (e.g. NF = 60 with NMX > 31) the launch needs
  // the dynamic-LDS attribute, as GS_LAUNCH sets it
#define GS_LNL_LAUNCH(NFC, NTC)                                                       \
  if (lds > 65536 && set_lds(k_lnlike_marg<NFC, NTC, WPB>, lds)) return 2;            \
  hipLaunchKernelGGL((k_lnlike_marg<NFC, NTC, WPB>), grid, dim3(64 * WPB), lds, s, a); \
  return 0;
  switch (a.NF) {
    case 20: GS_LNL_LAUNCH(20, 0)
    case 40: GS_LNL_LAUNCH(40, 0)
    case 60: GS_LNL_LAUNCH(60, 0)
    default: break;
  }
  if (a.NF <= 0 || a.NF > 64 || (a.NF & 1)) return 1;
  switch (a.NF / 16 + 1) {
    case 1: GS_LNL_LAUNCH(0, 1)
    case 2: GS_LNL_LAUNCH(0, 2)
    case 3: GS_LNL_LAUNCH(0, 3)
    case 4: GS_LNL_LAUNCH(0, 4)
    default: GS_LNL_LAUNCH(0, 5)
  }
#undef GS_LNL_LAUNCH
}

int launch_hyper_mh(hipStream_t s, const HyperMhArgs& a) {
  if (a.n_chain == 0) return 0;
  // x row, lnL_p, the 64-step proposal table, each wave's tile scratch
  const size_t lds = ((size_t)((a.ldx + a.n_psr + 1) & ~1) + 4 * 64 + GS_HY_W * gs_tile_scr(a.NF)) * sizeof(double);
  dim3 grid((unsigned)a.n_chain);
#define GS_HY_LAUNCH(NFC, NTC)                                                   \
  if (lds > 65536 && set_lds(k_hyper_mh<NFC, NTC>, lds)) return 2;               \
  hipLaunchKernelGGL((k_hyper_mh<NFC, NTC>), grid, dim3(64 * GS_HY_W), lds, s, a); \
  return 0;
  switch (a.NF) {
    case 20: GS_HY_LAUNCH(20, 0)
    case 40: GS_HY_LAUNCH(40, 0)
    case 60: GS_HY_LAUNCH(60, 0)
    default: break;
  }
  if (a.NF <= 0 || a.NF > 64 || (a.NF & 1)) return 1;
  switch (a.NF / 16 + 1) {
    case 1: GS_HY_LAUNCH(0, 1)
    case 2: GS_HY_LAUNCH(0, 2)
    case 3: GS_HY_LAUNCH(0, 3)
    case 4: GS_HY_LAUNCH(0, 4)
    default: GS_HY_LAUNCH(0, 5)
  }
#undef GS_HY_LAUNCH
}

// Workgroup shape of the tile-variant sweep (GS_OPT_SWEEP_SCHED 0: this cost model).  In units
// of one full round R (3 waves on each SIMD for the launch's sweeps; measured on MI355X, NF = 60,
// r03n/r03q): 4-wave workgroups take floor(q/3) R + g(q mod 3) with q = waves per SIMD and a
// part-filled last round of 1 / 2 waves per SIMD costing g = 0.46 / 0.74 R (latency-bound); the
// 12-wave hand-off workgroups (4/3 chains per wave) take ceil(workgroups / CUs) x 4/3 R whatever
// the last round's fill.  4096 chains: 1.46 R vs 1.33 R (2.232 vs 2.072 ms); 3072: 1 R vs 1.33 R;
// configs[2] (45 x 256): 3.74 R vs 4 R.
static int device_cus() {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
      ncu = 256;
  }
  return ncu;
}
// Largest dynamic LDS a workgroup may request (hipFuncSetAttribute opt-in limit; 160 KB on gfx950).
static size_t device_lds_optin() {
  static int lim = 0;
  if (!lim) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&lim, hipDeviceAttributeSharedMemPerBlockOptin, dev) != hipSuccess || lim <= 0)
      lim = 160 * 1024;
  }
  return (size_t)lim;
}
static bool sweep_handoff_wins(const SweepArgs& a) {
  if (a.sched) return a.sched == 1;
  const double ncu = device_cus();
  const double q = (double)a.n_psr * a.n_chain / (4.0 * ncu);
  const double k = std::floor(q / 3.0), r = q - 3.0 * k;
  const double g = r <= 0.0 ? 0.0 : r <= 1.0 ? 0.46 * r : r <= 2.0 ? 0.46 + 0.28 * (r - 1.0) : 0.74 + 0.26 * (r - 2.0);
  const double wg = (double)a.n_psr * ((a.n_chain + 15) / 16);
  const double c12 = std::ceil(wg / ncu) * (4.0 / 3.0);
  return c12 < 0.97 * (k + g);
}
// Two chains per wave (k_sweep_pair) against the one-chain shapes, in the same unit R.  Its waves run
// 2 per SIMD: a full round (8 waves per CU, 16 chains) takes P = 1.27 R and a last round of at most one
// wave per SIMD 0.70 P (r06l, 1 GPU: 4096 chains 1.965 ms = P, 8192 3.905 ms, 2048 and 1024 chains
// 1.37-1.38 ms; R = 1.55 ms from the 4096-chain one-chain / hand-off times above).  4096 chains: 1.27 R
// vs 1.33 R (hand-off); 8192: 2.54 R vs 2.67 R; 6144: 2.16 R vs 2 R; 2048: 0.89 R vs 0.74 R.
static bool sweep_pair_wins(const SweepArgs& a) {
  if (a.sched) return a.sched == 3;
  const double ncu = device_cus();
  const double q = (double)a.n_psr * a.n_chain / (4.0 * ncu);
  const double k = std::floor(q / 3.0), r = q - 3.0 * k;
  const double g = r <= 0.0 ? 0.0 : r <= 1.0 ? 0.46 * r : r <= 2.0 ? 0.46 + 0.28 * (r - 1.0) : 0.74 + 0.26 * (r - 2.0);
  const double wg = (double)a.n_psr * ((a.n_chain + 15) / 16);
  const double one = std::min(k + g, std::ceil(wg / ncu) * (4.0 / 3.0));
  const double w = (double)a.n_psr * (a.n_chain / 2) / (4.0 * ncu);  // pair waves per SIMD
  const double kp = std::floor(w / 2.0), rp = w - 2.0 * kp;
  const double pair = 1.27 * (kp + (rp <= 0.0 ? 0.0 : rp <= 1.0 ? 0.70 : 1.0));
  return pair < 0.97 * one;
}
int launch_sweep_freespec(hipStream_t s, const SweepArgs& a, int* shape) {
  const bool fixed = a.NF == 20 || a.NF == 40 || a.NF == 60;
  const bool tiled = GS_SWEEP_TILED && (!fixed || a.bcast == GS_BCAST_TILE);
  const size_t mlds = tiled ? (size_t)model_tiled_doubles(a.NF, a.NMX) : (size_t)a.mstride;
  // two chains per wave (k_sweep_pair): NF = 60 on the tiled block with a tiled fixed part, device
  // Philox (no injected draws), an even chain count
  const bool pair_ok = a.NF == 60 && tiled && model_tiled_fix(a.NMX) && !a.z0_inj && !a.z_inj && !a.u_inj &&
                       (a.n_chain % 2) == 0 && !a.dbg_handoff;
  if (pair_ok && sweep_pair_wins(a)) {
    constexpr int WPB = GS_PAIR_WPB;
    const size_t lds = (mlds + (size_t)WPB * GS_PAIR_SCR) * sizeof(double);
    if (lds <= device_lds_optin()) {
      const int nb = (a.n_chain + 2 * WPB - 1) / (2 * WPB);
      if (lds > 65536 && set_lds(k_sweep_pair<WPB>, lds)) return 2;
      hipLaunchKernelGGL((k_sweep_pair<WPB>), dim3((unsigned)(a.n_psr * nb)), dim3(64 * WPB), lds, s, a);
      *shape = 3;
      return 0;
    }
  }
  // the 12-wave hand-off shape holds 12 waves' scratch, save and park slots beside the model
  // block: at large NF x NMX (e.g. NF = 60, NMX = 64: 168 KB) it does not fit, and the 4-wave
  // shape (~102 KB there) runs instead, whatever the cost model or GS_OPT_SWEEP_SCHED say
  const size_t lds12 = (mlds + (size_t)12 * (gs_tile_scr(a.NF) + 128 + 256) + 4 * 256 + 2) * sizeof(double);
  if (tiled && lds12 <= device_lds_optin() && sweep_handoff_wins(a)) {
    const int nb = (a.n_chain + 15) / 16;
    dim3 grid((unsigned)(a.n_psr * nb));
    *shape = 1;
    return dispatch_nf_sweep<12>(a.NF, a.bcast, grid, lds12, s, a);
  }
  const int nb = (a.n_chain + GS_SWEEP_WPB - 1) / GS_SWEEP_WPB;
  dim3 grid((unsigned)(a.n_psr * nb));
  const size_t lds =
      (mlds + ((fixed ? GS_SCR_DOUBLES(a.bcast, a.NF) : gs_tile_scr(a.NF)) + 128) * GS_SWEEP_WPB) * sizeof(double);
  *shape = 2;
  return dispatch_nf_sweep<GS_SWEEP_WPB>(a.NF, a.bcast, grid, lds, s, a);
}

int launch_bdraw(hipStream_t s, const BdrawArgs& a) {
  if (a.NMX > 64) {
    constexpr int WPB = GS_SWEEP_WPB;
    const int nb = (a.n_chain + WPB - 1) / WPB;
    dim3 grid((unsigned)(a.n_psr * nb));
    const size_t lds = (size_t)gs_tile_scr(a.NF) * WPB * sizeof(double);
    if (a.NF <= 0 || a.NF > 64 || (a.NF & 1)) return 1;
    switch (a.NF / 16 + 1) {
      case 1: hipLaunchKernelGGL((k_bdraw_wide<1, WPB>), grid, dim3(64 * WPB), lds, s, a); return 0;
      case 2: hipLaunchKernelGGL((k_bdraw_wide<2, WPB>), grid, dim3(64 * WPB), lds, s, a); return 0;
      case 3: hipLaunchKernelGGL((k_bdraw_wide<3, WPB>), grid, dim3(64 * WPB), lds, s, a); return 0;
      case 4: hipLaunchKernelGGL((k_bdraw_wide<4, WPB>), grid, dim3(64 * WPB), lds, s, a); return 0;
      default: hipLaunchKernelGGL((k_bdraw_wide<5, WPB>), grid, dim3(64 * WPB), lds, s, a); return 0;
    }
  }
  constexpr int WPB = GS_BDRAW_WPB;
  const int nb = (a.n_chain + WPB - 1) / WPB;
  dim3 grid((unsigned)(a.n_psr * (a.model_per_sys ? nb : (nb + GS_BDRAW_LOOP - 1) / GS_BDRAW_LOOP)));
  const bool fixed = a.NF == 20 || a.NF == 40 || a.NF == 60;
  const bool tiled = GS_BDRAW_TILED && (!fixed || a.bcast == GS_BCAST_TILE);
  const size_t mlds = a.model_per_sys ? 0 : tiled ? (size_t)model_tiled_doubles(a.NF, a.NMX) : (size_t)a.mstride;
  const size_t lds = (mlds + (fixed ? GS_SCR_DOUBLES(a.bcast, a.NF) : gs_tile_scr(a.NF)) * WPB) *
                     sizeof(double);
  return dispatch_nf_bdraw<WPB>(a.NF, a.bcast, grid, lds, s, a);
}

int launch_model_tile(hipStream_t s, const double* model, int n_psr, int NF, int NMX, const int32_t* nm,
                      double* tiled) {
  if (n_psr == 0) return 0;
  hipLaunchKernelGGL(k_model_tile, dim3((unsigned)n_psr), dim3(256), 0, s, model, model_stride_doubles(NF, NMX), NF,
                     NMX, nm, tiled, model_tiled_doubles(NF, NMX));
  return 0;
}

// k_bdraw_pair where it applies (NF = 60, no lnL output, an even chain count) and its waves fill 2 per
// SIMD (n_psr x n_chain / 2 >= 8 waves per CU), or where GS_OPT_SWEEP_SCHED = 3 asks; 2 forces the
// one-chain kernel
// GS_BDRAW_PAIR (off): the cost model picks k_bdraw_pair where its pairs fill 2 waves per SIMD.
// Measured (r06s, curn engine, every chain drawing): 0.430 vs 0.4375-0.468 ms per launch on 3 pulsars
// x 30720 chains (all nM <= 16), but 0.554 vs 0.444-0.473 ms on the 45-pulsar array, whose two nM = 17
// pulsars draw one chain at a time inside the pair kernel and left the persistent ranges that cover
// them longer than the rest; with the ranges weighted by item cost (GS_BPAIR_RM_COST) 0.441-0.445 vs
// 0.444-0.445 ms (r06g3) -- within the noise, so it stays opt-in.  GS_OPT_SWEEP_SCHED = 3 runs it
// (bit-identical).
#ifndef GS_BDRAW_PAIR
#define GS_BDRAW_PAIR 0
#endif
static bool bdraw_pair_wins(const BdrawArgs& a) {
  if (a.NF != 60 || a.lnl || (a.n_chain & 1) || a.model_per_sys) return false;
  if (a.sched == 3) return true;
  if (a.sched || !GS_BDRAW_PAIR) return false;
  return (double)a.n_psr * (a.n_chain / 2) >= 8.0 * device_cus();
}
int launch_bdraw_tiled(hipStream_t s, const BdrawArgs& a0, int* shape) {
  constexpr int WPB = GS_BDRAW_WPB;
  BdrawArgs a = a0;
  if (bdraw_pair_wins(a)) {
    constexpr int PW = GS_PAIR_WPB;
    const size_t lds = ((size_t)a.mstride + (size_t)PW * GS_BPAIR_SCR) * sizeof(double);
    if (lds <= device_lds_optin()) {
      auto kern = k_bdraw_pair<PW>;
      if (lds > 65536 && set_lds(kern, lds)) return 2;
      const int64_t items = (int64_t)a.n_psr * ((a.n_chain + 2 * PW - 1) / (2 * PW));
      int per_cu = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * PW, lds) == hipSuccess && per_cu > 0 &&
          items > (int64_t)per_cu * device_cus())
        a.persist = per_cu * device_cus();
      hipLaunchKernelGGL(kern, dim3((unsigned)(a.persist ? a.persist : items)), dim3(64 * PW), lds, s, a);
      *shape = 3;
      return 0;
    }
  }
  *shape = 2;
  const int nb = (a.n_chain + WPB - 1) / WPB;
  const int64_t nwg = (int64_t)a.n_psr * ((nb + GS_BDRAW_LOOP - 1) / GS_BDRAW_LOOP);
  const size_t lds = ((size_t)a.mstride + (size_t)gs_tile_scr(a.NF) * WPB) * sizeof(double);
  const int NF = a.NF;
  static const int persist_env = getenv("GS_BDRAW_PERSIST") ? atoi(getenv("GS_BDRAW_PERSIST")) : 1;
  // persistent shape: one round of resident workgroups when the classic grid needs more than one
#define GS_TL_K(NFC, NTC, FX, LD)                                                                 \
  {                                                                                               \
    auto kern = k_bdraw_tiled<NFC, NTC, WPB, FX, LD>;                                             \
    if (lds > 65536 && set_lds(kern, lds)) return 2;                                              \
    int per_cu = 0;                                                                               \
    if (persist_env && hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * WPB, lds) == hipSuccess && \
        per_cu > 0 && nwg > (int64_t)per_cu * device_cus())                                       \
      a.persist = per_cu * device_cus();                                                          \
    dim3 grid((unsigned)(a.persist ? a.persist : nwg));                                           \
    hipLaunchKernelGGL(kern, grid, dim3(64 * WPB), lds, s, a);                                    \
    return 0;                                                                                     \
  }
#define GS_TL_LAUNCH(NFC, NTC)                 \
  if (fx) {                                    \
    if (a.lnl) GS_TL_K(NFC, NTC, true, true)   \
    GS_TL_K(NFC, NTC, true, false)             \
  } else {                                     \
    if (a.lnl) GS_TL_K(NFC, NTC, false, true)  \
    GS_TL_K(NFC, NTC, false, false)            \
  }
  const bool fx = model_tiled_fix(a.NMX);
  switch (NF) {
    case 20: GS_TL_LAUNCH(20, 0)
    case 40: GS_TL_LAUNCH(40, 0)
    case 60: GS_TL_LAUNCH(60, 0)
    default: break;
  }
  if (NF <= 0 || NF > 64 || (NF & 1)) return 1;
  switch (NF / 16 + 1) {
    case 1: GS_TL_LAUNCH(0, 1)
    case 2: GS_TL_LAUNCH(0, 2)
    case 3: GS_TL_LAUNCH(0, 3)
    case 4: GS_TL_LAUNCH(0, 4)
    default: GS_TL_LAUNCH(0, 5)
  }
#undef GS_TL_LAUNCH
#undef GS_TL_K
}

int launch_rho_analytic(hipStream_t s, const RhoArgs& a) {
  const int64_t n = (int64_t)a.n_psr * a.n_chain * (a.NF / 2);
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_rho_analytic, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
  return 0;
}
