// b|rho draws of TWO chains per wavefront: k_sweep_pair (the fused sweep's two-chains-per-wave shape, the
// headline's kernel) and k_bdraw_pair (gs_bdraw_tiled, opt-in); GS_OPT_SWEEP_SCHED = 3, DESIGN.md §3.3.
//
// The draw is gibbs_tile.h's bdraw_tile_core (register tiles in the v_mfma_f64_16x16x4f64 C layout,
// augmented Schur block, stored transposes, tiled fixed block) for two systems at once, with the same
// arithmetic per system, so both chains' draws are bit-identical to the one-chain kernel's.  What the
// pairing changes is the diagonal tiles' column elimination (63 % of a draw's VALU): both chains' tiles
// sit in ONE register set -- lanes 0..31 chain a, 32..63 chain b, register 2s + j holding row
// 4s + 2j + h at lane 32X + 16h + c -- so each elimination step's pivot broadcast, v_rcp_f64, Newton
// step and lane mask serve both chains (tile_elim_pair).  The layout is entered and left by
// v_permlane32_swap (16 32-bit swaps each way per tile pair); the TRSM and trailing update run per
// chain in the MFMA layout, their two instruction streams independent (ILP), and the solves and fixed
// block of both chains interleaved step by step (shared LDS round trips and G / R loads).  Both chains'
// 2 x 10 tiles fit 2 waves per SIMD (k_sweep_pair: 256 VGPRs, ~10 spilled outside the draw); measured in
// tools/probe/pair_fact_probe.hip (r06j): the factorisation at 2 waves/SIMD 8,187 SIMD cycles per chain
// against the one-chain kernel's 9,430 at its 3 waves/SIMD.
#pragma once
#include "gibbs_tile.h"

namespace gpair {

// exchange lanes 32..63 of a with lanes 0..31 of b (a double = two 32-bit swaps)
__device__ __forceinline__ void swap32(double& a, double& b) {
  const unsigned long long ua = (unsigned long long)__double_as_longlong(a);
  const unsigned long long ub = (unsigned long long)__double_as_longlong(b);
  auto lo = __builtin_amdgcn_permlane32_swap((unsigned)ua, (unsigned)ub, false, false);
  auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(ua >> 32), (unsigned)(ub >> 32), false, false);
  a = __longlong_as_double((long long)(((unsigned long long)hi[0] << 32) | lo[0]));
  b = __longlong_as_double((long long)(((unsigned long long)hi[1] << 32) | lo[1]));
}

// register of row k in the paired layout
__host__ __device__ constexpr int ptk(int k) { return 2 * (k >> 2) + ((k >> 1) & 1); }

}  // namespace gpair

// GS_PAIR_SKIP: the paired elimination updates only the registers holding rows it needs (one fmac
// fewer per step than the row-group granularity of tile_elim1)
#ifndef GS_PAIR_SKIP
#define GS_PAIR_SKIP 1
#endif
// GS_PAIR_T2: both chains' tile transposes in one LDS round trip (1) or one after the other (0).
// Measured (r06o, headline): 2.004-2.012 ms per launch against 1.953-1.962 -- the paired form holds
// both chains' tiles live across the round trip (20 VGPRs spilled instead of 10)
#ifndef GS_PAIR_T2
#define GS_PAIR_T2 0
#endif
// GS_PAIR_FIX_PRIO: issue priority of the pair draw's fixed block (the one-chain tile core: GS_FIX_PRIO
// = 0).  Measured on the headline (r06p2, 3 interleaved reps): 1.901-1.907 ms per launch at 1 against
// 1.910-1.922 at 0; the MFMA updates at 1 (1.908-1.913) and the elimination at 1 (1.936-1.943) not
#ifndef GS_PAIR_FIX_PRIO
#define GS_PAIR_FIX_PRIO 1
#endif
// GS_PAIR_LOOKAHEAD: step K's trailing updates other than the next diagonal tile are issued inside the
// next diagonal elimination, one tile-op per pivot step (each tile still sees its updates in K order, so
// the draws are unchanged bit for bit; at NT = 4 at most 10 tile-ops wait, fewer than the 16 steps).
// Measured on the headline (r06la, 3 interleaved reps): 1.912-1.920 ms per launch against 1.916-1.925
#ifndef GS_PAIR_LOOKAHEAD
#define GS_PAIR_LOOKAHEAD 1
#endif
// GS_PAIR_SOLVE_ILV: both chains' solves and fixed blocks interleaved (1) or one after the other (0)
#ifndef GS_PAIR_SOLVE_ILV
#define GS_PAIR_SOLVE_ILV 1
#endif

// gtile::transpose of two chains' tiles through their own LDS staging tiles, one round trip for both
__device__ __forceinline__ void transpose2(gs_d4& t0, gs_d4& t1, double* const (&tb)[2], int q, int c) {
  gtile::lds_fence();
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    tb[0][(4 * s + q) * 17 + c] = t0[s];
    tb[1][(4 * s + q) * 17 + c] = t1[s];
  }
  gtile::lds_fence();
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    t0[s] = tb[0][c * 17 + 4 * s + q];
    t1[s] = tb[1][c * 17 + 4 * s + q];
  }
  gtile::lds_fence();
}

// gtile::to_row of two chains' column vectors through their own LDS rows, one round trip for both
__device__ __forceinline__ void to_row2(const double (&v)[2], double* const (&vb)[2], gs_d4 (&o)[2], int q, int c) {
  gtile::lds_fence();
  vb[0][c] = v[0];
  vb[1][c] = v[1];
  gtile::lds_fence();
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    o[0][s] = vb[0][4 * s + q];
    o[1][s] = vb[1][4 * s + q];
  }
  gtile::lds_fence();
}

// tile_elim1's column elimination on two chains at once (paired layout): on return B * rsd is U^-1 of
// each chain's tile and A its column-eliminated tile, both paired; rsd the lane's chain's pivot^-1/2
// of column c.  Same operations per element as tile_elim1<KMAX, PR>.
struct gpair_nofill {
  __device__ void operator()(int) const {}
};
template <int KMAX, bool PR, typename F = gpair_nofill>
__device__ __forceinline__ void tile_elim_pair(double (&A)[8], double (&B)[8], double& rsd, int lane,
                                               F&& fill = F()) {
  using namespace gtile;
  using gpair::ptk;
  if constexpr (PR && GS_DIAG_PRIO > 0) __builtin_amdgcn_s_setprio(GS_DIAG_PRIO);
  const int h = (lane >> 4) & 1, c = lane & 15, base = lane & 32;
#pragma unroll
  for (int t = 0; t < 8; ++t) B[t] = (4 * (t >> 1) + 2 * (t & 1) + h == c) ? 1.0 : 0.0;
  double akc = bcast_lane_bp(A[ptk(0)], base + c);  // row 0 of the lane's chain
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    const int k1 = k >> 2;
    double rn = 0.0;
    if (k + 1 < KMAX) rn = bcast_lane_bp(A[ptk(k + 1)], base + 16 * ((k + 1) & 1) + c);
    __builtin_amdgcn_sched_barrier(0);
    const double akk = newbcast(akc, k);
    if (k + 1 < KMAX) {
#if GS_EXEC_MASK
      const double akm = zero_cols_le(akc, k);
#else
      const double akm = (c > opq(k)) ? akc : 0.0;
#endif
      const double i0 = __builtin_amdgcn_rcp(akk);
#if GS_PIV_NR2
      const double n1 = i0 * fma(akk, i0, -2.0);
      const double ng = (akm * n1) * fma(akk, n1, 2.0);
#else
      const double ng = (akm * i0) * fma(akk, i0, -2.0);
#endif
      akc = fmac_nb(rn, rn, ng, k);
      // registers holding a row >= k of A and <= k of B: from / up to ptk(k).  tile_elim1 also
      // updates the register's other rows of the row group (rows < k of A: eliminated rows nothing
      // reads again; rows > k of B: still identity rows, whose update adds ng x 0 = +-0 and leaves
      // them unchanged for a finite ng), so every value read afterwards is the same
#pragma unroll
      for (int t = GS_PAIR_SKIP ? ptk(k) : 2 * k1; t < 8; ++t) A[t] = fmac_nb(A[t], A[t], ng, k);
#pragma unroll
      for (int t = 0; t <= (GS_PAIR_SKIP ? ptk(k) : 2 * k1 + 1); ++t) B[t] = fmac_nb(B[t], B[t], ng, k);
    }
    fill(k);  // GS_PAIR_LOOKAHEAD: independent work for this step's dependency waits
  }
  // A[ptk(c)] as a select tree on the bits of ptk(c) (a select chain on a lane-varying index is turned
  // into a private-array load, i.e. scratch)
  int pk = ptk(c);
  asm volatile("" : "+v"(pk));
  const bool b0 = pk & 1, b1 = pk & 2, b2 = pk & 4;
  const double d01 = b0 ? A[1] : A[0], d23 = b0 ? A[3] : A[2], d45 = b0 ? A[5] : A[4], d67 = b0 ? A[7] : A[6];
  const double d03 = b1 ? d23 : d01, d47 = b1 ? d67 : d45;
  const double dg = b2 ? d47 : d03;
  double piv = bcast_lane_bp(dg, base + 16 * (c & 1) + c);
  if (KMAX < 16) piv = (c >= KMAX) ? 1.0 : piv;
  rsd = rsq_nr(piv);
  if constexpr (PR && GS_DIAG_PRIO > 0) __builtin_amdgcn_s_setprio(GS_BASE_PRIO);
}

// Two systems' draws (chains a = 0, b = 1) on the tiled model block M: bdraw_tile_core<NT = 4,
// CPC = 12 (NF = 60), LNL = 0, !WIDE, PR> for each, sharing the block's loads and the diagonal
// eliminations.  scr[ch]: each chain's gs_tile_scr(60) doubles of the wave's LDS scratch; zmslot: 128
// more (the chains' z_M, staged before the factorisation so they are not held in registers).  Returns each
// chain's first failed pivot (0: the draw is valid) in fail[ch].
template <bool PR>
__device__ __forceinline__ void bdraw_tile_pair60(const ModelTiled& M, int NMX, int nM, int lane, const double (&phinv)[2],
                                                  const double (&zF)[2], const double (&zM)[2], double (&bF)[2],
                                                  double (&bM)[2], double* const (&scr)[2], double* zmslot,
                                                  int (&fail)[2]) {
  using namespace gtile;
  constexpr int NT = 4, NF = 60, CP = 12, NTILE = NT * (NT + 1) / 2;
  const int q = lane >> 4, c = lane & 15;
  double* tb[2] = {scr[0], scr[1]};
  double* vb[2] = {scr[0] + 272, scr[1] + 272};
  double* ob[2] = {scr[0] + 336, scr[1] + 336};
  double* zm[2] = {zmslot, zmslot + 64};  // z_M of each chain, read by the fixed block

  lds_fence();
#pragma unroll
  for (int ch = 0; ch < 2; ++ch) {
    vb[ch][lane] = phinv[ch];
    ob[ch][lane] = (lane < NF) ? zF[ch] : 0.0;
    zm[ch][lane] = (lane < nM) ? zM[ch] : 0.0;
  }
  lds_fence();
  double phc[2][NT];
#pragma unroll
  for (int ch = 0; ch < 2; ++ch)
#pragma unroll
    for (int K = 0; K < NT; ++K) {
      const int i = 16 * K + c;
      phc[ch][K] = (i < NF) ? vb[ch][i] : 0.0;  // the tiled S' holds the padding's 1
    }
  lds_fence();

  // ---- S tiles of both chains: one load of the shared block, phiinv_F on each chain's diagonal
  int z0 = 0;
  asm volatile("" : "+s"(z0));
  gs_d4 t[2][NTILE];
  {
    const double* Sl = M.S + lane + z0;
#pragma unroll
    for (int I = 0; I < NT; ++I)
#pragma unroll
      for (int J = I; J < NT; ++J) {
        const int ti = tix(I, J, NT);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const double v = Sl[(4 * ti + s) * 64];
#pragma unroll
          for (int ch = 0; ch < 2; ++ch) {
#if GS_EXEC_MASK
            t[ch][ti][s] = (I == J) ? add_on_diag(v, phc[ch][I], s) : v;
#else
            t[ch][ti][s] = v + ((I == J && 4 * s + q == c) ? phc[ch][I] : 0.0);
#endif
          }
        }
      }
  }

  // ---- factorisation
  double ylast[2] = {0.0, 0.0};
  fail[0] = fail[1] = 0;
#pragma unroll
  for (int K = 0; K < NT; ++K) {
    const int kk = tix(K, K, NT);
    double PA[8], PB[8];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      PA[2 * s] = t[0][kk][s];
      PA[2 * s + 1] = t[1][kk][s];
      gpair::swap32(PA[2 * s], PA[2 * s + 1]);
    }
    double rsd;
#if GS_PAIR_LOOKAHEAD
    // the trailing updates of step K - 1 other than tile (K, K), one tile-op per elimination step
    auto fill = [&](int k) {
      if (K == 0) return;
      int n = 0;
#pragma unroll
      for (int I = K; I < NT; ++I)
#pragma unroll
        for (int J = I; J < NT; ++J) {
          if (I == K && J == K) continue;
#pragma unroll
          for (int ch = 0; ch < 2; ++ch) {
            if (n == k)
              t[ch][tix(I, J, NT)] =
                  mfma_tn_sub(t[ch][tix(I, J, NT)], t[ch][tix(K - 1, I, NT)], t[ch][tix(K - 1, J, NT)]);
            ++n;
          }
        }
    };
    if (K == NT - 1)
      tile_elim_pair<CP, PR>(PA, PB, rsd, lane, fill);
    else
      tile_elim_pair<16, PR>(PA, PB, rsd, lane, fill);
    if (K > 0) {  // row K - 1's stored transposes, now that its last updates are issued
#pragma unroll
      for (int ch = 0; ch < 2; ++ch)
#pragma unroll
        for (int J = K; J < NT; ++J) t[ch][tix(K - 1, J, NT)] = transpose(t[ch][tix(K - 1, J, NT)], tb[ch], q, c);
    }
#else
    if (K == NT - 1)
      tile_elim_pair<CP, PR>(PA, PB, rsd, lane);
    else
      tile_elim_pair<16, PR>(PA, PB, rsd, lane);
#endif
    if (K == NT - 1) {
      // y_last[k] = (row CP of the eliminated tile)[k] * pivot_k^-1/2, k < CP, of the lane's chain,
      // then to each chain's column layout (every row group)
      const double yl = bcast_lane_bp(PA[gpair::ptk(CP)], (lane & 32) + 16 * (CP & 1) + c);
      const double yp = (c < CP) ? yl * rsd : 0.0;
      ylast[0] = bcast_lane_bp(yp, c);
      ylast[1] = bcast_lane_bp(yp, 32 + c);
    }
    // first bad pivot of this tile, per chain (row h = 0 of each chain's lanes)
    const unsigned long long badm = __ballot(!(rsd > 0.0 && rsd < __builtin_inf()));
    const unsigned long long bada = badm & 0xffffull, badb = (badm >> 32) & 0xffffull;
    if (!fail[0] && bada) fail[0] = 16 * K + __ffsll((long long)bada);
    if (!fail[1] && badb) fail[1] = 16 * K + __ffsll((long long)badb);
    // U_KK^-1 of both chains back to the MFMA layout
    gs_d4 V[2];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      double x = PB[2 * s] * rsd, y = PB[2 * s + 1] * rsd;
      gpair::swap32(x, y);
      V[0][s] = x;
      V[1][s] = y;
    }
    if constexpr (PR && GS_UPD_PRIO > 0) __builtin_amdgcn_s_setprio(GS_UPD_PRIO);
#pragma unroll
    for (int ch = 0; ch < 2; ++ch) {
      t[ch][kk] = V[ch];
#pragma unroll
      for (int J = K + 1; J < NT; ++J) {
        const gs_d4 z = {0.0, 0.0, 0.0, 0.0};
        t[ch][tix(K, J, NT)] = mfma_tn(z, V[ch], t[ch][tix(K, J, NT)]);
      }
    }
#if GS_PAIR_T2
    t[0][kk] = V[0];
    t[1][kk] = V[1];
    transpose2(t[0][kk], t[1][kk], tb, q, c);
#else
#pragma unroll
    for (int ch = 0; ch < 2; ++ch) t[ch][kk] = transpose(V[ch], tb[ch], q, c);
#endif
#if GS_PAIR_LOOKAHEAD
    // only tile (K + 1, K + 1) now: the next elimination needs it; the rest go into its steps
    if (K + 1 < NT) {
#pragma unroll
      for (int ch = 0; ch < 2; ++ch)
        t[ch][tix(K + 1, K + 1, NT)] =
            mfma_tn_sub(t[ch][tix(K + 1, K + 1, NT)], t[ch][tix(K, K + 1, NT)], t[ch][tix(K, K + 1, NT)]);
    }
#else
#pragma unroll
    for (int I = K + 1; I < NT; ++I)
#pragma unroll
      for (int J = I; J < NT; ++J)
#pragma unroll
        for (int ch = 0; ch < 2; ++ch)
          t[ch][tix(I, J, NT)] = mfma_tn_sub(t[ch][tix(I, J, NT)], t[ch][tix(K, I, NT)], t[ch][tix(K, J, NT)]);
#endif
#if GS_PAIR_LOOKAHEAD
    // (row K's transposes follow the next elimination, after its last use by the pending updates)
#elif GS_PAIR_T2
#pragma unroll
    for (int J = K + 1; J < NT; ++J) transpose2(t[0][tix(K, J, NT)], t[1][tix(K, J, NT)], tb, q, c);
#else
#pragma unroll
    for (int ch = 0; ch < 2; ++ch)
#pragma unroll
      for (int J = K + 1; J < NT; ++J) t[ch][tix(K, J, NT)] = transpose(t[ch][tix(K, J, NT)], tb[ch], q, c);
#endif
    if constexpr (PR && GS_UPD_PRIO > 0) __builtin_amdgcn_s_setprio(GS_BASE_PRIO);
  }

#if GS_PAIR_SOLVE_ILV
  // ---- the solves and the fixed block of both chains interleaved step by step (each chain's
  // operations in the one-chain order); the LDS round trips of the row transposes and the fixed
  // block's G / R loads are shared
  {
    double ycol[2][NT];
#pragma unroll
    for (int ch = 0; ch < 2; ++ch) {
#pragma unroll
      for (int K = 0; K + 1 < NT; ++K) ycol[ch][K] = bcast_group_bp(t[ch][tix(K, NT - 1, NT)][CP >> 2], CP & 3, c);
      ycol[ch][NT - 1] = ylast[ch];
    }
    if constexpr (PR && GS_SOLVE_PRIO > 0) __builtin_amdgcn_s_setprio(GS_SOLVE_PRIO);
    double xcol[2][NT];
    gs_d4 xrow[2][NT];
#pragma unroll
    for (int K = NT - 1; K >= 0; --K) {
      double v[2];
#pragma unroll
      for (int ch = 0; ch < 2; ++ch) {
        double p = 0.0;
#pragma unroll
        for (int J = K + 1; J < NT; ++J) {
          const gs_d4 ut = t[ch][tix(K, J, NT)];
#pragma unroll
          for (int s = 0; s < 4; ++s) p = fma(ut[s], xrow[ch][J][s], p);
        }
        if (K + 1 < NT) p = qsum(p);
        v[ch] = ycol[ch][K] + ob[ch][16 * K + c] - p;
      }
      gs_d4 sr[2];
      to_row2(v, vb, sr, q, c);
#pragma unroll
      for (int ch = 0; ch < 2; ++ch) {
        const gs_d4 W = t[ch][tix(K, K, NT)];
        double p2 = 0.0;
#pragma unroll
        for (int s = 0; s < 4; ++s) p2 = fma(W[s], sr[ch][s], p2);
        xcol[ch][K] = qsum(p2);
      }
      const double xv[2] = {xcol[0][K], xcol[1][K]};
      gs_d4 xr[2];
      to_row2(xv, vb, xr, q, c);
      xrow[0][K] = xr[0];
      xrow[1][K] = xr[1];
    }
    lds_fence();
#pragma unroll
    for (int ch = 0; ch < 2; ++ch)
#pragma unroll
      for (int K = 0; K < NT; ++K) ob[ch][16 * K + c] = xcol[ch][K];
    lds_fence();
#pragma unroll
    for (int ch = 0; ch < 2; ++ch) bF[ch] = (lane < NF) ? ob[ch][lane] : 0.0;
    lds_fence();
    if constexpr (PR && GS_SOLVE_PRIO > 0) __builtin_amdgcn_s_setprio(GS_BASE_PRIO);

    if constexpr (PR && GS_PAIR_FIX_PRIO > 0) __builtin_amdgcn_s_setprio(GS_PAIR_FIX_PRIO);
    // fixed-prior block x_M = h + R z_M - G x_F (tiled G' = -G and R', nM <= 16: one chunk); z_M was
    // staged in the chains' zm slots before the factorisation
    const int row = c;
    const bool rok = row < nM;
    double p[2] = {0.0, 0.0};
    const double* Gl = M.G + lane + z0;
#pragma unroll
    for (int J = 0; J < NT; ++J)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const double g = Gl[(4 * J + s) * 64];
        p[0] = fma(g, xrow[0][J][s], p[0]);
        p[1] = fma(g, xrow[1][J][s], p[1]);
      }
    const double* Rl = M.R + lane + z0;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const double r = Rl[s * 64];
      p[0] = fma(r, zm[0][4 * s + q], p[0]);
      p[1] = fma(r, zm[1][4 * s + q], p[1]);
    }
    const double hr = M.h[row + z0];
#pragma unroll
    for (int ch = 0; ch < 2; ++ch) {
      const double pp = qsum(p[ch]);
      ob[ch][row] = rok ? hr + pp : 0.0;
    }
    lds_fence();
#pragma unroll
    for (int ch = 0; ch < 2; ++ch) bM[ch] = (lane < nM) ? ob[ch][lane] : 0.0;
    lds_fence();
    if constexpr (PR && GS_PAIR_FIX_PRIO > 0) __builtin_amdgcn_s_setprio(GS_BASE_PRIO);
  }
#else
  // ---- the solves and the fixed block, one chain after the other: chain a's tiles and solution rows
  // are dead before chain b's solve needs its own (interleaving the two held ~250 VGPRs and spilled)
#pragma unroll
  for (int ch = 0; ch < 2; ++ch) {
    // forward (augmented): y_K = column CP of U_K,last = row CP of the stored U_K,last^T
    double ycol[NT];
#pragma unroll
    for (int K = 0; K + 1 < NT; ++K) ycol[K] = bcast_group_bp(t[ch][tix(K, NT - 1, NT)][CP >> 2], CP & 3, c);
    ycol[NT - 1] = ylast[ch];

    if constexpr (PR && GS_SOLVE_PRIO > 0) __builtin_amdgcn_s_setprio(GS_SOLVE_PRIO);
    // backward: U x = y + zF
    double xcol[NT];
    gs_d4 xrow[NT];
#pragma unroll
    for (int K = NT - 1; K >= 0; --K) {
      double p = 0.0;
#pragma unroll
      for (int J = K + 1; J < NT; ++J) {
        const gs_d4 ut = t[ch][tix(K, J, NT)];
#pragma unroll
        for (int s = 0; s < 4; ++s) p = fma(ut[s], xrow[J][s], p);
      }
      if (K + 1 < NT) p = qsum(p);
      const gs_d4 sr = to_row(ycol[K] + ob[ch][16 * K + c] - p, vb[ch], q, c);
      const gs_d4 W = t[ch][tix(K, K, NT)];
      double p2 = 0.0;
#pragma unroll
      for (int s = 0; s < 4; ++s) p2 = fma(W[s], sr[s], p2);
      xcol[K] = qsum(p2);
      xrow[K] = to_row(xcol[K], vb[ch], q, c);
    }
    lds_fence();
#pragma unroll
    for (int K = 0; K < NT; ++K) ob[ch][16 * K + c] = xcol[K];
    lds_fence();
    bF[ch] = (lane < NF) ? ob[ch][lane] : 0.0;
    lds_fence();
    if constexpr (PR && GS_SOLVE_PRIO > 0) __builtin_amdgcn_s_setprio(GS_BASE_PRIO);

    if constexpr (PR && GS_PAIR_FIX_PRIO > 0) __builtin_amdgcn_s_setprio(GS_PAIR_FIX_PRIO);
    // fixed-prior block x_M = h + R z_M - G x_F (tiled G' = -G and R', nM <= 16: one chunk); z_M was
    // staged in the chain's zm slot before the factorisation
    {
      const int row = c;
      const bool rok = row < nM;
      double p = 0.0;
      const double* Gl = M.G + lane + z0;
#pragma unroll
      for (int J = 0; J < NT; ++J)
#pragma unroll
        for (int s = 0; s < 4; ++s) p = fma(Gl[(4 * J + s) * 64], xrow[J][s], p);
      const double* Rl = M.R + lane + z0;
#pragma unroll
      for (int s = 0; s < 4; ++s) p = fma(Rl[s * 64], zm[ch][4 * s + q], p);
      p = qsum(p);
      const double xm = rok ? M.h[row + z0] + p : 0.0;
      ob[ch][row] = xm;
    }
    lds_fence();
    bM[ch] = (lane < nM) ? ob[ch][lane] : 0.0;
    lds_fence();
    if constexpr (PR && GS_PAIR_FIX_PRIO > 0) __builtin_amdgcn_s_setprio(GS_BASE_PRIO);
  }
#endif
}
