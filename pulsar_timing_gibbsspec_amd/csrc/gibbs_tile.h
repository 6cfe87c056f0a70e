// b|rho draw on 16x16 fp64 MFMA tiles, one wavefront per system.
//
// Measured on MI355X (tools/probe/mfma_probe.hip): a v_readlane x2 + v_fma_f64
// broadcast step costs ~23 SIMD cycles, and f64 VALU and f64 MFMA do not overlap
// on a SIMD, while v_mfma_f64_16x16x4f64 runs at 77.7 TFLOP/s with the operand
// broadcast built in.  So the NF x NF Schur block S = S0 + diag(phiinv_F) is
// factorised as an UPPER Cholesky S = U^T U on NT = ceil(NF/16) tile rows:
//
//   C layout: lane l = 16q + c holds X[4s+q][c] in register s (s = 0..3), the
//   v_mfma_f64_16x16x4f64 C/D layout.  With A operand = register s of X and
//   B operand = register s of Y, four MFMAs accumulate X^T Y (probe-verified),
//   so every tile product below reads its operands straight from registers.
//
//   for K: factor diag tile T_KK -> W_K = U_KK^-T by row operations on [T_KK | I]
//          (VALU, rows broadcast through the wave's LDS scratch);
//          V_K = U_KK^-1 = W_K^T (LDS transpose);
//          U_KJ = V_K^T T_KJ                      (TRSM, 4 MFMA per tile);
//          T_IJ -= U_KI^T U_KJ, K < I <= J        (update, 4 MFMA per tile).
//   forward  U^T y = dF and backward U x = y + zF by tile GEMVs with the
//   diagonal inverses (no serial substitution), x_M = h + R z_M - G x_F.
//
// Padding rows/columns (NF..16 NT-1) are an identity block with zero RHS, so they
// decouple exactly.  Same law and same normals as bdraw_wave (lane-row readlane
// path): the draws agree to rounding.
#pragma once
#include "gibbs_common.h"

typedef double gs_d4 __attribute__((ext_vector_type(4)));

// Phase profiling (variant builds only, -DGS_PHASE_PROF): cycles per phase summed over
// waves, read back with gs_debug_phase_cycles.
#ifdef GS_PHASE_PROF
static __device__ unsigned long long gs_phase_cyc[8];
// per-wave accumulators in the wave's LDS scratch (doubles 416..423), flushed once
#define GS_PH_ACC(scr) reinterpret_cast<unsigned long long*>((scr) + 416)
#define GS_PH_INIT(scr) \
  if ((threadIdx.x & 63) < 8) GS_PH_ACC(scr)[threadIdx.x & 63] = 0ull;
#define GS_PH_FLUSH(scr) \
  if ((threadIdx.x & 63) < 8) atomicAdd(&gs_phase_cyc[threadIdx.x & 63], GS_PH_ACC(scr)[threadIdx.x & 63]);
#define GS_PH_BEGIN                   \
  __builtin_amdgcn_sched_barrier(0); \
  unsigned long long _ph_t = clock64(); \
  __builtin_amdgcn_sched_barrier(0);
#define GS_PH(i)                                                             \
  {                                                                          \
    __builtin_amdgcn_sched_barrier(0);                                       \
    const unsigned long long _t = clock64();                                 \
    __builtin_amdgcn_sched_barrier(0);                                       \
    if ((threadIdx.x & 63) == 0) atomicAdd(&GS_PH_ACC(scr)[i], _t - _ph_t); \
    _ph_t = _t;                                                              \
  }
#else
#define GS_PH_INIT(scr)
#define GS_PH_FLUSH(scr)
#define GS_PH_BEGIN
#define GS_PH(i)
#endif

namespace gtile {

// Ordering of the wave's cross-lane LDS traffic: wavefront-scope release/acquire
// fences around the wave barrier (the hardware executes a wave's DS instructions in
// order, so no s_barrier is needed).  A bare wave_barrier + asm memory clobber is NOT
// enough: the backend scheduler reordered a transpose's LDS reads past another
// transpose's writes (found by the likelihood tests, tests/test_gpu_lnlike.py).
__device__ __forceinline__ void lds_fence() { wave_lds_sync(); }

// acc + X^T Y for C-layout tiles X, Y
__device__ __forceinline__ gs_d4 mfma_tn(gs_d4 acc, const gs_d4 x, const gs_d4 y) {
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x[0], y[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x[1], y[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x[2], y[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x[3], y[3], acc, 0, 0, 0);
  return acc;
}

// acc - X^T Y: on gfx950 the f64 MFMA's blgp field is the operand-negate modifier (blgp = 1:
// neg:[1,0,0]), so the trailing update needs no v_xor per register to negate X (bit-identical:
// (-x) y and -(x y) round the same)
#ifndef GS_MFMA_NEG
#define GS_MFMA_NEG 1
#endif
__device__ __forceinline__ gs_d4 mfma_tn_sub(gs_d4 acc, const gs_d4 x, const gs_d4 y) {
#if GS_MFMA_NEG
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x[0], y[0], acc, 0, 0, 1);
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x[1], y[1], acc, 0, 0, 1);
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x[2], y[2], acc, 0, 0, 1);
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x[3], y[3], acc, 0, 0, 1);
  return acc;
#else
  return mfma_tn(acc, -x, y);
#endif
}

__device__ __forceinline__ gs_d4 transpose(const gs_d4 t, double* tb, int q, int c) {
  lds_fence();
#pragma unroll
  for (int s = 0; s < 4; ++s) tb[(4 * s + q) * 17 + c] = t[s];
  lds_fence();
  gs_d4 o;
#pragma unroll
  for (int s = 0; s < 4; ++s) o[s] = tb[c * 17 + 4 * s + q];
  lds_fence();
  return o;
}

// column layout (lane (q, c) holds v[c]) -> row layout (register s holds v[4s+q])
__device__ __forceinline__ gs_d4 to_row(double v, double* vb, int q, int c) {
  lds_fence();
  vb[c] = v;  // the four lanes of column c write the same value
  lds_fence();
  gs_d4 o;
#pragma unroll
  for (int s = 0; s < 4; ++s) o[s] = vb[4 * s + q];
  lds_fence();
  return o;
}

// v from row group g (lanes 16g..16g+15) to all four row groups, same column, through
// the LDS crossbar (ds_bpermute_b32 x2): no VALU slots; the latency is hidden when the
// row is requested a step ahead.
__device__ __forceinline__ double bcast_group_bp(double v, int g, int c) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const int addr = (16 * g + c) * 4;
  const unsigned lo = (unsigned)__builtin_amdgcn_ds_bpermute(addr, (int)(unsigned)u);
  const unsigned hi = (unsigned)__builtin_amdgcn_ds_bpermute(addr, (int)(unsigned)(u >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// v of lane `src` (per-lane source) through the LDS crossbar
__device__ __forceinline__ double bcast_lane_bp(double v, int src) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_ds_bpermute(src * 4, (int)(unsigned)u);
  const unsigned hi = (unsigned)__builtin_amdgcn_ds_bpermute(src * 4, (int)(unsigned)(u >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// an SGPR copy of a compile-time int the compiler cannot see through
__device__ __forceinline__ int opq(int v) {
  asm volatile("" : "+s"(v));
  return v;
}

// lane n of each 16-lane row to the whole row (DPP row_newbcast, n compile-time)
template <int N>
__device__ __forceinline__ double newbcast_c(double v) {
  return __builtin_amdgcn_mov_dpp(v, 0x150 + N, 0xf, 0xf, false);  // no "old": every lane is written
}
__device__ __forceinline__ double newbcast(double v, int n) {
  switch (n) {  // n is constant after unrolling: the switch folds away
    case 0: return newbcast_c<0>(v);
    case 1: return newbcast_c<1>(v);
    case 2: return newbcast_c<2>(v);
    case 3: return newbcast_c<3>(v);
    case 4: return newbcast_c<4>(v);
    case 5: return newbcast_c<5>(v);
    case 6: return newbcast_c<6>(v);
    case 7: return newbcast_c<7>(v);
    case 8: return newbcast_c<8>(v);
    case 9: return newbcast_c<9>(v);
    case 10: return newbcast_c<10>(v);
    case 11: return newbcast_c<11>(v);
    case 12: return newbcast_c<12>(v);
    case 13: return newbcast_c<13>(v);
    case 14: return newbcast_c<14>(v);
    default: return newbcast_c<15>(v);
  }
}

// acc + (lane n of this 16-lane row's v) * m as ONE v_fmac_f64_dpp row_newbcast:n.
// fmac_nb: the s_nop only at step 0 of a tile (the DPP sources of later steps were
// written by the previous step).
// The s_nop covers the VALU-write -> DPP-read hazard (the compiler cannot see into asm).
// Not volatile: a pure function of its operands, so the scheduler may hoist the
// row broadcast (ds_bpermute) of the next step above it.
template <int N>
__device__ __forceinline__ double fmac_nb_c(double acc, double v, double m) {
  asm("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
               : "+v"(acc)
               : "v"(v), "v"(m), "n"(N));
  return acc;
}
// Same without the s_nop, for a DPP source last written by VALU at least two
// instructions earlier (the previous elimination step).
template <int N>
__device__ __forceinline__ double fmac_nb_c_nn(double acc, double v, double m) {
  asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
      : "+v"(acc)
      : "v"(v), "v"(m), "n"(N));
  return acc;
}
__device__ __forceinline__ double fmac_nb(double acc, double v, double m, int n) {
  switch (n) {
    case 0: return fmac_nb_c<0>(acc, v, m);
    case 1: return fmac_nb_c_nn<1>(acc, v, m);
    case 2: return fmac_nb_c_nn<2>(acc, v, m);
    case 3: return fmac_nb_c_nn<3>(acc, v, m);
    case 4: return fmac_nb_c_nn<4>(acc, v, m);
    case 5: return fmac_nb_c_nn<5>(acc, v, m);
    case 6: return fmac_nb_c_nn<6>(acc, v, m);
    case 7: return fmac_nb_c_nn<7>(acc, v, m);
    case 8: return fmac_nb_c_nn<8>(acc, v, m);
    case 9: return fmac_nb_c_nn<9>(acc, v, m);
    case 10: return fmac_nb_c_nn<10>(acc, v, m);
    case 11: return fmac_nb_c_nn<11>(acc, v, m);
    case 12: return fmac_nb_c_nn<12>(acc, v, m);
    case 13: return fmac_nb_c_nn<13>(acc, v, m);
    case 14: return fmac_nb_c_nn<14>(acc, v, m);
    default: return fmac_nb_c_nn<15>(acc, v, m);
  }
}

// v with the lanes of columns c = lane & 15 <= K zeroed: exec set by two SALU moves of a
// literal around ONE v_mov_b64, then back to all lanes (instead of v_cmp + two v_cndmask_b32
// per elimination step).  The tile routines run on full waves only (their DPP and
// ds_bpermute exchanges read every lane), so exec is all ones on entry; restoring -1
// instead of a saved copy needs no SGPR pair (the sweep kernel's SGPRs are at their limit:
// 15 saved pairs spilled 26 more SGPRs into VGPR lanes, +164 v_readlane).  No DPP reads
// inside the block (a VALU exec write needs wait states before a DPP op; SALU ones do not).
template <int K>
__device__ __forceinline__ double zero_cols_le_c(double v) {
  constexpr unsigned P16 = (2u << K) - 1u;
  constexpr unsigned P32 = P16 | (P16 << 16);
  asm("s_mov_b32 exec_lo, %1\n\t"
      "s_mov_b32 exec_hi, %1\n\t"
      "v_mov_b64 %0, 0\n\t"
      "s_mov_b64 exec, -1"
      : "+v"(v)
      : "n"(P32));
  return v;
}
__device__ __forceinline__ double zero_cols_le(double v, int k) {
#define GS_ZC(N) \
  case N: return zero_cols_le_c<N>(v);
  switch (k) {  // k constant after unrolling
    GS_ZC(0) GS_ZC(1) GS_ZC(2) GS_ZC(3) GS_ZC(4) GS_ZC(5) GS_ZC(6) GS_ZC(7)
    GS_ZC(8) GS_ZC(9) GS_ZC(10) GS_ZC(11) GS_ZC(12) GS_ZC(13) GS_ZC(14)
    default: return zero_cols_le_c<15>(v);
  }
#undef GS_ZC
}

// x^-1/2: v_rsq_f64 + two Newton steps (x > 0 normal; NaN/inf/<= 0 propagate to a
// non-finite or non-positive result, caught by the pivot ballot)
__device__ __forceinline__ double rsq_nr(double x) {
  double y = __builtin_amdgcn_rsq(x);
  const double hx = 0.5 * x;
  y = y * fma(-hx * y, y, 1.5);
  y = y * fma(-hx * y, y, 1.5);
  return y;
}

// sum over the four lanes of a column (q = 0..3)
__device__ __forceinline__ double qsum(double p) {
  p += __shfl_xor(p, 16);
  p += __shfl_xor(p, 32);
  return p;
}

__device__ __forceinline__ constexpr int tix(int I, int J, int NT) {
  return I * NT - (I * (I - 1)) / 2 + (J - I);
}

}  // namespace gtile

// Inverse factor of one diagonal tile (C layout, symmetric positive definite on its
// first KMAX rows/columns, identity-padded beyond): on return V = B * rsd is U^-1
// for the upper Cholesky factor U of the tile, rsd the pivot^-1/2 of the lane's
// column (1 on padding), and A holds the column-eliminated tile (A E, lower).
//
// Column elimination on [A ; I] -> B = E (unit upper) with A E lower triangular;
// U^-1 = E diag(pivot^-1/2).  Column c of both lives in lane column c, so the
// pivot scale is lane-local; A[r][k], B[r][k] come from lane k of the same
// 16-lane row (DPP row_newbcast, fused into v_fmac_f64_dpp) and row k of A from row
// group k&3 (ds_bpermute): no LDS traffic, no transpose.  Step k: pivot A[k][k] by
// DPP from row k (replicated in every row group), -1/pivot by v_rcp_f64 + one Newton
// step.  Row k+1 (as before step k) is requested ahead of the pivot chain and
// updated by the same column operation.  Measured on MI355X against an LDS
// row-broadcast version and a v_permlane32/16_swap broadcast: 1.7x and 1.04x faster.
// Issue priority (s_setprio) per phase.  Two independent waves share each SIMD; VALU issue is
// arbitrated by priority, then age (MI355X_MICROARCH.md, co-resident waves items 2 and 4).
// Raising the wave that runs the latency-bound dependent chains -- the diagonal-tile
// elimination (GS_DIAG_PRIO) and the backward solve (GS_SOLVE_PRIO) -- lets its next link
// issue as soon as it is ready while the partner fills the gaps with MFMAs and independent
// VALU.  Measured on MI355X (4096 chains, NF = 60, 100-sweep launches; tools/gpu_ab_lib.sh):
// 2.96-3.09 ms -> 2.77-2.92 ms per launch with DIAG 2 / SOLVE 1; raising the update,
// fixed-block or rho phases as well, or DIAG 3, was no better.
#ifndef GS_DIAG_PRIO
#define GS_DIAG_PRIO 2
#endif
#ifndef GS_BASE_PRIO
#define GS_BASE_PRIO 0
#endif
#ifndef GS_UPD_PRIO  // ... while it runs the TRSM / trailing-update MFMAs
#define GS_UPD_PRIO 0
#endif
#ifndef GS_SOLVE_PRIO  // ... while it runs the backward solve
#define GS_SOLVE_PRIO 1
#endif
#ifndef GS_FIX_PRIO  // ... while it runs the fixed-prior block
#define GS_FIX_PRIO 0
#endif
#ifndef GS_RHO_PRIO  // ... while it runs the sweep's rho|b draw and gate (k_sweep_freespec)
#define GS_RHO_PRIO 0
#endif
#ifndef GS_PIV_NR2
#define GS_PIV_NR2 0
#endif
#ifndef GS_EXEC_MASK
#define GS_EXEC_MASK 1
#endif
template <int KMAX, bool PR = false>
__device__ __forceinline__ void tile_elim1(gs_d4& A, gs_d4& B, double& rsd, int q, int c) {
  using namespace gtile;
  if constexpr (PR && GS_DIAG_PRIO > 0) __builtin_amdgcn_s_setprio(GS_DIAG_PRIO);
#pragma unroll
  for (int s = 0; s < 4; ++s) B[s] = (4 * s + q == c) ? 1.0 : 0.0;
  double akc = bcast_group_bp(A[0], 0, c);  // row 0
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    const int k1 = k >> 2;
    // row k+1 as before step k, requested first so the crossbar latency overlaps
    // the pivot chain below (the barrier keeps the scheduler from sinking it)
    double rn = 0.0;
    if (k + 1 < KMAX) rn = bcast_group_bp(A[(k + 1) >> 2], (k + 1) & 3, c);
    __builtin_amdgcn_sched_barrier(0);
    const double akk = newbcast(akc, k);  // A[k][k]
    if (k + 1 < KMAX) {
      // lane mask c > k from an opaque k: one v_cmp per step instead of loop-invariant
      // 64-bit masks held in (spilled) SGPRs across the caller's sweep loop; applied to
      // the row before the pivot arrives, so it is off the critical path
#if GS_EXEC_MASK
      const double akm = zero_cols_le(akc, k);
#else
      const double akm = (c > opq(k)) ? akc : 0.0;
#endif
      // -A[k][c]/A[k][k] = akm i0 (akk i0 - 2) (one Newton step on v_rcp_f64): the two
      // products run side by side, 4 dependent ops from pivot to multiplier
      // (akk keeps two uses: a single-use DPP move feeding v_rcp_f64 is folded by the compiler's
      // DPP combiner into v_rcp_f64_dpp, which returns 1/0 on MI355X -- tools/probe/rcpdpp_probe.hip)
      const double i0 = __builtin_amdgcn_rcp(akk);
#if GS_PIV_NR2
      // two Newton steps: -1/akk to ~1 ulp instead of ~2^-50 relative
      const double n1 = i0 * fma(akk, i0, -2.0);           // -1/akk, one step
      const double ng = (akm * n1) * fma(akk, n1, 2.0);
#else
      const double ng = (akm * i0) * fma(akk, i0, -2.0);
#endif
      akc = fmac_nb(rn, rn, ng, k);                        // row k+1 after step k
#pragma unroll
      for (int s = k1; s < 4; ++s) A[s] = fmac_nb(A[s], A[s], ng, k);
#pragma unroll
      for (int s = 0; s <= k1; ++s) B[s] = fmac_nb(B[s], B[s], ng, k);
    }
  }
  // column elimination leaves A[k][k] = pivot k on the diagonal: lane (c&3, c) holds
  // it in register c>>2; fetch it for every lane of column c
  double dg = A[0];
#pragma unroll
  for (int s = 1; s < 4; ++s) dg = ((c >> 2) == s) ? A[s] : dg;
  double piv = bcast_lane_bp(dg, 16 * (c & 3) + c);
  if (KMAX < 16) piv = (c >= KMAX) ? 1.0 : piv;  // padding (incl. an augmented pivot)
  rsd = rsq_nr(piv);
  if constexpr (PR && GS_DIAG_PRIO > 0) __builtin_amdgcn_s_setprio(GS_BASE_PRIO);
}

namespace gtile {
// fmac_nb with a compile-time choice of the hazard s_nop (n constant after unrolling)
template <bool NOP>
__device__ __forceinline__ double fmac_nbx(double acc, double v, double m, int n) {
#define GS_FMX(N) \
  case N: return NOP ? fmac_nb_c<N>(acc, v, m) : fmac_nb_c_nn<N>(acc, v, m);
  switch (n) {
    GS_FMX(0) GS_FMX(1) GS_FMX(2) GS_FMX(3) GS_FMX(4) GS_FMX(5) GS_FMX(6) GS_FMX(7)
    GS_FMX(8) GS_FMX(9) GS_FMX(10) GS_FMX(11) GS_FMX(12) GS_FMX(13) GS_FMX(14)
    default: return NOP ? fmac_nb_c<15>(acc, v, m) : fmac_nb_c_nn<15>(acc, v, m);
  }
#undef GS_FMX
}
}  // namespace gtile

// Same contract as tile_elim1 (column steps k = 0..KMAX-2, each eliminating row k from
// every column c > k), but two steps per link of the dependent chain: for columns
// c > k+1 the 2x2 pivot block P = [[a, b], [c', d]] of rows/columns k, k+1 gives
// col_c -= g0 col_k + g1 col_{k+1} with P g = (A[k][c], A[k+1][c]); column k+1 takes
// step k alone (g0 = b/a).  The pivot chain per pair is det -> rcp -> Newton -> scale
// (both multipliers side by side), so a 16-column tile costs 8 chain links instead of
// 15.  The two column operations read the ORIGINAL columns k and k+1: column k+1 is
// applied first (its own multiplier is 0 on lanes k and k+1), then column k.  Same
// arithmetic as block LDL^T of the tile (the trailing block stays symmetric), equal to
// tile_elim1 to rounding.
template <int KMAX>
__device__ __forceinline__ void tile_elim2(gs_d4& A, gs_d4& B, double& rsd, int q, int c) {
  using namespace gtile;
  constexpr int NS = KMAX - 1;  // column steps 0..KMAX-2
  constexpr int NP = NS > 0 ? NS / 2 : 0;
#pragma unroll
  for (int s = 0; s < 4; ++s) B[s] = (4 * s + q == c) ? 1.0 : 0.0;
  double r0 = bcast_group_bp(A[0], 0, c);                 // row 0
  double r1 = (NP > 0) ? bcast_group_bp(A[0], 1, c) : 0.0;  // row 1
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int k = 2 * p, k1 = k >> 2;
    const bool nx0 = k + 2 <= NS - 1, nx1 = k + 3 <= NS - 1;
    // the next pivot rows as before this pair, requested ahead of the pivot chain
    double n0 = 0.0, n1 = 0.0;
    if (nx0) n0 = bcast_group_bp(A[(k + 2) >> 2], (k + 2) & 3, c);
    if (nx1) n1 = bcast_group_bp(A[(k + 3) >> 2], (k + 3) & 3, c);
    __builtin_amdgcn_sched_barrier(0);
    const double a = newbcast(r0, k), b = newbcast(r0, k + 1);
    const double cq = newbcast(r1, k), d = newbcast(r1, k + 1);
    const bool beyond = c > opq(k + 1);
    const double r0m = beyond ? r0 : 0.0, r1m = beyond ? r1 : 0.0;
    const double det = fma(a, d, -(b * cq));
    const double i0 = __builtin_amdgcn_rcp(det);
    const double sd = i0 * fma(det, i0, -2.0);  // -1/det (one Newton step)
    const double ia = __builtin_amdgcn_rcp(a);
    const double sa = ia * fma(a, ia, -2.0);    // -1/a
    const double ng1 = fma(a, r1m, -(cq * r0m)) * sd;
    double ng0 = fma(d, r0m, -(b * r1m)) * sd;
    ng0 = (c == k + 1) ? b * sa : ng0;
    // pass 1: original column k+1 (multiplier 0 on lanes <= k+1)
    if (nx0) n0 = fmac_nbx<false>(n0, n0, ng1, k + 1);
    if (nx1) n1 = fmac_nbx<false>(n1, n1, ng1, k + 1);
#pragma unroll
    for (int s = k1; s < 4; ++s) A[s] = fmac_nbx<false>(A[s], A[s], ng1, k + 1);
#pragma unroll
    for (int s = 0; s <= k1; ++s) B[s] = fmac_nbx<false>(B[s], B[s], ng1, k + 1);
    // pass 2: original column k (unchanged by pass 1); the s_nop covers a DPP read
    // scheduled right after pass 1's write of the same register
    if (nx0) n0 = fmac_nbx<true>(n0, n0, ng0, k);
    if (nx1) n1 = fmac_nbx<true>(n1, n1, ng0, k);
#pragma unroll
    for (int s = k1; s < 4; ++s) A[s] = fmac_nbx<true>(A[s], A[s], ng0, k);
#pragma unroll
    for (int s = 0; s <= k1; ++s) B[s] = fmac_nbx<true>(B[s], B[s], ng0, k);
    r0 = n0;
    r1 = n1;
  }
  if constexpr (NS > 0 && (NS & 1)) {
    // trailing single step k = KMAX-2 (row k is r0)
    constexpr int k = NS - 1, k1 = k >> 2;
    __builtin_amdgcn_sched_barrier(0);
    const double akk = newbcast(r0, k);
    const double akm = (c > opq(k)) ? r0 : 0.0;
    const double i0 = __builtin_amdgcn_rcp(akk);
    const double ng = (akm * i0) * fma(akk, i0, -2.0);
#pragma unroll
    for (int s = k1; s < 4; ++s) A[s] = fmac_nbx<true>(A[s], A[s], ng, k);
#pragma unroll
    for (int s = 0; s <= k1; ++s) B[s] = fmac_nbx<true>(B[s], B[s], ng, k);
  }
  double dg = A[0];
#pragma unroll
  for (int s = 1; s < 4; ++s) dg = ((c >> 2) == s) ? A[s] : dg;
  double piv = bcast_lane_bp(dg, 16 * (c & 3) + c);
  if (KMAX < 16) piv = (c >= KMAX) ? 1.0 : piv;
  rsd = rsq_nr(piv);
}

// Off by default: measured on MI355X (4096 chains, NF = 60) the pair variant is slower,
// 3.40 vs 3.00 ms per 100-sweep launch -- at 2 waves/SIMD the diag factor is bound by
// VALU issue (the pair adds det, a second rcp and two more DPP broadcasts per link, and
// 17 more spilled VGPRs), not by the length of the dependent chain.
#ifndef GS_TILE_PAIR
#define GS_TILE_PAIR 0
#endif
template <int KMAX, bool PR = false>
__device__ __forceinline__ void tile_elim(gs_d4& A, gs_d4& B, double& rsd, int q, int c) {
  if constexpr (GS_TILE_PAIR)
    tile_elim2<KMAX>(A, B, rsd, q, c);
  else
    tile_elim1<KMAX, PR>(A, B, rsd, q, c);
}

// tile_elim with a runtime KMAX (0..16): one instantiation per value, a uniform switch
// that folds away when kmax is a compile-time constant after inlining.
template <bool PR = false>
__device__ __forceinline__ void tile_elim_rt(int kmax, gs_d4& A, gs_d4& B, double& rsd, int q, int c) {
  switch (kmax) {
#define GS_TE(K) \
  case K: tile_elim<K, PR>(A, B, rsd, q, c); return;
    GS_TE(0) GS_TE(1) GS_TE(2) GS_TE(3) GS_TE(4) GS_TE(5) GS_TE(6) GS_TE(7)
    GS_TE(8) GS_TE(9) GS_TE(10) GS_TE(11) GS_TE(12) GS_TE(13) GS_TE(14) GS_TE(15)
#undef GS_TE
    default: tile_elim<16, PR>(A, B, rsd, q, c); return;
  }
}

namespace gtile {
// register i (runtime, 0..3) of a C-layout tile without a dynamically indexed vector
__device__ __forceinline__ double d4_get(const gs_d4 v, int i) {
  double r = v[0];
  r = (i == 1) ? v[1] : r;
  r = (i == 2) ? v[2] : r;
  r = (i == 3) ? v[3] : r;
  return r;
}

// v + a on the four diagonal lanes of register S of a C-layout tile (lane 16q + c with
// c = 4S + q), v elsewhere: exec set by two SALU moves around one v_add_f64 (instead of two
// v_cndmask_b32 and an add per register)
template <int S>
__device__ __forceinline__ double add_on_diag(double v, double a) {
  constexpr unsigned LO = (1u << (4 * S)) | (1u << (17 + 4 * S));     // q = 0, 1
  constexpr unsigned HI = (1u << (4 * S + 2)) | (1u << (19 + 4 * S));  // q = 2, 3
  asm("s_mov_b32 exec_lo, %2\n\t"
      "s_mov_b32 exec_hi, %3\n\t"
      "v_add_f64 %0, %0, %1\n\t"
      "s_mov_b64 exec, -1"
      : "+v"(v)
      : "v"(a), "n"(LO), "n"(HI));
  return v;
}
__device__ __forceinline__ double add_on_diag(double v, double a, int s) {
  switch (s) {  // s constant after unrolling
    case 0: return add_on_diag<0>(v, a);
    case 1: return add_on_diag<1>(v, a);
    case 2: return add_on_diag<2>(v, a);
    default: return add_on_diag<3>(v, a);
  }
}
}  // namespace gtile

// A pulsar's model block in the register-tile layout (gibbs_internal.h model_tiled_*), built
// once per fused-sweep launch in LDS (gibbs_bdraw.hip stage_model_tiled): every tile element a
// lane needs sits at lane + 64 (4 tile + register), so the per-draw loads are lane-linear with
// immediate offsets -- no per-element address arithmetic, no exec branches for the ragged edges,
// no bank conflicts.  S: the augmented Schur block with dF on its first padding row/column and
// 1 on the padding diagonal (phiinv_F is added on the real diagonal); G: -G, zero beyond nM rows
// / NF columns; R: zero beyond nM.
struct ModelTiled {
  static constexpr bool tiled = true;
  const double* S;
  const double* G;  // G' tiles, or row-major G (NMX x (NF+1)) when !fixt
  const double* R;  // R' tiles, or row-major R (NMX x NMX) when !fixt
  const double* h;
  bool fixt = true;  // fixed block in tiles (NMX <= 16, model_tiled_fix)
  const double* S0 = nullptr;  // unused (the row-major fields of ModelLds)
  const double* dF = nullptr;
};
template <typename ModelT>
struct model_is_tiled {
  static constexpr bool value = false;
};
template <>
struct model_is_tiled<ModelTiled> {
  static constexpr bool value = true;
};

// Model block view (see gibbs_bdraw.hip ModelLds): S0 NF x (NF+1), dF, G NMX x (NF+1),
// h, R NMX x NMX.  Same interface and outputs as bdraw_wave.
// LNL = true (the marginalised likelihood, gs_lnlike_marg): stop after the factorisation
// and return, wave-uniform, bF = |y|^2 = dF^T S^-1 dF and bM = log det S (sum of the log
// pivots of the real columns).
//
// NT tile rows with NF < 16 NT, so the augmented row/column always fits in the last tile
// (CP = NF - 16 (NT - 1) <= 15).  NF is a function argument: the fixed-NF entry point
// bdraw_tile<NF> passes a constant (everything folds as before); bdraw_tile_n<NT> serves
// any even NF < 16 NT with one instantiation per tile count.
//
// WIDE (64 < nM <= 128 timing-model columns, gs_bdraw only): z_M rows 64..127 arrive in zMa
// (lane l holds row 64 + l), the R z_M operand is staged in tb, and rows >= 64 of x_M are
// stored straight to bext[mrow[row]] (rows < 64 still return in bM, one per lane).
// PR: the issue-priority raises of GS_DIAG_PRIO / GS_SOLVE_PRIO (the persistent fused sweep
// only: in the short-lived k_bdraw waves at 3 waves/SIMD they cost 25 %).
// The likelihood terms of a factorised system from the wave's LDS scratch: lane l < NF holds y_l
// (U^T y = dF) at tb[128 + l] and the pivot^-1/2 of column l at tb[l] (bdraw_tile_core, LNL != 0);
// |y|^2 = sum y_l^2 and log det S = sum -2 log(pivot^-1/2), one term per lane, wave-summed in one
// fixed order.  The draw (after its solves) and the likelihood mode run the same code: bit-identical.
// The logs are gs_log_pos (0.77 ulp, ~35 VALU) rather than libm's (~90): with the phiinv term below
// they were about a fifth of a likelihood-mode factorisation's VALU (k_hyper_mh, r05).
__device__ __forceinline__ void lnl_terms(const double* tb, int lane, int NF, double& yy, double& lp) {
  const double y = lane < NF ? tb[128 + lane] : 0.0;
  yy = y * y;
  lp = lane < NF ? -2.0 * gs_log_lnl(tb[lane]) : 0.0;  // (a failed pivot's lane: the caller returns -inf)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    yy += __shfl_xor(yy, o);
    lp += __shfl_xor(lp, o);
  }
}

// LNL: 0 the draw; 1 the likelihood terms only (bF = |y|^2, bM = log det S, no solves); 2 the draw,
// leaving y and the pivots in the scratch for the caller's lnl_terms (tb is not touched after the
// factorisation on the draw's non-WIDE path).
template <int NT, int CPC, int LNL, bool WIDE = false, bool PR = false, typename ModelT>
__device__ __forceinline__ int bdraw_tile_core(const ModelT& M, int NMX, int nM, int lane, double phinv,
                                               double zF, double zM, double& bF, double& bM,
                                               double* __restrict__ scr, const int nf_rt, double zMa = 0.0,
                                               double* __restrict__ bext = nullptr,
                                               const int32_t* __restrict__ mrow = nullptr) {
  using namespace gtile;
  // CPC >= 0: NF = 16 (NT - 1) + CPC fixed at compile time; CPC < 0: NF = nf_rt
  const int NF = CPC >= 0 ? 16 * (NT - 1) + CPC : nf_rt;
  const int LD = NF + 1;
  constexpr bool TILED = model_is_tiled<ModelT>::value;
  static_assert(!(TILED && WIDE), "the tiled model block serves nM <= 64 only");
  constexpr int NTILE = NT * (NT + 1) / 2;
  const int q = lane >> 4, c = lane & 15;
  GS_PH_BEGIN
  double* tb = scr;        // 272
  double* vb = scr + 272;  // 64
  double* ob = scr + 336;  // 80

  // phinv_F and z_F (lane-row) -> column layout per tile row
  // z_F stays in ob (zero beyond NF) until the backward solve reads it back per tile row:
  // not held in registers through the factorisation
  lds_fence();
  vb[lane] = phinv;
  ob[lane] = (lane < NF) ? zF : 0.0;
  if (NT > 4 && lane < 16) ob[64 + lane] = 0.0;
  lds_fence();
  double phc[NT];
#pragma unroll
  for (int K = 0; K < NT; ++K) {
    const int i = 16 * K + c;
    phc[K] = (i < NF) ? vb[i] : (TILED ? 0.0 : 1.0);  // tiled: S' holds the padding's 1
  }
  lds_fence();

  // ---- S tiles (upper), C layout.  `z0` is an opaque 0: keeps the (sweep-invariant)
  // S0 loads inside the caller's sweep loop instead of hoisting 80 VGPRs out of it.
  int z0 = 0;
  asm volatile("" : "+s"(z0));
  // Augmented system: with NF % 16 != 0 the first padding row/column (index NF,
  // local column CP of the last tile) carries dF, so the factorisation of
  // [[S, dF], [dF^T, 1]] yields y = U^-T dF on the way (column CP of U_I,last for
  // I < last; row CP of the eliminated last diagonal tile scaled by the pivots^-1/2):
  // no forward solve.  S0 stores dF in its padding column NF (gs_prefix).
  constexpr bool AUG = true;
  const int CP = NF - 16 * (NT - 1);  // local index of the augmented column (0..15)
  gs_d4 t[NTILE];
  if constexpr (TILED) {
    // lane-linear loads at immediate offsets (ModelTiled), phiinv_F added on the diagonal lanes
    const double* Sl = M.S + lane + z0;
#pragma unroll
    for (int I = 0; I < NT; ++I) {
#pragma unroll
      for (int J = I; J < NT; ++J) {
        const int ti = tix(I, J, NT);
        gs_d4 v;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          v[s] = Sl[(4 * ti + s) * 64];
#if GS_EXEC_MASK
          if (I == J) v[s] = add_on_diag(v[s], phc[I], s);
#else
          if (I == J) v[s] += (4 * s + q == c) ? phc[I] : 0.0;
#endif
        }
        t[ti] = v;
      }
    }
  } else
#pragma unroll
  for (int I = 0; I < NT; ++I) {
#pragma unroll
    for (int J = I; J < NT; ++J) {
      gs_d4 v;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int r = 16 * I + 4 * s + q, col = 16 * J + c;
        // one LDS load per element: S0[r][col], or dF (S0's column NF) on the
        // augmented row/column of the last tile column
        int a = (r < NF && col < NF) ? r * LD + col : -1;
        if (AUG && J == NT - 1) {
          if (r < NF && col == NF) a = r * LD + NF;    // dF[r]
          if (r == NF && col < NF) a = col * LD + NF;  // dF[col]
        }
        double e = (a >= 0) ? M.S0[a + z0] : 0.0;
        if (I == J) e += (4 * s + q == c) ? phc[I] : 0.0;
        v[s] = e;
      }
      t[tix(I, J, NT)] = v;
    }
  }

  GS_PH(0)
  // ---- factorisation
  double ycol[NT];
  gs_d4 yrow[NT];
  int fail = 0;
  double ylast = 0.0;  // AUG: y of the last tile row, column layout
#pragma unroll
  for (int K = 0; K < NT; ++K) {
    // diag tile: column elimination on [T_KK ; I] -> B = E (unit upper), with
    // T_KK E lower triangular; U_KK^-1 = E diag(pivot^-1/2).  Column c of both
    // lives in lane column c, so the pivot scale is lane-local; A[r][k], B[r][k]
    // come from lane k of the same 16-lane row (DPP row_newbcast) and row k of A
    // from row group k&3 (permlane swaps): no LDS, no transpose.
    gs_d4 A = t[tix(K, K, NT)], B;
    double rsd;
    if (K == NT - 1) {
      if constexpr (CPC >= 0)
        tile_elim<CPC, PR>(A, B, rsd, q, c);
      else
        tile_elim_rt<PR>(CP, A, B, rsd, q, c);
    } else {
      tile_elim<16, PR>(A, B, rsd, q, c);
    }
    if (AUG && K == NT - 1) {
      // y_last[k] = (row CP of the eliminated tile)[k] * pivot_k^-1/2, k < CP
      const double yl = bcast_group_bp(CPC >= 0 ? A[(CPC >= 0 ? CPC : 0) >> 2] : d4_get(A, CP >> 2), CP & 3, c);
      ylast = (c < CP) ? yl * rsd : 0.0;
    }
    GS_PH(1)
    // first bad pivot of this tile (columns c of row group 0)
    const unsigned long long badm = __ballot(!(rsd > 0.0 && rsd < __builtin_inf())) & 0xffffull;
    if (!fail && badm) fail = 16 * K + __ffsll((long long)badm);
    gs_d4 V;  // U_KK^-1
#pragma unroll
    for (int s = 0; s < 4; ++s) V[s] = B[s] * rsd;
    t[tix(K, K, NT)] = V;
    if constexpr (PR && GS_UPD_PRIO > 0) __builtin_amdgcn_s_setprio(GS_UPD_PRIO);
    // TRSM: U_KJ = U_KK^-T T_KJ
#pragma unroll
    for (int J = K + 1; J < NT; ++J) {
      const gs_d4 z = {0.0, 0.0, 0.0, 0.0};
      t[tix(K, J, NT)] = mfma_tn(z, V, t[tix(K, J, NT)]);
    }
    // the backward solve wants U_KK^-T: transpose in place while the MFMAs run
    if constexpr (AUG) t[tix(K, K, NT)] = transpose(V, tb, q, c);
    // trailing update: T_IJ -= U_KI^T U_KJ
#pragma unroll
    for (int I = K + 1; I < NT; ++I) {
#pragma unroll
      for (int J = I; J < NT; ++J) t[tix(I, J, NT)] = mfma_tn_sub(t[tix(I, J, NT)], t[tix(K, I, NT)], t[tix(K, J, NT)]);
    }
    if constexpr (AUG) {
      // block row K is final: keep U_KJ^T (what the backward solve reads)
#pragma unroll
      for (int J = K + 1; J < NT; ++J) t[tix(K, J, NT)] = transpose(t[tix(K, J, NT)], tb, q, c);
    }
    if constexpr (PR && GS_UPD_PRIO > 0) __builtin_amdgcn_s_setprio(GS_BASE_PRIO);
    GS_PH(2)
  }

  // ---- forward: U^T y = dF   (y_K = U_KK^-T (dF_K - sum_{I<K} U_IK^T y_I))
  if constexpr (AUG) {
    // y_K = column CP of U_K,last = row CP of the stored U_K,last^T (row group CP&3)
#pragma unroll
    for (int K = 0; K + 1 < NT; ++K)
      ycol[K] = bcast_group_bp(CPC >= 0 ? t[tix(K, NT - 1, NT)][(CPC >= 0 ? CPC : 0) >> 2]
                                        : d4_get(t[tix(K, NT - 1, NT)], CP >> 2), CP & 3, c);
    ycol[NT - 1] = ylast;
  } else
#pragma unroll
  for (int K = 0; K < NT; ++K) {
    double p = 0.0;
#pragma unroll
    for (int I = 0; I < K; ++I)
#pragma unroll
      for (int s = 0; s < 4; ++s) p = fma(t[tix(I, K, NT)][s], yrow[I][s], p);
    if (K > 0) p = qsum(p);
    const int i = 16 * K + c;
    const double r = ((i < NF) ? M.dF[i + z0] : 0.0) - p;
    const gs_d4 rr = to_row(r, vb, q, c);
    double p2 = 0.0;
#pragma unroll
    for (int s = 0; s < 4; ++s) p2 = fma(t[tix(K, K, NT)][s], rr[s], p2);
    ycol[K] = qsum(p2);
    if (K + 1 < NT) yrow[K] = to_row(ycol[K], vb, q, c);
  }

  GS_PH(3)
  if constexpr (LNL) {
    static_assert(AUG && !WIDE, "the likelihood terms read y off the augmented factorisation");
    // y (column layout, row group 0) and the diagonal of each U_KK^-1 (= pivot^-1/2 exactly: the
    // eliminated B is unit upper), held by the lanes with q == c & 3 in register c >> 2
#pragma unroll
    for (int K = 0; K < NT; ++K) {
      const int i = 16 * K + c;
      if (q == 0 && i < NF) tb[128 + i] = ycol[K];
      if (q == (c & 3) && i < NF) tb[i] = d4_get(t[tix(K, K, NT)], c >> 2);
    }
    lds_fence();
    if constexpr (LNL == 1) {
      lnl_terms(tb, lane, NF, bF, bM);
      return fail;
    }
  }
  if constexpr (PR && GS_SOLVE_PRIO > 0) __builtin_amdgcn_s_setprio(GS_SOLVE_PRIO);
  // ---- backward: U x = y + zF   (x_K = U_KK^-1 (w_K - sum_{J>K} U_KJ x_J))
  double xcol[NT];
  gs_d4 xrow[NT];
#pragma unroll
  for (int K = NT - 1; K >= 0; --K) {
    double p = 0.0;
#pragma unroll
    for (int J = K + 1; J < NT; ++J) {
      const gs_d4 ut = AUG ? t[tix(K, J, NT)] : transpose(t[tix(K, J, NT)], tb, q, c);
#pragma unroll
      for (int s = 0; s < 4; ++s) p = fma(ut[s], xrow[J][s], p);
    }
    if (K + 1 < NT) p = qsum(p);
    const gs_d4 sr = to_row(ycol[K] + ob[16 * K + c] - p, vb, q, c);
    const gs_d4 W = AUG ? t[tix(K, K, NT)] : transpose(t[tix(K, K, NT)], tb, q, c);
    double p2 = 0.0;
#pragma unroll
    for (int s = 0; s < 4; ++s) p2 = fma(W[s], sr[s], p2);
    xcol[K] = qsum(p2);
    xrow[K] = to_row(xcol[K], vb, q, c);
  }
  lds_fence();
#pragma unroll
  for (int K = 0; K < NT; ++K) ob[16 * K + c] = xcol[K];
  lds_fence();
  bF = (lane < NF) ? ob[lane] : 0.0;
  lds_fence();

  if constexpr (PR && GS_SOLVE_PRIO > 0) __builtin_amdgcn_s_setprio(GS_BASE_PRIO);
  GS_PH(4)
  if constexpr (PR && GS_FIX_PRIO > 0) __builtin_amdgcn_s_setprio(GS_FIX_PRIO);
  // ---- fixed-prior block: x_M = h + R z_M - G x_F, 16 rows per chunk
  double* zb = WIDE ? tb : vb;  // z_M staging (tb is free after the factorisation)
  zb[lane] = (lane < nM) ? zM : 0.0;
  if constexpr (WIDE) zb[64 + lane] = (64 + lane < nM) ? zMa : 0.0;
  lds_fence();
  const int nP = (nM + 15) >> 4;
  for (int P = 0; P < nP; ++P) {
    const int row = 16 * P + c;
    const bool rok = row < nM;
    double p = 0.0;
    bool fixt = false;
    if constexpr (TILED) fixt = M.fixt;
    if (fixt) {
      // G' = -G and R' as C-layout tiles, zero beyond nM rows / NF columns (ModelTiled)
      const int nPl = (NMX + 15) >> 4;
      const double* Gl = M.G + lane + z0 + P * (NT * 256);
#pragma unroll
      for (int J = 0; J < NT; ++J)
#pragma unroll
        for (int s = 0; s < 4; ++s) p = fma(Gl[(4 * J + s) * 64], xrow[J][s], p);
      const double* Rl = M.R + lane + z0 + (P * nPl - (P * (P - 1)) / 2) * 256;
      for (int Q = P; Q < nP; ++Q)
#pragma unroll
        for (int s = 0; s < 4; ++s) p = fma(Rl[(4 * (Q - P) + s) * 64], zb[16 * Q + 4 * s + q], p);
    } else {
#pragma unroll
    for (int J = 0; J < NT; ++J)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int f = 16 * J + 4 * s + q;
        const double g = (rok && f < NF) ? M.G[row * LD + f + z0] : 0.0;
        p = fma(-g, xrow[J][s], p);
      }
    for (int Q = P; Q < nP; ++Q)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int mm = 16 * Q + 4 * s + q;
        const double rv = (rok && mm < nM) ? M.R[row * NMX + mm + z0] : 0.0;
        p = fma(rv, zb[mm], p);
      }
    }
    p = qsum(p);
    const double xm = rok ? M.h[row + z0] + p : 0.0;
    if (!WIDE || P < 4)
      ob[row] = xm;
    else if (rok && q == 0 && !fail)  // a failed draw leaves the caller's b untouched
      bext[mrow[row]] = xm;
  }
  lds_fence();
  bM = (lane < nM) ? ob[lane] : 0.0;
  lds_fence();
  if constexpr (PR && GS_FIX_PRIO > 0) __builtin_amdgcn_s_setprio(GS_BASE_PRIO);
  GS_PH(5)
  return fail;
}

// Fixed NF (the tuned 20 / 40 / 60 instantiations); NF % 16 != 0.
template <int NF, int LNL = 0, bool PR = false, typename ModelT>
__device__ __forceinline__ int bdraw_tile(const ModelT& M, int NMX, int nM, int lane, double phinv,
                                          double zF, double zM, double& bF, double& bM,
                                          double* __restrict__ scr) {
  static_assert(NF % 16 != 0, "the augmented column needs a free slot in the last tile");
  return bdraw_tile_core<(NF + 15) / 16, NF % 16, LNL, false, PR>(M, NMX, nM, lane, phinv, zF, zM, bF, bM, scr,
                                                                  NF);
}

// Any even NF with NF / 16 + 1 == NT (NF <= 64: one lane per free-spectrum column).
template <int NT, int LNL = 0, bool PR = false, typename ModelT>
__device__ __forceinline__ int bdraw_tile_n(const ModelT& M, int NMX, int nM, int lane, double phinv,
                                            double zF, double zM, double& bF, double& bM,
                                            double* __restrict__ scr, int NF) {
  return bdraw_tile_core<NT, -1, LNL, false, PR>(M, NMX, nM, lane, phinv, zF, zM, bF, bM, scr, NF);
}

// Same with up to 128 timing-model columns (see bdraw_tile_core, WIDE).
template <int NT, typename ModelT>
__device__ __forceinline__ int bdraw_tile_wide(const ModelT& M, int NMX, int nM, int lane, double phinv,
                                               double zF, double zM, double zMa, double& bF, double& bM,
                                               double* __restrict__ scr, int NF, double* bext,
                                               const int32_t* mrow) {
  return bdraw_tile_core<NT, -1, 0, true>(M, NMX, nM, lane, phinv, zF, zM, bF, bM, scr, NF, zMa, bext, mrow);
}
