// Paired-layout helpers of the two-chains-per-wave probes (pair_elim_probe.hip, pair_fact_probe.hip):
// two chains' 16 x 16 tiles in one register set -- lanes 0..31 chain a, 32..63 chain b, register 2s + j
// holding row 4s + 2j + h at lane 32X + 16h + c -- entered and left by v_permlane32_swap.
#pragma once
#include "../../pulsar_timing_gibbsspec_amd/csrc/gibbs_tile.h"

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

// tile_elim1's column elimination on two chains at once (paired layout; see the file comment)
template <int KMAX>
__device__ __forceinline__ void tile_elim_pair(double (&A)[8], double (&B)[8], double& rsd, int lane) {
  using namespace gtile;
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
      const double akm = zero_cols_le(akc, k);
      const double i0 = __builtin_amdgcn_rcp(akk);
      const double ng = (akm * i0) * fma(akk, i0, -2.0);
      akc = fmac_nb(rn, rn, ng, k);
#pragma unroll
      for (int t = 2 * k1; t < 8; ++t) A[t] = fmac_nb(A[t], A[t], ng, k);
#pragma unroll
      for (int t = 0; t <= 2 * k1 + 1; ++t) B[t] = fmac_nb(B[t], B[t], ng, k);
    }
  }
  double dg = A[0];
#pragma unroll
  for (int t = 1; t < 8; ++t) dg = (ptk(c) == t) ? A[t] : dg;
  double piv = bcast_lane_bp(dg, base + 16 * (c & 1) + c);
  if (KMAX < 16) piv = (c >= KMAX) ? 1.0 : piv;
  rsd = rsq_nr(piv);
}

