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

namespace gtile {

// compiler-level ordering of the wave's LDS traffic (the hardware executes a
// wave's DS instructions in order, so no s_barrier is needed)
__device__ __forceinline__ void lds_fence() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// acc + X^T Y for C-layout tiles X, Y
__device__ __forceinline__ gs_d4 mfma_tn(gs_d4 acc, const gs_d4 x, const gs_d4 y) {
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x[0], y[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x[1], y[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x[2], y[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x[3], y[3], acc, 0, 0, 0);
  return acc;
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

// Model block view (see gibbs_bdraw.hip ModelLds): S0 NF x (NF+1), dF, G NMX x (NF+1),
// h, R NMX x NMX.  Same interface and outputs as bdraw_wave.
template <int NF, typename ModelT>
__device__ __forceinline__ int bdraw_tile(const ModelT& M, int NMX, int nM, int lane, double phinv,
                                          double zF, double zM, double& bF, double& bM,
                                          double* __restrict__ scr) {
  using namespace gtile;
  constexpr int NT = (NF + 15) / 16;
  constexpr int LD = NF + 1;
  constexpr int NTILE = NT * (NT + 1) / 2;
  const int q = lane >> 4, c = lane & 15;
  double* tb = scr;        // 272
  double* vb = scr + 272;  // 64
  double* ob = scr + 336;  // 64

  // phinv_F and z_F (lane-row) -> column layout per tile row
  lds_fence();
  vb[lane] = phinv;
  ob[lane] = zF;
  lds_fence();
  double phc[NT], zfc[NT];
#pragma unroll
  for (int K = 0; K < NT; ++K) {
    const int i = 16 * K + c;
    phc[K] = (i < NF) ? vb[i] : 1.0;
    zfc[K] = (i < NF) ? ob[i] : 0.0;
  }
  lds_fence();

  // ---- S tiles (upper), C layout.  `z0` is an opaque 0: keeps the (sweep-invariant)
  // S0 loads inside the caller's sweep loop instead of hoisting 80 VGPRs out of it.
  int z0 = 0;
  asm volatile("" : "+s"(z0));
  gs_d4 t[NTILE];
#pragma unroll
  for (int I = 0; I < NT; ++I) {
#pragma unroll
    for (int J = I; J < NT; ++J) {
      gs_d4 v;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int r = 16 * I + 4 * s + q, col = 16 * J + c;
        double e = (r < NF && col < NF) ? M.S0[r * LD + col + z0] : 0.0;
        if (I == J) e += (4 * s + q == c) ? phc[I] : 0.0;
        v[s] = e;
      }
      t[tix(I, J, NT)] = v;
    }
  }

  // ---- factorisation
  int fail = 0;
#pragma unroll
  for (int K = 0; K < NT; ++K) {
    gs_d4 A = t[tix(K, K, NT)], B;
#pragma unroll
    for (int s = 0; s < 4; ++s) B[s] = (4 * s + q == c) ? 1.0 : 0.0;
    double rsd[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int k0 = k & 3, k1 = k >> 2;
      lds_fence();
      tb[q * 16 + c] = A[k1];
      tb[64 + q * 16 + c] = B[k1];
      lds_fence();
      const double akk = tb[k0 * 16 + k];
      const double akc = tb[k0 * 16 + c];
      const double bkc = tb[64 + k0 * 16 + c];
      double akr[4];
#pragma unroll
      for (int s = k1; s < 4; ++s) akr[s] = tb[k0 * 16 + 4 * s + q];
      lds_fence();
      const double rs = rsqrt(akk);
      const double inv = rs * rs;
      rsd[k1] = (q == k0) ? rs : rsd[k1];
      const double ga = akc * inv, gb = bkc * inv;
#pragma unroll
      for (int s = k1; s < 4; ++s) {
        const double cf = (s == k1) ? ((q > k0) ? akr[s] : 0.0) : akr[s];
        A[s] = fma(-cf, ga, A[s]);
        B[s] = fma(-cf, gb, B[s]);
      }
    }
    // W = U_KK^-T (row r scaled by 1/sqrt(pivot_r)); first bad pivot of this tile
    gs_d4 W;
    unsigned long long badrow = 0;  // bit r: pivot r not > 0
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      W[s] = B[s] * rsd[s];
      const unsigned long long bm = __ballot(!(rsd[s] > 0.0 && rsd[s] < __builtin_inf()));
#pragma unroll
      for (int qq = 0; qq < 4; ++qq)
        if ((bm >> (16 * qq)) & 0xffffull) badrow |= 1ull << (4 * s + qq);
    }
    if (!fail && badrow) fail = 16 * K + __ffsll((long long)badrow);
    const gs_d4 V = transpose(W, tb, q, c);  // U_KK^-1
    t[tix(K, K, NT)] = V;
    // TRSM: U_KJ = U_KK^-T T_KJ
#pragma unroll
    for (int J = K + 1; J < NT; ++J) {
      const gs_d4 z = {0.0, 0.0, 0.0, 0.0};
      t[tix(K, J, NT)] = mfma_tn(z, V, t[tix(K, J, NT)]);
    }
    // trailing update: T_IJ -= U_KI^T U_KJ
#pragma unroll
    for (int I = K + 1; I < NT; ++I) {
      const gs_d4 nx = -t[tix(K, I, NT)];
#pragma unroll
      for (int J = I; J < NT; ++J) t[tix(I, J, NT)] = mfma_tn(t[tix(I, J, NT)], nx, t[tix(K, J, NT)]);
    }
  }

  // ---- forward: U^T y = dF   (y_K = U_KK^-T (dF_K - sum_{I<K} U_IK^T y_I))
  double ycol[NT];
  gs_d4 yrow[NT];
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

  // ---- backward: U x = y + zF   (x_K = U_KK^-1 (w_K - sum_{J>K} U_KJ x_J))
  double xcol[NT];
  gs_d4 xrow[NT];
#pragma unroll
  for (int K = NT - 1; K >= 0; --K) {
    double p = 0.0;
#pragma unroll
    for (int J = K + 1; J < NT; ++J) {
      const gs_d4 ut = transpose(t[tix(K, J, NT)], tb, q, c);
#pragma unroll
      for (int s = 0; s < 4; ++s) p = fma(ut[s], xrow[J][s], p);
    }
    if (K + 1 < NT) p = qsum(p);
    const gs_d4 sr = to_row(ycol[K] + zfc[K] - p, vb, q, c);
    const gs_d4 W = transpose(t[tix(K, K, NT)], tb, q, c);
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

  // ---- fixed-prior block: x_M = h + R z_M - G x_F, 16 rows per chunk
  vb[lane] = (lane < nM) ? zM : 0.0;
  lds_fence();
  const int nP = (nM + 15) >> 4;
  for (int P = 0; P < nP; ++P) {
    const int row = 16 * P + c;
    const bool rok = row < nM;
    double p = 0.0;
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
        p = fma(rv, vb[mm], p);
      }
    p = qsum(p);
    ob[row] = rok ? M.h[row + z0] + p : 0.0;
  }
  lds_fence();
  bM = (lane < nM) ? ob[lane] : 0.0;
  lds_fence();
  return fail;
}
