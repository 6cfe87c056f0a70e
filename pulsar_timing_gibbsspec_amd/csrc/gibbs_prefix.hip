// TNT/d and the fixed-prior prefix in double-double.
//
// Reference: PulsarBlockGibbs.update_b forms TNT = T^T N^-1 T and d = T^T N^-1 r
// (pulsar_gibbs.py:500-502, pta_gibbs.py:523-526) and factorises Sigma = TNT + diag(phiinv)
// (:505-509) in fp64 on every draw.  The device factorises the timing-model block once
// (phiinv_M is constant) and per draw only the NF x NF Schur block
// S = S0 + diag(phiinv_F), S0 = A_FF - W^T W, W = L_M^-1 A_MF (the gs_prefix outputs).
//
// Why double-double here (tools/accuracy_sim.py, profiles/r03a/accuracy_sim.txt): the
// draw's distance from the exact (long-double) draw is set by two fp64 roundings that
// happen BEFORE the per-draw factorisation, not by the factorisation itself:
//  * TNT rounded to fp64: |TNT| is dominated by the timing-model directions, so a
//    relative 1e-16 rounding of its entries is a much larger relative perturbation of
//    the Schur block S0 (configs[4] at 10^4 TOAs: 8.7e-10 from exact on its own);
//  * S0 = A_FF - W^T W in fp64 cancels 2-3 digits (the timing model absorbs most of
//    A_FF): 2.6e-9 from exact at configs[4] with an fp64 prefix.
// With TNT/d carried as (hi, lo) pairs from exact products and the prefix in
// double-double, the unchanged fp64 tile draw is 1.4e-12 from exact at configs[4]
// (numpy/LAPACK on the same inputs: 1.2e-9).  Both kernels run once per noise state
// (once per run in configs 1-4), so their cost is off the sweep's critical path.
#include "gibbs_dd.h"
#include "gibbs_internal.h"

namespace {

// ------------------------------------------------------------------ TNT, d (a2)
// w_t = 1/N_t as a double-double: w_hi = fl(1/N), w_lo = fl((1 - N w_hi) / N) with the
// residual 1 - N w_hi exact by fma.
__device__ __forceinline__ gs_dd recip_dd(double N) {
  const double w = 1.0 / N;
  return {w, fma(-N, w, 1.0) / N};
}

constexpr int TNT_CHUNK = 64;  // TOAs staged per step

// grid (n_psr, nb (nb + 1) / 2): upper 16 x 16 blocks (bi <= bj) of TNT; thread (i, j) =
// (tid & 15, tid >> 4) accumulates D[i][j] = sum_t (T[t][I0+i] w_t) T[t][J0+j] with exact
// products (Dot2) and writes it to both triangles (TNT exactly symmetric).
__global__ __launch_bounds__(256) void k_tnt_dd(const gs_tnt_desc* desc, int nb, const double* T,
                                                const double* Nv, double* TNT, double* TNT_lo) {
  __shared__ double uh[TNT_CHUNK][17], ul[TNT_CHUNK][17], tj[TNT_CHUNK][17];
  const gs_tnt_desc D = desc[blockIdx.x];
  // upper-triangular block index -> (bi, bj)
  int bi = 0, rem = blockIdx.y;
  while (rem >= nb - bi) {
    rem -= nb - bi;
    ++bi;
  }
  const int bj = bi + rem;
  const int m = (int)D.m;
  if (bi * 16 >= m || bj * 16 >= m) return;  // whole workgroup: no barrier below is skipped by part
  const int tid = threadIdx.x, i = tid & 15, j = tid >> 4;
  const double* Tp = T + D.T_off;
  const double* Np = Nv + D.toa_off;
  const int64_t n = D.n_toa;
  gs_dot2 acc;
  for (int64_t t0 = 0; t0 < n; t0 += TNT_CHUNK) {
    __syncthreads();
    for (int q = tid; q < TNT_CHUNK * 16; q += 256) {
      const int tt = q >> 4, cc = q & 15;
      const int64_t t = t0 + tt;
      const int ci = bi * 16 + cc, cj = bj * 16 + cc;
      gs_dd u = {0.0, 0.0};
      double v = 0.0;
      if (t < n) {
        if (ci < m) u = dd_mul_d(recip_dd(Np[t]), Tp[t * m + ci]);
        if (cj < m) v = Tp[t * m + cj];
      }
      uh[tt][cc] = u.hi;
      ul[tt][cc] = u.lo;
      tj[tt][cc] = v;
    }
    __syncthreads();
#pragma unroll 8
    for (int tt = 0; tt < TNT_CHUNK; ++tt) acc.fma_ddd(gs_dd{uh[tt][i], ul[tt][i]}, tj[tt][j]);
  }
  const int row = bi * 16 + i, col = bj * 16 + j;
  if (row < m && col < m && (bi < bj || i <= j)) {  // diagonal blocks: thread (i <= j) writes both
    const gs_dd v = acc.get();
    const int64_t o1 = D.tnt_off + (int64_t)row * m + col, o2 = D.tnt_off + (int64_t)col * m + row;
    TNT[o1] = v.hi;
    TNT[o2] = v.hi;
    if (TNT_lo) {
      TNT_lo[o1] = v.lo;
      TNT_lo[o2] = v.lo;
    }
  }
}

// d = T^T (r / N): grid (n_psr, ceil(m / 64)), column j = lane, 4 waves split the TOAs.
__global__ __launch_bounds__(256) void k_tnr_dd(const gs_tnt_desc* desc, const double* T, const double* Nv,
                                                const double* r, double* d, double* d_lo) {
  __shared__ double red[2][4][64];
  const gs_tnt_desc D = desc[blockIdx.x];
  const int w = gs_wave_id(), l = threadIdx.x & 63;
  const int m = (int)D.m;
  const int j = blockIdx.y * 64 + l;
  gs_dot2 acc;
  if (j < m) {
    const double* Tp = T + D.T_off;
    const double* rp = r + D.toa_off;
    const double* Np = Nv + D.toa_off;
    for (int64_t t = w; t < D.n_toa; t += 4) acc.fma_ddd(dd_mul_d(recip_dd(Np[t]), rp[t]), Tp[t * m + j]);
  }
  const gs_dd v = acc.get();
  red[0][w][l] = v.hi;
  red[1][w][l] = v.lo;
  __syncthreads();
  if (w == 0 && j < m) {
    gs_dd s = {red[0][0][l], red[1][0][l]};
    for (int u = 1; u < 4; ++u) s = dd_add(s, gs_dd{red[0][u][l], red[1][u][l]});
    d[D.d_off + j] = s.hi;
    if (d_lo) d_lo[D.d_off + j] = s.lo;
  }
}

// ------------------------------------------------------------------ prefix
// One 256-thread workgroup per system (p, c).  Scratch (doubles): Lh, Ll [NMX x NMX] (L_M in
// double-double; Ll later holds R = L_M^-T), Wh, Wl [NMX x (NF+1)] (W = L_M^-1 A_MF and, in
// column NF, e = L_M^-1 d_M), in LDS when it fits, else in a context workspace slice (the
// same code through generic pointers; __syncthreads orders both at workgroup scope).
//
// Outputs (gs_prefix layout, rounded to fp64): S0 = A_FF - W^T W and dF = d_F - W^T e in
// double-double; G = R W, h = R e, R in fp64 from the rounded L_M and W (x_M = h + R z_M -
// G x_F is not cancellation-limited: tools/accuracy_sim.py FP64_GHR); aux = sum log diag L_M,
// |e|^2.
__global__ __launch_bounds__(256) void k_prefix_dd(PrefixArgs a) {
  extern __shared__ double sm[];
  const int sys = blockIdx.x;
  const int p = sys / a.n_chain, c = sys % a.n_chain;
  const gs_prefix_desc D = a.desc[p];
  const int NF = a.NF, NMX = a.NMX, ldw = NF + 1;
  const int m = (int)D.m, nM = (int)D.n_fixed;
  const int64_t toff = D.tnt_off + (int64_t)c * a.tnt_cstride, doff = D.d_off + (int64_t)c * a.d_cstride;
  const double* A = a.TNT + toff;
  const double* Al = a.TNT_lo ? a.TNT_lo + toff : nullptr;
  const double* dv = a.d + doff;
  const double* dl = a.d_lo ? a.d_lo + doff : nullptr;
  const int32_t* Fi = a.fidx + (int64_t)p * NF;
  const int32_t* Mi = a.midx + (int64_t)p * NMX;
  double* scr = a.gscr ? a.gscr + (int64_t)sys * a.gstride : sm;
  double* Lh = scr;
  double* Ll = Lh + NMX * NMX;
  double* Wh = Ll + NMX * NMX;
  double* Wl = Wh + NMX * ldw;
  double* Rm = Ll;  // after W and S0 are done
  __shared__ int s_fail;
  const int tid = threadIdx.x, nt = blockDim.x;
  auto ldA = [&](int r, int col) -> gs_dd {
    const int64_t q = (int64_t)r * m + col;
    return {A[q], Al ? Al[q] : 0.0};
  };
  auto ldd = [&](int r) -> gs_dd { return {dv[r], dl ? dl[r] : 0.0}; };
  auto L = [&](int i, int j) -> gs_dd { return {Lh[i * NMX + j], Ll[i * NMX + j]}; };

  __shared__ double rinv[2 * GS_NMX_WIDE];  // 1 / L_kk (double-double): divisions become products
  if (tid == 0) s_fail = 0;
  for (int q = tid; q < NMX * NMX; q += nt) {
    const int i = q / NMX, j = q % NMX;
    gs_dd v = {0.0, 0.0};
    if (i < nM && j <= i) {
      v = ldA(Mi[i], Mi[j]);
      if (i == j) v = dd_add_d(v, a.phfix[(int64_t)p * NMX + i]);
    }
    Lh[q] = v.hi;
    Ll[q] = v.lo;
  }
  __syncthreads();
  // right-looking Cholesky A_MM = L L^T (lower) in double-double
  for (int k = 0; k < nM; ++k) {
    if (tid == 0) {
      const gs_dd piv = L(k, k);
      if (!(piv.hi > 0.0) && s_fail == 0) s_fail = k + 1;
      const gs_dd s = dd_sqrt(piv);
      Lh[k * NMX + k] = s.hi;
      Ll[k * NMX + k] = s.lo;
      const gs_dd ri = dd_div(gs_dd{1.0, 0.0}, s);
      rinv[2 * k] = ri.hi;
      rinv[2 * k + 1] = ri.lo;
    }
    __syncthreads();
    const gs_dd rk = {rinv[2 * k], rinv[2 * k + 1]};
    for (int i = k + 1 + tid; i < nM; i += nt) {
      const gs_dd v = dd_mul(L(i, k), rk);
      Lh[i * NMX + k] = v.hi;
      Ll[i * NMX + k] = v.lo;
    }
    __syncthreads();
    const int len = nM - k - 1;
    for (int q = tid; q < len * len; q += nt) {
      const int i = k + 1 + q / len, j = k + 1 + q % len;
      if (j <= i) {
        const gs_dd v = dd_sub(L(i, j), dd_mul(L(i, k), L(j, k)));
        Lh[i * NMX + j] = v.hi;
        Ll[i * NMX + j] = v.lo;
      }
    }
    __syncthreads();
  }
  // W = L_M^-1 A_MF (columns < NF) and e = L_M^-1 d_M (column NF): column f by thread f
  for (int f = tid; f <= NF; f += nt) {
    for (int i = 0; i < nM; ++i) {
      gs_dot2 s;
      s.init(f < NF ? ldA(Mi[i], Fi[f]) : ldd(Mi[i]));
      for (int j = 0; j < i; ++j) s.fma_dd(dd_neg(L(i, j)), gs_dd{Wh[j * ldw + f], Wl[j * ldw + f]});
      const gs_dd w = dd_mul(s.get(), gs_dd{rinv[2 * i], rinv[2 * i + 1]});
      Wh[i * ldw + f] = w.hi;
      Wl[i * ldw + f] = w.lo;
    }
  }
  __syncthreads();
  double* out = a.model + (int64_t)sys * a.mstride;
  double* S0 = out;
  double* dF = S0 + NF * (NF + 1);
  double* G = dF + NF;
  double* h = G + NMX * (NF + 1);
  double* R = h + NMX;
  // S0 (upper triangle computed, mirrored: exactly symmetric) and its padding column NF = dF:
  // the NF (NF + 3) / 2 pairs f <= g <= NF enumerated row by row (row f: NF + 1 - f entries)
  const int Lr = NF + 1, n_up = NF * (NF + 3) / 2;
  for (int q = tid; q < n_up; q += nt) {
    // f = the row whose offset f Lr - f (f - 1) / 2 is the last one <= q
    const double B = 2.0 * Lr + 1.0;
    int f = (int)((B - sqrt(B * B - 8.0 * q)) * 0.5);
    auto off = [&](int r) { return r * Lr - (r * (r - 1)) / 2; };
    if (f > 0 && off(f) > q) --f;
    if (off(f + 1) <= q) ++f;
    const int g = f + (q - off(f));
    gs_dot2 s;
    s.init(g < NF ? ldA(Fi[f], Fi[g]) : ldd(Fi[f]));
    for (int i = 0; i < nM; ++i)
      s.fma_dd(gs_dd{-Wh[i * ldw + f], -Wl[i * ldw + f]}, gs_dd{Wh[i * ldw + g], Wl[i * ldw + g]});
    const double v = s.get().hi;
    S0[f * (NF + 1) + g] = v;
    if (g < NF) S0[g * (NF + 1) + f] = v;
    else dF[f] = v;
  }
  if (tid == 0) {
    double lm = 0.0;
    gs_dot2 ee;
    for (int i = 0; i < nM; ++i) {
      lm += dd_log(L(i, i));
      const gs_dd e = {Wh[i * ldw + NF], Wl[i * ldw + NF]};
      ee.fma_dd(e, e);
    }
    const int64_t ao = model_aux_offset(NF, NMX);
    out[ao] = lm;
    out[ao + 1] = ee.get().hi;
    if (a.info) a.info[sys] = s_fail;
  }
  __syncthreads();  // Ll is overwritten by R below
  // R = L_M^-T (upper) from the rounded L_M: column j by thread j, rows bottom-up
  for (int j = tid; j < NMX; j += nt) {
    for (int i = NMX - 1; i >= 0; --i) {
      double s = 0.0;
      if (i < nM && j < nM) {
        s = (i == j) ? 1.0 : 0.0;
        for (int q = i + 1; q < nM; ++q) s = fma(-Lh[q * NMX + i], Rm[q * NMX + j], s);
        s /= Lh[i * NMX + i];
      }
      Rm[i * NMX + j] = s;
    }
  }
  __syncthreads();
  for (int q = tid; q < NMX * (NF + 1); q += nt) {
    const int mm = q / (NF + 1), f = q % (NF + 1);
    double s = 0.0;
    if (f < NF)
      for (int j = mm; j < nM; ++j) s = fma(Rm[mm * NMX + j], Wh[j * ldw + f], s);
    G[q] = s;
  }
  for (int mm = tid; mm < NMX; mm += nt) {
    double s = 0.0;
    for (int j = mm; j < nM; ++j) s = fma(Rm[mm * NMX + j], Wh[j * ldw + NF], s);
    h[mm] = s;
  }
  for (int q = tid; q < NMX * NMX; q += nt) R[q] = Rm[q];
  for (int64_t q = model_aux_offset(NF, NMX) + 2 + tid; q < a.mstride; q += nt) out[q] = 0.0;
}

}  // namespace

int64_t prefix_scratch_doubles(int NF, int NMX) {
  return 2 * (int64_t)NMX * NMX + 2 * (int64_t)NMX * (NF + 1);
}

// dynamic LDS next to the kernel's 2 KB of static LDS (rinv, s_fail)
bool prefix_scratch_in_lds(int NF, int NMX) { return prefix_scratch_doubles(NF, NMX) * 8 <= 156 * 1024; }

hipError_t launch_prefix_dd(hipStream_t s, const PrefixArgs& a) {
  const int64_t n_sys = (int64_t)a.n_psr * a.n_chain;
  const size_t lds = a.gscr ? 0 : (size_t)prefix_scratch_doubles(a.NF, a.NMX) * sizeof(double);
  if (lds > 64 * 1024) {
    const hipError_t e =
        hipFuncSetAttribute((const void*)k_prefix_dd, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_prefix_dd, dim3((unsigned)n_sys), dim3(256), lds, s, a);
  return hipGetLastError();
}

hipError_t launch_tnt_dd(hipStream_t s, int n_psr, int m_max, const gs_tnt_desc* desc, const double* T,
                         const double* Nvec, const double* r, double* TNT, double* TNT_lo, double* d, double* d_lo) {
  const int nb = (m_max + 15) / 16;
  if (TNT) {
    hipLaunchKernelGGL(k_tnt_dd, dim3(n_psr, nb * (nb + 1) / 2), dim3(256), 0, s, desc, nb, T, Nvec, TNT, TNT_lo);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (d) {
    hipLaunchKernelGGL(k_tnr_dd, dim3(n_psr, (m_max + 63) / 64), dim3(256), 0, s, desc, T, Nvec, r, d, d_lo);
    return hipGetLastError();
  }
  return hipSuccess;
}
