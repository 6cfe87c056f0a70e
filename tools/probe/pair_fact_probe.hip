// Two chains per wave vs one on the whole b|rho FACTORISATION of the headline's Schur block (NF = 60:
// NT = 4 tile rows, the last holding 12 columns + the augmented one): per tile row K the diagonal
// tile's column elimination, U_KK^-1, the 4-MFMA TRSM of the tiles right of it and the trailing
// MFMA updates -- the production bdraw_tile_core's factorisation loop (gibbs_tile.h), without the
// solves.  The S tiles come from LDS as in the fused sweep (one block shared by the workgroup's waves;
// phiinv added on the diagonal per chain).
//
//  single: one chain per wave (tile_elim1 on the diagonal tiles);
//  pair:   two chains per wave, both chains' 10 tiles in registers, the diagonal tiles eliminated
//          together in the paired layout (pair_tile.h), TRSM / updates per chain in the MFMA layout.
//
// 4-wave workgroups; waves per SIMD set by the workgroup's dynamic LDS (the 20 KB block + padding).
// Reports SIMD cycles per chain-factorisation at 1..3 waves/SIMD, the VGPR count of each kernel, and
// checks that both variants give bit-identical sums of the pivots^-1/2.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -pragma-unroll-threshold=1000000 pair_fact_probe.hip
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "pair_tile.h"

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                       \
    }                                                                                \
  } while (0)

constexpr int NT = 4, NTILE = NT * (NT + 1) / 2, CP = 12;  // NF = 60

// element (r, c) of a fixed SPD 64 x 64 block (identity beyond the 60 x 60 part; the augmented
// row/column 60 is left as identity here: the probe measures the factorisation's cost)
__device__ __forceinline__ double s_elem(int r, int c) {
  if (r >= 60 || c >= 60) return r == c ? 1.0 : 0.0;
  const double off = 0.3 / (1.0 + (double)(r > c ? r - c : c - r));
  return r == c ? 4.0 + 0.01 * r : off;
}

// the shared block in LDS: tile ti (upper, row-major over (I, J >= I)), register s, lane
__device__ void stage_block(double* L) {
  for (int e = threadIdx.x; e < NTILE * 256; e += blockDim.x) {
    const int ti = e / 256, s = (e / 64) % 4, lane = e % 64, q = lane >> 4, c = lane & 15;
    int I = 0, J = 0, t = ti;
    for (I = 0; I < NT; ++I) {
      if (t < NT - I) { J = I + t; break; }
      t -= NT - I;
    }
    L[e] = s_elem(16 * I + 4 * s + q, 16 * J + c);
  }
  __syncthreads();
}

// tiles of one chain from the shared block, phinv on the real diagonal (chain-specific)
__device__ __forceinline__ void load_tiles(gs_d4 (&t)[NTILE], const double* L, int lane, double ph) {
  const int q = lane >> 4, c = lane & 15;
#pragma unroll
  for (int I = 0; I < NT; ++I)
#pragma unroll
    for (int J = I; J < NT; ++J) {
      const int ti = gtile::tix(I, J, NT);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        double v = L[(4 * ti + s) * 64 + lane];
        if (I == J && 4 * s + q == c && 16 * I + c < 60) v += ph;
        t[ti][s] = v;
      }
    }
}

// TRSM of block row K and the trailing update (production order)
__device__ __forceinline__ void trsm_update(gs_d4 (&t)[NTILE], int K, const gs_d4 V) {
  using namespace gtile;
#pragma unroll
  for (int J = K + 1; J < NT; ++J) {
    const gs_d4 z = {0.0, 0.0, 0.0, 0.0};
    t[tix(K, J, NT)] = mfma_tn(z, V, t[tix(K, J, NT)]);
  }
#pragma unroll
  for (int I = K + 1; I < NT; ++I)
#pragma unroll
    for (int J = I; J < NT; ++J) t[tix(I, J, NT)] = mfma_tn_sub(t[tix(I, J, NT)], t[tix(K, I, NT)], t[tix(K, J, NT)]);
}

// the factorisation's per-pivot output, reduced with one add per tile (a log per pivot would cost the
// single variant twice what it costs the pair, which takes it once per lane for both chains)
__device__ __forceinline__ double logsum(double rsd, int lane, int K) {
  const int q = lane >> 4, c = lane & 15;
  return (q == 0 && 16 * K + c < 60) ? rsd : 0.0;
}

__global__ __launch_bounds__(256, 3) void k_single(int reps, int n_chain, double* __restrict__ out) {
  extern __shared__ double L[];
  stage_block(L);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, q = lane >> 4, c = lane & 15;
  const int i = blockIdx.x * 4 + wave;
  if (i >= n_chain) return;
  double acc = 0.0, last = 0.0;
#pragma unroll 1
  for (int r = 0; r < reps; ++r) {
    gs_d4 t[NTILE];
    load_tiles(t, L, lane, 0.5 + 1e-3 * i + 0.0 * acc);
    double ld = 0.0;
#pragma unroll
    for (int K = 0; K < NT; ++K) {
      gs_d4 A = t[gtile::tix(K, K, NT)], B;
      double rsd;
      if (K == NT - 1)
        tile_elim1<CP + 1>(A, B, rsd, q, c);
      else
        tile_elim1<16>(A, B, rsd, q, c);
      gs_d4 V;
#pragma unroll
      for (int s = 0; s < 4; ++s) V[s] = B[s] * rsd;
      t[gtile::tix(K, K, NT)] = V;
      trsm_update(t, K, V);
      ld += logsum(rsd, lane, K);
    }
    acc += ld;
    last = ld;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) last += __shfl_xor(last, o);
  if (lane == 0) out[i] = last + 0.0 * acc;
}

__global__ __launch_bounds__(256, 2) void k_pair(int reps, int n_chain, double* __restrict__ out) {
  extern __shared__ double L[];
  stage_block(L);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ia = 2 * (blockIdx.x * 4 + wave), ib = ia + 1;
  if (ib >= n_chain) return;
  double acca = 0.0, lasta = 0.0, lastb = 0.0;
#pragma unroll 1
  for (int r = 0; r < reps; ++r) {
    gs_d4 ta[NTILE], tb[NTILE];
    load_tiles(ta, L, lane, 0.5 + 1e-3 * ia + 0.0 * acca);
    load_tiles(tb, L, lane, 0.5 + 1e-3 * ib + 0.0 * acca);
    double lda = 0.0, ldb = 0.0;
#pragma unroll
    for (int K = 0; K < NT; ++K) {
      const int kk = gtile::tix(K, K, NT);
      double PA[8], PB[8];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        PA[2 * s] = ta[kk][s];
        PA[2 * s + 1] = tb[kk][s];
        swap32(PA[2 * s], PA[2 * s + 1]);
      }
      double rsd;
      if (K == NT - 1)
        tile_elim_pair<CP + 1>(PA, PB, rsd, lane);
      else
        tile_elim_pair<16>(PA, PB, rsd, lane);
      // rsd of the lane's chain (lanes 0..31 chain a) -> per-chain column values in the MFMA layout
      gs_d4 Va, Vb;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        double x = PB[2 * s] * rsd, y = PB[2 * s + 1] * rsd;
        swap32(x, y);
        Va[s] = x;
        Vb[s] = y;
      }
      // the log pivots: rsd at lanes 0..15 (chain a) and 32..47 (chain b), column c
      const int c = lane & 15;
      const double lp = (16 * K + c < 60 && (lane & 16) == 0) ? rsd : 0.0;
      lda += (lane < 32) ? lp : 0.0;
      ldb += (lane >= 32) ? lp : 0.0;
      ta[kk] = Va;
      tb[kk] = Vb;
      trsm_update(ta, K, Va);
      trsm_update(tb, K, Vb);
    }
    acca += lda + ldb;
    lasta = lda;
    lastb = ldb;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lasta += __shfl_xor(lasta, o);
    lastb += __shfl_xor(lastb, o);
  }
  if (lane == 0) {
    out[ia] = lasta + 0.0 * acca;
    out[ib] = lastb;
  }
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 200;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const size_t lds_cu = prop.maxSharedMemoryPerMultiProcessor;
  const size_t blk = (size_t)NTILE * 256 * 8;
  hipFuncAttributes fa;
  CHECK(hipFuncGetAttributes(&fa, (const void*)k_single));
  const int vs = fa.numRegs;
  CHECK(hipFuncGetAttributes(&fa, (const void*)k_pair));
  printf("%d CUs, %zu B LDS per CU, block %zu B, reps %d; VGPRs single %d, pair %d\n", cus, lds_cu, blk, reps, vs,
         fa.numRegs);
  const int n_max = 4 * 4 * cus * 2;
  double *o1, *o2;
  CHECK(hipMalloc(&o1, (size_t)n_max * 8));
  CHECK(hipMalloc(&o2, (size_t)n_max * 8));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int variant = 0; variant < 2; ++variant) {
    for (int w = 1; w <= 3; ++w) {
      // w 4-wave workgroups per CU = w waves per SIMD (if the registers allow it)
      size_t lds = lds_cu / w - 2048;
      if (lds < blk) lds = blk;
      if (lds > 65536) {  // > 64 KB dynamic LDS needs the attribute
        CHECK(hipFuncSetAttribute(variant ? (const void*)k_pair : (const void*)k_single,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      }
      const int blocks = w * cus;
      const int nc = blocks * 4 * (variant ? 2 : 1);
      float best = 1e30f;
      for (int it = 0; it < 3; ++it) {
        CHECK(hipEventRecord(e0));
        if (variant == 0)
          hipLaunchKernelGGL(k_single, dim3(blocks), dim3(256), lds, 0, reps, nc, o1);
        else
          hipLaunchKernelGGL(k_pair, dim3(blocks), dim3(256), lds, 0, reps, nc, o2);
        CHECK(hipGetLastError());
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
      }
      const double per = best * 1e6 / ((double)nc * reps);
      const double cyc = per * 1e-9 * 2.4e9 * 4 * cus;
      printf("%-6s requested waves/SIMD %d  chains %6d  %.3f ms  %.3f ns per chain-factorisation  %.0f SIMD cycles\n",
             variant ? "pair" : "single", w, nc, best, per, cyc);
    }
  }
  // correctness: the same chains' log-det sums from both variants
  const int nchk = 8 * cus;
  hipLaunchKernelGGL(k_single, dim3(nchk / 4), dim3(256), blk, 0, 1, nchk, o1);
  hipLaunchKernelGGL(k_pair, dim3(nchk / 8), dim3(256), blk, 0, 1, nchk, o2);
  CHECK(hipDeviceSynchronize());
  double* h1 = (double*)malloc((size_t)nchk * 8);
  double* h2 = (double*)malloc((size_t)nchk * 8);
  CHECK(hipMemcpy(h1, o1, (size_t)nchk * 8, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(h2, o2, (size_t)nchk * 8, hipMemcpyDeviceToHost));
  int bad = 0;
  double maxd = 0.0;
  for (int j = 0; j < nchk; ++j) {
    const double d = fabs(h1[j] - h2[j]);
    if (d > 0.0) ++bad;
    if (d > maxd) maxd = d;
  }
  printf("sum of pivots^-1/2, single vs pair, over %d chains: %d differ, max |diff| %.3g (chain 0: %.17g, finite %d)\n", nchk, bad,
         maxd, h1[0], (int)isfinite(h1[0]));
  return (bad != 0 || !isfinite(h1[0])) ? 1 : 0;
}
