// Two chains per wave vs one, measured on the part of the tile core the pairing
// would change: the diagonal-tile column elimination (gibbs_tile.h tile_elim1, 63 % of a draw's VALU).
//
//  single: one chain per wave, the production tile_elim1<16> on its 16x16 tile (4 + 4 registers in
//          the MFMA C layout: lane 16q + c holds row 4s + q in register s);
//  pair:   two chains per wave in the paired layout -- lanes 0..31 chain a, 32..63 chain b, register
//          2s + j holding row 4s + 2j + h at lane 32X + 16h + c -- so every pivot broadcast, v_rcp_f64,
//          Newton step and lane mask serves both chains; entered and left by v_permlane32_swap (16
//          32-bit swaps in for the tile, 16 out for U^-1, the MFMA layout the TRSM / update need).
//
// Each wave repeats the elimination REPS times on its chains' tiles (fixed SPD tiles, a chain-specific
// diagonal shift); occupancy (waves per SIMD) is set by the dynamic LDS each one-wave workgroup asks
// for.  Prints ns per chain-tile elimination for each (variant, waves/SIMD) and checks that both
// variants return bit-identical U^-1 for every chain.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 pair_elim_probe.hip -o pair_elim_probe  (make -C tools/probe)
#include <hip/hip_runtime.h>
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

// the tile of chain i: a fixed SPD 16 x 16 matrix (diagonally dominant) + i * 1e-3 on the diagonal
__device__ __forceinline__ double tile_elem(int r, int c, int i) {
  const double off = 1.0 / (1.0 + (double)((r * 7 + c * 3) % 11) + (double)(r > c ? r - c : c - r));
  return r == c ? 20.0 + 0.5 * r + 1e-3 * i : off;
}

__global__ void k_single(int reps, int n_chain, double* __restrict__ V, double* __restrict__ sink) {
  extern __shared__ double lds_pad[];  // occupancy control only
  const int lane = threadIdx.x, q = lane >> 4, c = lane & 15;
  const int i = blockIdx.x;
  if (i >= n_chain) return;
  gs_d4 A0;
#pragma unroll
  for (int s = 0; s < 4; ++s) A0[s] = tile_elem(4 * s + q, c, i);
  double acc = 0.0;
  gs_d4 Vs;
#pragma unroll 1
  for (int r = 0; r < reps; ++r) {
    gs_d4 A = A0, B;
    double rsd;
    tile_elim1<16>(A, B, rsd, q, c);
#pragma unroll
    for (int s = 0; s < 4; ++s) Vs[s] = B[s] * rsd;
    acc += Vs[0] + Vs[3];
    A0[0] += 0.0 * acc;  // loop-carried: the compiler cannot hoist the elimination
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) V[(int64_t)i * 256 + s * 64 + lane] = Vs[s];
  if (lane == 0) sink[i] = acc + lds_pad[0] * 0.0;
}

__global__ void k_pair(int reps, int n_chain, double* __restrict__ V, double* __restrict__ sink) {
  extern __shared__ double lds_pad[];
  const int lane = threadIdx.x, q = lane >> 4, c = lane & 15;
  const int ia = 2 * blockIdx.x, ib = ia + 1;
  if (ib >= n_chain) return;
  double Aa[4], Ab[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    Aa[s] = tile_elem(4 * s + q, c, ia);
    Ab[s] = tile_elem(4 * s + q, c, ib);
  }
  double acc = 0.0;
  double Va[4], Vb[4];
#pragma unroll 1
  for (int r = 0; r < reps; ++r) {
    double PA[8], PB[8];
#pragma unroll
    for (int s = 0; s < 4; ++s) {  // into the paired layout (the MFMA-layout tiles of both chains)
      PA[2 * s] = Aa[s];
      PA[2 * s + 1] = Ab[s];
      swap32(PA[2 * s], PA[2 * s + 1]);
    }
    double rsd;
    tile_elim_pair<16>(PA, PB, rsd, lane);
#pragma unroll
    for (int s = 0; s < 4; ++s) {  // U^-1 of both chains back to the MFMA layout
      double x = PB[2 * s] * rsd, y = PB[2 * s + 1] * rsd;
      swap32(x, y);
      Va[s] = x;
      Vb[s] = y;
    }
    acc += Va[0] + Vb[3];
    Aa[0] += 0.0 * acc;
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    V[(int64_t)ia * 256 + s * 64 + lane] = Va[s];
    V[(int64_t)ib * 256 + s * 64 + lane] = Vb[s];
  }
  if (lane == 0) sink[blockIdx.x] = acc + lds_pad[0] * 0.0;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 400;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const size_t lds_cu = prop.maxSharedMemoryPerMultiProcessor;
  printf("device %s, %d CUs, %zu B LDS per CU, reps %d\n", prop.name, cus, lds_cu, reps);
  const int n_chain = 4 * 4 * cus * 2;  // enough one-wave workgroups for 4 waves/SIMD, pairs or not
  double *V1, *V2, *sink;
  CHECK(hipMalloc(&V1, (size_t)n_chain * 256 * 8));
  CHECK(hipMalloc(&V2, (size_t)n_chain * 256 * 8));
  CHECK(hipMalloc(&sink, (size_t)n_chain * 8));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int variant = 0; variant < 2; ++variant) {
    for (int w = 1; w <= 3; ++w) {
      // w one-wave workgroups per SIMD: the LDS of a CU split over 4 w of them
      const size_t lds = lds_cu / (4 * w) - 1024;
      const int chains_per_wave = variant ? 2 : 1;
      const int blocks = 4 * w * cus;  // one round at w waves/SIMD
      const int nc = blocks * chains_per_wave;
      float best = 1e30f;
      for (int it = 0; it < 3; ++it) {
        CHECK(hipEventRecord(e0));
        if (variant == 0)
          hipLaunchKernelGGL(k_single, dim3(blocks), dim3(64), lds, 0, reps, nc, V1, sink);
        else
          hipLaunchKernelGGL(k_pair, dim3(blocks), dim3(64), lds, 0, reps, nc, V2, sink);
        CHECK(hipGetLastError());
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
      }
      const double per = best * 1e6 / ((double)nc * reps);  // ns per chain-tile elimination
      const double cyc = per * 1e-9 * 2.4e9 * 4 * cus;      // SIMD cycles per chain-tile (2.4 GHz)
      printf("%-6s waves/SIMD %d  chains %6d  %.3f ms  %.3f ns per chain-tile  %.0f SIMD cycles per chain-tile\n",
             variant ? "pair" : "single", w, nc, best, per, cyc);
    }
  }
  // correctness: U^-1 of the same chains from both variants (last runs: 3 waves/SIMD)
  const int nchk = 4 * 3 * cus;
  hipLaunchKernelGGL(k_single, dim3(nchk), dim3(64), 0, 0, 1, nchk, V1, sink);
  hipLaunchKernelGGL(k_pair, dim3(nchk / 2), dim3(64), 0, 0, 1, nchk, V2, sink);
  CHECK(hipDeviceSynchronize());
  double* h1 = (double*)malloc((size_t)nchk * 256 * 8);
  double* h2 = (double*)malloc((size_t)nchk * 256 * 8);
  CHECK(hipMemcpy(h1, V1, (size_t)nchk * 256 * 8, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(h2, V2, (size_t)nchk * 256 * 8, hipMemcpyDeviceToHost));
  long bad = 0;
  double maxd = 0.0;
  for (long j = 0; j < (long)nchk * 256; ++j) {
    const double d = h1[j] - h2[j];
    if (d != 0.0) ++bad;
    if (fabs(d) > maxd) maxd = fabs(d);
  }
  printf("U^-1 single vs pair over %d chains: %ld differing elements, max |diff| %.3g (V[0][0] = %.17g)\n", nchk, bad,
         maxd, h1[0]);
  return bad != 0;
}
