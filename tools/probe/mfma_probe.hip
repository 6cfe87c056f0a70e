// Microbenchmark + layout probe for the f64 tile Cholesky design (gfx950).
//  1. D = X^T Y from two C-layout 16x16 tiles with 4 x v_mfma_f64_16x16x4f64
//     (A operand = reg s of X's C layout, B operand = reg s of Y's C layout).
//  2. ds_swizzle broadcast of lane k within each 16-lane row (and 0x10 | or k).
//  3. Throughput: f64 MFMA (4 independent chains), dependent-MFMA latency,
//     v_fma_f64, v_readlane_b32 + fma.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>

typedef double d4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void k_layout(const double* X, const double* Y, double* D, double* sw) {
  const int l = threadIdx.x;
  const int q = l >> 4, c = l & 15;
  d4 x, y, acc = {0, 0, 0, 0};
  for (int s = 0; s < 4; ++s) { x[s] = X[(4 * s + q) * 16 + c]; y[s] = Y[(4 * s + q) * 16 + c]; }
  for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x[s], y[s], acc, 0, 0, 0);
  for (int s = 0; s < 4; ++s) D[(4 * s + q) * 16 + c] = acc[s];
  // swizzle: broadcast lane 5 within each row of 16 (BitMode: and 0x10, or 5, xor 0)
  const int v = l * 10 + 1;
  const int pat = (0x10) | (5 << 5) | (0 << 10);
  sw[l] = __builtin_amdgcn_ds_swizzle(v, pat);
}

__global__ void k_mfma_tput(double* out, int iters) {
  const int l = threadIdx.x & 63;
  double a = 1.0 + l * 1e-3, b = 1.0 - l * 1e-3;
  d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, b, c3, 0, 0, 0);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
}

__global__ void k_mfma_lat(double* out, long long* cyc, int iters) {
  const int l = threadIdx.x & 63;
  double a = 1.0 + l * 1e-3, b = 1.0 - l * 1e-3;
  d4 c0 = {0, 0, 0, 0};
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
  long long t1 = clock64();
  out[threadIdx.x] = c0[0] + c0[3];
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_fma_tput(double* out, int iters) {
  const int l = threadIdx.x;
  double a0 = l, a1 = l + 1, a2 = l + 2, a3 = l + 3, a4 = l + 4, a5 = l + 5, a6 = l + 6, a7 = l + 7;
  const double m = 0.999999, k = 1e-7;
  for (int i = 0; i < iters; ++i) {
    a0 = fma(a0, m, k); a1 = fma(a1, m, k); a2 = fma(a2, m, k); a3 = fma(a3, m, k);
    a4 = fma(a4, m, k); a5 = fma(a5, m, k); a6 = fma(a6, m, k); a7 = fma(a7, m, k);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

// mixed: one wave stream of MFMA + independent VALU FMAs (does VALU overlap MFMA?)
__global__ void k_mixed(double* out, int iters) {
  const int l = threadIdx.x & 63;
  double a = 1.0 + l * 1e-3, b = 1.0 - l * 1e-3;
  d4 c0 = {0, 0, 0, 0}, c1 = c0;
  double a0 = l, a1 = l + 1, a2 = l + 2, a3 = l + 3;
  const double m = 0.999999, k = 1e-7;
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    a0 = fma(a0, m, k); a1 = fma(a1, m, k); a2 = fma(a2, m, k); a3 = fma(a3, m, k);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, c1, 0, 0, 0);
    a0 = fma(a0, m, k); a1 = fma(a1, m, k); a2 = fma(a2, m, k); a3 = fma(a3, m, k);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0[0] + c1[1] + a0 + a1 + a2 + a3;
}


// MFMA + b32 VALU (int xor/add): do 32-bit VALU ops overlap the f64 matrix pipe?
__global__ void k_mixed_int(double* out, int iters) {
  const int l = threadIdx.x & 63;
  double a = 1.0 + l * 1e-3, b = 1.0 - l * 1e-3;
  d4 c0 = {0, 0, 0, 0}, c1 = c0;
  unsigned u0 = l, u1 = l + 1, u2 = l + 2, u3 = l + 3;
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 4; ++r) { u0 = (u0 ^ 0x9e37u) + u1; u1 = (u1 ^ 0x7f4au) + u2; u2 = (u2 ^ 0x1234u) + u3; u3 = (u3 ^ 0x5555u) + u0; }
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, c1, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 4; ++r) { u0 = (u0 ^ 0x9e37u) + u1; u1 = (u1 ^ 0x7f4au) + u2; u2 = (u2 ^ 0x1234u) + u3; u3 = (u3 ^ 0x5555u) + u0; }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0[0] + c1[1] + (double)(u0 + u1 + u2 + u3);
}

__global__ void k_int_only(double* out, int iters) {
  const int l = threadIdx.x & 63;
  unsigned u0 = l, u1 = l + 1, u2 = l + 2, u3 = l + 3;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 8; ++r) { u0 = (u0 ^ 0x9e37u) + u1; u1 = (u1 ^ 0x7f4au) + u2; u2 = (u2 ^ 0x1234u) + u3; u3 = (u3 ^ 0x5555u) + u0; }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (double)(u0 + u1 + u2 + u3);
}

// readlane broadcast + fma (the current lane-per-row update)
__global__ void k_readlane_fma(double* out, int iters) {
  const int l = threadIdx.x & 63;
  double a[8];
  for (int j = 0; j < 8; ++j) a[j] = l + j;
  double f = 1e-9 * l;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const unsigned long long u = (unsigned long long)__double_as_longlong(a[(j + 1) & 7]);
      const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u & 0xffffffffull), (j * 7 + i) & 63);
      const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), (j * 7 + i) & 63);
      a[j] = fma(-f, __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo)), a[j]);
    }
  }
  double s = 0; for (int j = 0; j < 8; ++j) s += a[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename F>
float timeit(F f) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  f();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms;
}

int main() {
  // ---- layout
  double hX[256], hY[256], hD[256], hsw[64];
  srand(1);
  for (int i = 0; i < 256; ++i) { hX[i] = rand() / (double)RAND_MAX - 0.5; hY[i] = rand() / (double)RAND_MAX - 0.5; }
  double *dX, *dY, *dD, *dsw;
  CK(hipMalloc(&dX, 2048)); CK(hipMalloc(&dY, 2048)); CK(hipMalloc(&dD, 2048)); CK(hipMalloc(&dsw, 512));
  CK(hipMemcpy(dX, hX, 2048, hipMemcpyHostToDevice)); CK(hipMemcpy(dY, hY, 2048, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, 0, dX, dY, dD, dsw);
  CK(hipMemcpy(hD, dD, 2048, hipMemcpyDeviceToHost)); CK(hipMemcpy(hsw, dsw, 512, hipMemcpyDeviceToHost));
  double err = 0;
  for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) {
    double s = 0; for (int k = 0; k < 16; ++k) s += hX[k * 16 + i] * hY[k * 16 + j];
    err = fmax(err, fabs(s - hD[i * 16 + j]));
  }
  printf("layout D = X^T Y max err %.3e\n", err);
  int swok = 1;
  for (int l = 0; l < 64; ++l) { int src = (l & 0x30) | 5; if ((int)hsw[l] != src * 10 + 1) swok = 0; }
  printf("swizzle broadcast-in-16 %s (lane 17 got %g, lane 40 got %g)\n", swok ? "OK" : "MISMATCH", hsw[17], hsw[40]);
  // ---- throughput
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  const double clk = prop.clockRate * 1e3;
  printf("CUs %d clock %.0f MHz\n", ncu, clk / 1e6);
  double* out; CK(hipMalloc(&out, (size_t)ncu * 64 * 1024 * 8));
  long long* cyc; CK(hipMalloc(&cyc, 8));
  const int it = 20000;
  for (int wpc : {4, 8, 16}) {
    int blocks = ncu * wpc / 4;
    float ms = timeit([&] { hipLaunchKernelGGL(k_mfma_tput, dim3(blocks), dim3(256), 0, 0, out, it); });
    double fl = (double)blocks * 4 * it * 4 * 2048;
    printf("MFMA f64 16x16x4, %2d waves/CU: %.1f TFLOP/s\n", wpc, fl / ms / 1e9);
  }
  for (int wpc : {4, 8, 16}) {
    int blocks = ncu * wpc / 4;
    float ms = timeit([&] { hipLaunchKernelGGL(k_fma_tput, dim3(blocks), dim3(256), 0, 0, out, it); });
    double fl = (double)blocks * 256 * it * 8 * 2;
    printf("v_fma_f64, %2d waves/CU: %.1f TFLOP/s\n", wpc, fl / ms / 1e9);
  }
  for (int wpc : {4, 8, 16}) {
    int blocks = ncu * wpc / 4;
    float ms = timeit([&] { hipLaunchKernelGGL(k_mixed, dim3(blocks), dim3(256), 0, 0, out, it); });
    double fl = (double)blocks * 4 * it * (2 * 2048 + 8 * 64 * 2);
    printf("mixed MFMA+VALU, %2d waves/CU: %.1f TFLOP/s (%.3f ms)\n", wpc, fl / ms / 1e9, ms);
  }
  hipLaunchKernelGGL(k_mfma_lat, dim3(1), dim3(64), 0, 0, out, cyc, 1000);
  long long hc; CK(hipMemcpy(&hc, cyc, 8, hipMemcpyDeviceToHost));
  printf("dependent MFMA f64 latency: %.1f clock64 ticks / instr\n", hc / 1000.0);
  for (int wpc : {8, 16}) {
    int blocks = ncu * wpc / 4;
    float ms = timeit([&] { hipLaunchKernelGGL(k_mixed_int, dim3(blocks), dim3(256), 0, 0, out, it); });
    float ms2 = timeit([&] { hipLaunchKernelGGL(k_int_only, dim3(blocks), dim3(256), 0, 0, out, it); });
    float ms3 = timeit([&] { hipLaunchKernelGGL(k_mfma_tput, dim3(blocks), dim3(256), 0, 0, out, it / 2); });
    // per-wave cycles per iteration
    double cyc = ms * 1e-3 * clk / ((double)blocks * 4 / (ncu * 4)) / it;
    printf("%2d w/CU: mfma2+int32(32 ops) %.3f ms | int32 only (32 ops) %.3f ms | mfma 2/iter %.3f ms  [SIMD cycles/iter mixed %.1f]\n",
           wpc, ms, ms2, ms3, cyc);
    float ms4 = timeit([&] { hipLaunchKernelGGL(k_readlane_fma, dim3(blocks), dim3(256), 0, 0, out, it); });
    double cyc4 = ms4 * 1e-3 * clk / ((double)blocks * 4 / (ncu * 4)) / it;
    printf("    readlane x2 + fma, 8 per iter: %.3f ms -> %.1f SIMD cycles per (2 readlane + fma)\n", ms4, cyc4 / 8);
  }
  return 0;
}
