// Cross-lane primitive probe (gfx950): v_permlane32_swap / v_permlane16_swap group
// broadcast and DPP row_newbcast on 64-bit values.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int G>
__device__ double bcast_group(double v) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  unsigned w[2] = {(unsigned)u, (unsigned)(u >> 32)};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    auto a = __builtin_amdgcn_permlane32_swap(w[h], w[h], false, false);
    const unsigned y = (G < 2) ? a[0] : a[1];
    auto b = __builtin_amdgcn_permlane16_swap(y, y, false, false);
    w[h] = (G & 1) ? b[1] : b[0];
  }
  return __longlong_as_double((long long)(((unsigned long long)w[1] << 32) | w[0]));
}

template <int N>
__device__ double newbcast(double v) {
  return __builtin_amdgcn_update_dpp(0.0, v, 0x150 + N, 0xf, 0xf, false);
}

__global__ void k(double* o) {
  const int l = threadIdx.x;
  const double v = 1000.0 + l;
  o[0 * 64 + l] = bcast_group<0>(v);
  o[1 * 64 + l] = bcast_group<1>(v);
  o[2 * 64 + l] = bcast_group<2>(v);
  o[3 * 64 + l] = bcast_group<3>(v);
  o[4 * 64 + l] = newbcast<5>(v);
  o[5 * 64 + l] = newbcast<0>(v);
  o[6 * 64 + l] = newbcast<15>(v);
}

int main() {
  double* d;
  hipMalloc(&d, 7 * 64 * 8);
  k<<<1, 64>>>(d);
  double h[7 * 64];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* nm[7] = {"grp0", "grp1", "grp2", "grp3", "nb5", "nb0", "nb15"};
  int bad = 0;
  for (int t = 0; t < 7; ++t) {
    printf("%-5s", nm[t]);
    for (int l = 0; l < 64; l += 1) {
      double e = t < 4 ? 1000 + 16 * t + (l & 15) : 1000 + (l & ~15) + (t == 4 ? 5 : t == 5 ? 0 : 15);
      if (h[t * 64 + l] != e) bad++;
      if (l % 8 == 0) printf(" %g", h[t * 64 + l] - 1000);
    }
    printf("\n");
  }
  printf("mismatches: %d\n", bad);
  return bad != 0;
}
