// v_rcp_f64_dpp row_newbcast probe (gfx950).  Measured on MI355X (r03f): every variant below
// returns 1/0 = inf on every lane -- including the "reference", because the compiler's DPP
// combiner folds the single-use v_mov_b64_dpp into v_rcp_f64_dpp.  So the tile elimination keeps
// its pivot broadcast multi-use and never feeds a DPP move straight into v_rcp_f64 alone.
// The expected value is printed next to what the hardware returns.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int N, int NOP>
__device__ __forceinline__ double rcp_nb(double v) {
  double r;
  if (NOP)
    asm volatile("s_nop 1\n\tv_rcp_f64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf\n\ts_nop 0" : "=v"(r) : "v"(v), "n"(N));
  else
    asm volatile("s_nop 1\n\tv_rcp_f64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(v), "n"(N));
  return r;
}

__global__ void k(double* o, const double* in) {
  const int l = threadIdx.x;
  const double v = in[l] * 1.5;  // a VALU write right before the DPP read
  const double r0 = __builtin_amdgcn_rcp(__builtin_amdgcn_update_dpp(0.0, v, 0x150 + 5, 0xf, 0xf, false));
  const double r1 = rcp_nb<5, 1>(v);
  const double x1 = r1 * 2.0;  // consumer right after
  const double r2 = rcp_nb<5, 0>(v);
  const double x2 = r2 * 2.0;
  o[l] = r0 * 2.0;
  o[64 + l] = x1;
  o[128 + l] = x2;
}

int main() {
  double *d, *in, h[192], hin[64];
  for (int l = 0; l < 64; ++l) hin[l] = 3.0 + l;
  hipMalloc(&d, sizeof(h));
  hipMalloc(&in, sizeof(hin));
  hipMemcpy(in, hin, sizeof(hin), hipMemcpyHostToDevice);
  k<<<1, 64>>>(d, in);
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int bad1 = 0, bad2 = 0;
  for (int l = 0; l < 64; ++l) {
    bad1 += h[64 + l] != h[l];
    bad2 += h[128 + l] != h[l];
  }
  const double want = 2.0 / ((3.0 + 5) * 1.5);
  printf("rcp_dpp probe: lane0 expected %.17g; combined-mov %.17g asm+nop %.17g asm %.17g; mismatches %d %d\n",
         want, h[0], h[64], h[128], bad1, bad2);
  return h[0] == want ? 0 : 1;
}
