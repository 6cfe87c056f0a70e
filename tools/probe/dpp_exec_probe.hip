// Does a 64-bit DPP row_newbcast read its source lane when that lane is disabled in EXEC?
// The diagonal-tile elimination (gibbs_tile.h tile_elim1) zeroes the multiplier of columns c <= k
// with one exec-masked v_mov_b64 per step; if the column updates could instead run with
// exec = {c > k} (an SALU exec write), the source lane k of row_newbcast:k would be disabled.
// Prints the result on an enabled lane for both cases: source enabled and source disabled.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k(double* out) {
  const int lane = threadIdx.x & 63;
  double acc = 100.0 + lane;           // destination
  double v = 1000.0 + lane;            // DPP source: lane k of each row holds 1000 + k (+16 row)
  double m = 1.0;
  // case 0: all lanes on
  double a0 = acc;
  asm volatile("s_nop 4\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf"
               : "+v"(a0) : "v"(v), "v"(m));
  // case 1: exec = lanes with (lane & 15) > 3 (lane 3 of every row disabled)
  double a1 = acc;
  asm volatile("s_mov_b32 exec_lo, 0xfff0fff0\n\t"
               "s_mov_b32 exec_hi, 0xfff0fff0\n\t"
               "s_nop 4\n\t"
               "v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
               "s_mov_b64 exec, -1"
               : "+v"(a1) : "v"(v), "v"(m));
  // case 2: same with bound_ctrl (DPP_BOUND_ZERO)
  double a2 = acc;
  asm volatile("s_mov_b32 exec_lo, 0xfff0fff0\n\t"
               "s_mov_b32 exec_hi, 0xfff0fff0\n\t"
               "s_nop 4\n\t"
               "v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
               "s_mov_b64 exec, -1"
               : "+v"(a2) : "v"(v), "v"(m));
  out[lane] = a0;
  out[64 + lane] = a1;
  out[128 + lane] = a2;
}

int main() {
  double* d;
  double h[192];
  (void)hipMalloc(&d, sizeof(h));
  k<<<1, 64>>>(d);
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const int ls[] = {0, 3, 4, 5, 15, 16, 20, 63};
  for (int i = 0; i < 8; ++i) {
    const int l = ls[i];
    printf("lane %2d: all-on %.1f  src-disabled %.1f  src-disabled+bound_ctrl %.1f  (expect %.1f)\n", l, h[l],
           h[64 + l], h[128 + l], 100.0 + l + 1000.0 + 3 + 16 * (l / 16));
  }
  return 0;
}
