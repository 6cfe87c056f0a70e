// Issue cost of single VALU instructions on gfx950 (the f64 ops the Gibbs kernels are made
// of): every CU full (8 waves per SIMD), each wave a stream of 8 independent chains of one
// instruction (inline asm, so nothing is folded), 1024 instructions per chain.  Prints SIMD
// cycles per wave-instruction: 4 = full rate for a wave of 64.
//   hipcc -O3 --offload-arch=gfx950 tools/probe/valu_rate_probe.hip -o tools/probe/valu_rate_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REP8(X) X X X X X X X X

// one instruction kind per kernel; v[0..7] are the independent chains
#define KERNEL(NAME, ASM)                                                                 \
  __global__ __launch_bounds__(256) void NAME(double* out, int iters) {                  \
    double v0 = threadIdx.x * 1e-3 + 1.0, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3;          \
    double v4 = v0 + 4, v5 = v0 + 5, v6 = v0 + 6, v7 = v0 + 7;                           \
    const double c = 1.0000001;                                                           \
    for (int it = 0; it < iters; ++it) {                                                  \
      REP8(asm volatile(ASM : "+v"(v0) : "v"(c)); asm volatile(ASM : "+v"(v1) : "v"(c));   \
           asm volatile(ASM : "+v"(v2) : "v"(c)); asm volatile(ASM : "+v"(v3) : "v"(c));   \
           asm volatile(ASM : "+v"(v4) : "v"(c)); asm volatile(ASM : "+v"(v5) : "v"(c));   \
           asm volatile(ASM : "+v"(v6) : "v"(c)); asm volatile(ASM : "+v"(v7) : "v"(c));)  \
    }                                                                                     \
    const double s = v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7;                               \
    if (s == 1.2345) out[threadIdx.x] = s;                                                \
  }

KERNEL(k_fma, "v_fma_f64 %0, %0, %1, %0")
KERNEL(k_mul, "v_mul_f64 %0, %0, %1")
KERNEL(k_add, "v_add_f64 %0, %0, %1")
KERNEL(k_max, "v_max_f64 %0, %0, %1")
KERNEL(k_rcp, "v_rcp_f64 %0, %0")
KERNEL(k_rsq, "v_rsq_f64 %0, %0")
KERNEL(k_sqrt, "v_sqrt_f64 %0, %0")
KERNEL(k_rndne, "v_rndne_f64 %0, %0")
KERNEL(k_ldexp, "v_ldexp_f64 %0, %0, 1")
KERNEL(k_frexp, "v_frexp_mant_f64 %0, %0")
KERNEL(k_mov64, "v_mov_b64 %0, %0")
KERNEL(k_dpp, "v_fmac_f64_dpp %0, %0, %1 row_newbcast:3 row_mask:0xf bank_mask:0xf")

// 32-bit / mixed forms: chains of unsigned
#define KERNEL32(NAME, ASM, CLOB)                                                               \
  __global__ __launch_bounds__(256) void NAME(double* out, int iters) {                  \
    unsigned v0 = threadIdx.x + 1, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3;                 \
    unsigned v4 = v0 + 4, v5 = v0 + 5, v6 = v0 + 6, v7 = v0 + 7;                         \
    const unsigned c = 0xD2511F53u;                                                       \
    for (int it = 0; it < iters; ++it) {                                                  \
      REP8(asm volatile(ASM : "+v"(v0) : "v"(c) CLOB); asm volatile(ASM : "+v"(v1) : "v"(c) CLOB); \
           asm volatile(ASM : "+v"(v2) : "v"(c) CLOB); asm volatile(ASM : "+v"(v3) : "v"(c) CLOB); \
           asm volatile(ASM : "+v"(v4) : "v"(c) CLOB); asm volatile(ASM : "+v"(v5) : "v"(c) CLOB); \
           asm volatile(ASM : "+v"(v6) : "v"(c) CLOB); asm volatile(ASM : "+v"(v7) : "v"(c) CLOB);) \
    }                                                                                     \
    const unsigned s = v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7;                             \
    if (s == 12345u) out[threadIdx.x] = s;                                                \
  }
KERNEL32(k_mullo, "v_mul_lo_u32 %0, %0, %1", )
KERNEL32(k_mulhi, "v_mul_hi_u32 %0, %0, %1", )
KERNEL32(k_add32, "v_add_u32 %0, %0, %1", )
KERNEL32(k_xor32, "v_xor_b32 %0, %0, %1", )
#define CVT_CLOB : "v250", "v251"
KERNEL32(k_cvt, "v_cvt_f64_u32 v[250:251], %0\n\tv_cvt_u32_f64 %0, v[250:251]", CVT_CLOB)  // a pair

int main() {
  int dev = 0, ncu = 0, clk = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);  // kHz
  const int blocks = ncu * 8, iters = 128;
  double* out;
  (void)hipMalloc(&out, sizeof(double) * 256);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  struct K {
    const char* name;
    void (*f)(double*, int);
    int per;  // instructions per asm statement
  } ks[] = {{"v_fma_f64", k_fma, 1},     {"v_mul_f64", k_mul, 1},         {"v_add_f64", k_add, 1},
            {"v_max_f64", k_max, 1},     {"v_rcp_f64", k_rcp, 1},         {"v_rsq_f64", k_rsq, 1},
            {"v_sqrt_f64", k_sqrt, 1},   {"v_rndne_f64", k_rndne, 1},     {"v_ldexp_f64", k_ldexp, 1},
            {"v_frexp_mant_f64", k_frexp, 1}, {"v_cvt_f64_u32+v_cvt_u32_f64", k_cvt, 2},
            {"v_mov_b64", k_mov64, 1},   {"v_mul_lo_u32", k_mullo, 1},   {"v_mul_hi_u32", k_mulhi, 1},
            {"v_add_u32", k_add32, 1},   {"v_xor_b32", k_xor32, 1},      {"v_fmac_f64_dpp", k_dpp, 1}};
  printf("{\"clock_mhz\": %.0f", clk / 1e3);
  for (auto& k : ks) {
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
      (void)hipEventRecord(e0, 0);
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, iters);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep > 0 && ms < best) best = ms;
    }
    // wave-instructions per SIMD: blocks * 4 waves / (4 * ncu) SIMDs * 64 per iter * iters * per
    const double winst = (double)blocks * 4 / (4.0 * ncu) * 64.0 * iters * k.per;
    const double cyc = best * 1e-3 * clk * 1e3;
    printf(", \"%s\": %.2f", k.name, cyc / winst);
  }
  printf("}\n");
  return 0;
}
