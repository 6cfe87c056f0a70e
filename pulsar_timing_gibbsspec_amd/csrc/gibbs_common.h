// Shared device helpers for the gfx950 Gibbs kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define GS_WAVE 64

// per-wave LDS scratch (doubles) of the tile b-draw (gibbs_tile.h): 272 transpose /
// factor rows + 64 vector + max(64, 16 NT) output (NT = NF / 16 + 1 <= 5).  Sized per NF,
// not at the 5-tile maximum: the LDS of a k_bdraw workgroup (model block + 4 scratches) sits
// at the 3-workgroups-per-CU edge for the simulated array (NF = 60, NMX = 17: 53320 B at 400
// doubles per wave vs 53832 B at 416), and dropping to 2 workgroups per CU cost 25 %
// (0.665 -> 0.835 ms per launch measured on MI355X).
#define GS_TILE_SCR_MAX 416
__host__ __device__ constexpr int gs_tile_scr(int NF) {
#ifdef GS_PHASE_PROF
  return GS_TILE_SCR_MAX + 8;  // + the phase-profile accumulators at 416..423
#else
  return 336 + (NF / 16 + 1 > 4 ? 16 * (NF / 16 + 1) : 64);  // output: max(64 lanes, 16 NT)
#endif
}

// ---------------------------------------------------------------- intra-wave LDS sync
// Lanes of one wavefront exchanging data through LDS: wavefront-scope release/acquire
// fences around the wave barrier (a bare wave barrier does not order the LDS accesses
// for the compiler backend).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------------------------------------------------------- cross-lane
// Broadcast lane `l` of a double to every lane (two v_readlane_b32 -> SGPRs).
__device__ __forceinline__ double rdlane(double v, int l) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u & 0xffffffffull), l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// ---------------------------------------------------------------- Philox4x32-10
struct gs_u4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ gs_u4 philox4x32_10(gs_u4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
    gs_u4 n;
    n.x = hi1 ^ c.y ^ k0;
    n.y = lo1;
    n.z = hi0 ^ c.w ^ k1;
    n.w = lo0;
    c = n;
  }
  return c;
}

// 53-bit uniform in [0,1) from two words (hi first).
__device__ __forceinline__ double gs_u53(uint32_t hi, uint32_t lo) {
  return (double)((((unsigned long long)hi << 32) | lo) >> 11) * 0x1.0p-53;
}

struct gs_key {
  uint32_t k0, k1;
};

__device__ __forceinline__ gs_u4 gs_counter(uint32_t slot, long long sweep, long long chain,
                                            int psr, int event) {
  gs_u4 c;
  c.x = slot;
  c.y = (uint32_t)sweep;
  c.z = (uint32_t)chain;
  c.w = ((uint32_t)psr << 8) | (uint32_t)(event & 0xff);
  return c;
}

// Sweep index of a Philox counter: the launch argument, plus the context's device-side
// sweep counter when one is attached (graph-captured sweeps advance it on the device).
__device__ __forceinline__ long long gs_sweep(int64_t s, const int64_t* dev) {
  return dev ? (long long)(s + *dev) : (long long)s;
}

// Two uniforms in [0,1) for one counter.
__device__ __forceinline__ void gs_uniform2(gs_u4 c, gs_key k, double& u1, double& u2) {
  const gs_u4 w = philox4x32_10(c, k.k0, k.k1);
  u1 = gs_u53(w.x, w.y);
  u2 = gs_u53(w.z, w.w);
}

// Two independent standard normals (Box-Muller) for one counter.
__device__ __forceinline__ void gs_normal2(gs_u4 c, gs_key k, double& n1, double& n2) {
  double u1, u2;
  gs_uniform2(c, k, u1, u2);
  const double r = sqrt(-2.0 * log(1.0 - u1));
  double s, co;
  sincospi(2.0 * u2, &s, &co);
  n1 = r * co;
  n2 = r * s;
}

// ---------------------------------------------------------------- numpy npy_logaddexp
__device__ __forceinline__ double np_logaddexp(double x, double y) {
  if (x == y) return x + 0.693147180559945309417232121458176568;  // x + log(2)
  const double t = x - y;
  if (t > 0) return x + log1p(exp(-t));
  if (t <= 0) return y + log1p(exp(t));
  return t;  // NaN
}

