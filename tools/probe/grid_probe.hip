// Ceiling of the free-spectrum grid conditionals (pta_gibbs.py:189-212, 254-274) on gfx950:
// how many grid-point evaluations per second the chip sustains for the per-point op mix
// of the device kernels, with no memory traffic at all (operands in registers, every CU
// busy, 8 waves per SIMD).  This is the "peak" the bench prices the grid kernels against
// (MI355X_MICROARCH.md has no fp64 transcendental rate).
//
//   red  : red_lane_cumsum (gibbs_gridpt.h) -- k_rho_red_wave's per-point work: h = (tau/2) /
//          (gw + rho_g) with one reciprocal per four points, pdf' = h exp(-h) by the LDS-table
//          exp, the lane's running sum; 16 points per lane, (tau, gw) changing every row as in
//          the kernel.  red_libm_evals_per_s: the first kernel's op mix (ratio by rcp + two
//          Newton steps per point, the device library's exp), for reference.
//   curn : a = irn + rho_g; N = N a + tau D; D *= a (rescaled every 8 pulsars)
//          -- k_rho_curn_fast's per-(point, pulsar) work (no transcendental, no division)
//
// Build: hipcc --offload-arch=gfx950 -O3 -I pulsar_timing_gibbsspec_amd/csrc tools/probe/grid_probe.hip -o tools/probe/grid_probe
// Run:   tools/probe/grid_probe  -> one JSON line
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "gibbs_common.h"
#include "gibbs_gridpt.h"

constexpr double LN10 = 2.302585092994045684017991454684364208;

__device__ __forceinline__ double rcp_nr(double a) {
  double r = __builtin_amdgcn_rcp(a);
  r = fma(r, fma(-a, r, 1.0), r);
  return fma(r, fma(-a, r, 1.0), r);
}

// each lane: 16 grid points in registers, npts/16 rows of (tau, gw) (the kernel's loop)
__global__ __launch_bounds__(256) void k_red(int npts, double q, double* out) {
  __shared__ double tb[64];
  if (threadIdx.x < 64) tb[threadIdx.x] = GS_EXP2_64[threadIdx.x];
  __syncthreads();
  double rg[16], cum[16];
  double r0 = 1e-20 * (1.0 + 1e-3 * (threadIdx.x & 63));
  for (int j = 0; j < 16; ++j) {
    rg[j] = r0;
    r0 *= q;
  }
  double th = 0.5e-14 * (1.0 + 0.01 * (threadIdx.x & 255)), gw = 3e-15, acc = 0.0;
  for (int row = 0; row < npts / 16; ++row) {
    acc += red_lane_cumsum<16>(th, gw, rg, tb, cum);
    th *= 1.0001;
    gw *= 0.9999;
  }
  for (int j = 0; j < 16; ++j) acc += cum[j];
  if (acc == 1.2345) out[blockIdx.x * blockDim.x + threadIdx.x] = acc;  // keep the work alive
}

// the first red kernel's op mix: 8 independent rows per thread, one division + libm exp per point
__global__ __launch_bounds__(256) void k_red_libm(int npts, double q, double* out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  double tau[8], cum[8];
  for (int j = 0; j < 8; ++j) {
    tau[j] = 1e-14 * (1.0 + 0.01 * ((t + j) & 255));
    cum[j] = 0.0;
  }
  double rg = 1e-20;
  const double gw = 3e-15;
  for (int g = 0; g < npts; ++g) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const double ratio = tau[j] * rcp_nr(gw + rg);
      cum[j] += ratio * exp(-ratio / 2) * LN10;
    }
    rg *= q;
  }
  double s = 0.0;
  for (int j = 0; j < 8; ++j) s += cum[j];
  if (s == 1.2345) out[t] = s;
}

__global__ __launch_bounds__(256) void k_curn(int npts, double q, double* out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  double nn[8], dd[8], rg[8];
  for (int j = 0; j < 8; ++j) {
    nn[j] = 0.0;
    dd[j] = 1.0;
    rg[j] = 1e-18 * (1.0 + j);
  }
  const double tau = 1e-14 * (1.0 + 0.01 * (t & 255));
  for (int p = 0; p < npts; ++p) {
    const double irn = 1e-15 * (1.0 + 1e-3 * p);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const double a = irn + rg[j];
      nn[j] = fma(nn[j], a, tau * dd[j]);
      dd[j] *= a;
    }
    if ((p & 7) == 7)
      for (int j = 0; j < 8; ++j) {
        const int e = __builtin_amdgcn_frexp_exp(dd[j]);
        dd[j] = __builtin_amdgcn_frexp_mant(dd[j]);
        nn[j] = ldexp(nn[j], -e);
      }
  }
  double s = 0.0;
  for (int j = 0; j < 8; ++j) s += nn[j] + dd[j];
  if (s == 1.2345) out[t] = s;
}

// k_rho_curn_sum_wave's per-point work: log pdf = c_g - S w_g (one FMA), the wave maximum,
// the LDS-table exp, the lane's running sum (16 points per lane, S changing every row)
__global__ __launch_bounds__(256) void k_curn_sum(int npts, double q, double* out) {
  __shared__ double tb[64];
  if (threadIdx.x < 64) tb[threadIdx.x] = GS_EXP2_64[threadIdx.x];
  __syncthreads();
  double cg[16], wg[16], lp[16];
  double r0 = 1e-18 * (1.0 + 1e-3 * (threadIdx.x & 63));
  for (int j = 0; j < 16; ++j) {
    cg[j] = -45.0 * log(r0);
    wg[j] = 0.5 / r0;
    r0 *= q;
  }
  double nS = -1e-14 * (1.0 + 0.01 * (threadIdx.x & 255)), acc = 0.0;
  for (int row = 0; row < npts / 16; ++row) {
    double mx = -__builtin_inf();
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      lp[j] = fma(nS, wg[j], cg[j]);
      mx = fmax(mx, lp[j]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
    double loc = 0.0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      loc += exp_neg_t64(lp[j] - mx, tb);
      lp[j] = loc;
    }
    acc += loc;
    nS *= 1.0001;
  }
  for (int j = 0; j < 16; ++j) acc += lp[j];
  if (acc == 1.2345) out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
  int dev = 0, ncu = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const int blocks = ncu * 8;  // 8 x 256 threads per CU = 8 waves per SIMD
  const int npts = 4000;
  double* out;
  (void)hipMalloc(&out, sizeof(double) * blocks * 256);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  double rates[4];
  for (int kind = 0; kind < 4; ++kind) {
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      (void)hipEventRecord(e0, 0);
      if (kind == 0)
        hipLaunchKernelGGL(k_red, dim3(blocks), dim3(256), 0, 0, npts, 1.0277, out);
      else if (kind == 2)
        hipLaunchKernelGGL(k_red_libm, dim3(blocks), dim3(256), 0, 0, npts, 1.0277, out);
      else if (kind == 3)
        hipLaunchKernelGGL(k_curn_sum, dim3(blocks), dim3(256), 0, 0, npts, 1.0277, out);
      else
        hipLaunchKernelGGL(k_curn, dim3(blocks), dim3(256), 0, 0, npts, 1.0277, out);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep > 0 && ms < best) best = ms;
    }
    rates[kind] = (double)blocks * 256 * ((kind == 0 || kind == 3) ? 1 : 8) * npts / (best * 1e-3);  // wave kernels: npts per lane
  }
  printf("{\"cus\": %d, \"red_evals_per_s\": %.6e, \"curn_pulsar_terms_per_s\": %.6e, \"red_libm_evals_per_s\": %.6e, "
         "\"curn_sum_evals_per_s\": %.6e}\n",
         ncu, rates[0], rates[1], rates[2], rates[3]);
  return 0;
}
