// Accuracy of the short f64 math of gibbs_common.h (gs_log_pos, gs_sincos2pi) and of the
// raw v_rcp_f64 / v_rsq_f64 on gfx950, against long double on the host.
//   hipcc -O3 --offload-arch=gfx950 -I pulsar_timing_gibbsspec_amd/csrc tools/probe/fastmath_probe.hip
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "gibbs_common.h"

__global__ void k(const double* x, const double* u, double* lg, double* sn, double* cs, double* rc, double* rs,
                  double* lgl, double* ex, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  lg[i] = gs_log_pos(x[i]);
  lgl[i] = log(x[i]);
  // exp on [-750, 0]: x mapped from the log test's inputs
  ex[i] = gs_exp_neg(-750.0 * u[i]);
  gs_sincos2pi(u[i], sn[i], cs[i]);
  rc[i] = __builtin_amdgcn_rcp(x[i]);
  rs[i] = __builtin_amdgcn_rsq(x[i]);
}

static double ulp_err(double got, long double want) {
  const double w = (double)want;
  const double ulp = nextafter(fabs(w), INFINITY) - fabs(w);
  return fabsl((long double)got - want) / ulp;
}

int main() {
  const int n = 1 << 22;
  double* h[9];
  for (int j = 0; j < 9; ++j) h[j] = (double*)malloc(n * 8);
  srand(1);
  for (int i = 0; i < n; ++i) {
    const double a = rand() / (double)RAND_MAX, b = rand() / (double)RAND_MAX;
    // half log-uniform over [1e-300, 1e300], half 1 - u53 (the Box-Muller argument)
    h[0][i] = (i & 1) ? pow(10.0, -300.0 + 600.0 * a)
                      : 1.0 - (double)(((unsigned long long)rand() << 31 ^ (unsigned long long)rand()) >> 9) * 0x1.0p-53;
    if (h[0][i] <= 0) h[0][i] = 0x1.0p-53;
    h[1][i] = (double)(unsigned long long)(b * 9007199254740992.0) * 0x1.0p-53;
  }
  double* d[9];
  for (int j = 0; j < 9; ++j) (void)hipMalloc(&d[j], n * 8);
  (void)hipMemcpy(d[0], h[0], n * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(d[1], h[1], n * 8, hipMemcpyHostToDevice);
  k<<<n / 256, 256>>>(d[0], d[1], d[2], d[3], d[4], d[5], d[6], d[7], d[8], n);
  for (int j = 2; j < 9; ++j) (void)hipMemcpy(h[j], d[j], n * 8, hipMemcpyDeviceToHost);
  const long double TWO_PI = 6.283185307179586476925286766559005768L;
  double e[7] = {0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < n; ++i) {
    const long double x = h[0][i];
    // exact quadrant reduction on the host too: the long double angle 2 pi u alone loses the
    // relative accuracy of sin / cos near their zeros
    const double q = rint(4.0 * h[1][i]);
    const long double r = (long double)h[1][i] - (long double)q / 4, sr = sinl(TWO_PI * r), cr = cosl(TWO_PI * r);
    const int qi = (int)q & 3;
    const long double a = (qi & 1) ? cr : sr, b = (qi & 1) ? sr : cr;
    const long double ws = (qi & 2) ? -a : a, wc = ((qi + 1) & 2) ? -b : b;
    const double v[6] = {ulp_err(h[2][i], logl(x)), ulp_err(h[7][i], logl(x)), ulp_err(h[3][i], ws),
                         ulp_err(h[4][i], wc), ulp_err(h[5][i], 1.0L / x),
                         ulp_err(h[6][i], 1.0L / sqrtl(x))};
    for (int j = 0; j < 6; ++j)
      if (v[j] > e[j]) e[j] = v[j];
    const long double xe = (long double)(-750.0 * h[1][i]);  // the device's (rounded) argument
    const long double we = expl(xe);
    if (we > 0x1.0p-1020L) {  // normal results (denormals: absolute error below 2^-1074)
      const double ve = ulp_err(h[8][i], we);
      if (ve > e[6]) e[6] = ve;
    }
  }
  printf("{\"gs_log_pos_ulp\": %.3f, \"ocml_log_ulp\": %.3f, \"gs_sin2pi_ulp\": %.3f, \"gs_cos2pi_ulp\": %.3f, "
         "\"v_rcp_f64_ulp\": %.4g, \"v_rsq_f64_ulp\": %.4g, \"gs_exp_neg_ulp\": %.3f, \"n\": %d}\n",
         e[0], e[1], e[2], e[3], e[4], e[5], e[6], n);
  return 0;
}
