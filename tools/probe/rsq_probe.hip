// Accuracy of the raw f64 transcendental instructions on gfx950 (v_rsq_f64, v_rcp_f64)
// against long double references over log-uniform inputs.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <math.h>
#include <stdlib.h>

__global__ void k(const double* x, double* rsq, double* rcp, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { rsq[i] = __builtin_amdgcn_rsq(x[i]); rcp[i] = __builtin_amdgcn_rcp(x[i]); }
}

int main() {
  const int n = 1 << 20;
  double *hx = (double*)malloc(n * 8), *hr = (double*)malloc(n * 8), *hc = (double*)malloc(n * 8);
  srand(1);
  for (int i = 0; i < n; ++i) hx[i] = pow(10.0, -30.0 + 60.0 * (rand() / (double)RAND_MAX));
  double *dx, *dr, *dc;
  (void)hipMalloc(&dx, n * 8); (void)hipMalloc(&dr, n * 8); (void)hipMalloc(&dc, n * 8);
  (void)hipMemcpy(dx, hx, n * 8, hipMemcpyHostToDevice);
  k<<<n / 256, 256>>>(dx, dr, dc, n);
  (void)hipMemcpy(hr, dr, n * 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(hc, dc, n * 8, hipMemcpyDeviceToHost);
  double er = 0, ec = 0;
  for (int i = 0; i < n; ++i) {
    long double x = hx[i];
    long double r = 1.0L / sqrtl(x), c = 1.0L / x;
    double a = fabs((double)((hr[i] - r) / r)), b = fabs((double)((hc[i] - c) / c));
    if (a > er) er = a;
    if (b > ec) ec = b;
  }
  printf("v_rsq_f64 max rel err %.3e (%.2f ulp)\nv_rcp_f64 max rel err %.3e (%.2f ulp)\n", er, er / 2.22e-16, ec, ec / 2.22e-16);
  return 0;
}
