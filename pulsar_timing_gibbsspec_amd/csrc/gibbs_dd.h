// Double-double (hi + lo, ~106-bit significand) arithmetic for the once-per-state
// precomputes whose fp64 rounding sets the b|rho draw's accuracy:
// TNT/d with exact products and the fixed-prior Schur complement S0 = A_FF - W^T W,
// where the timing model absorbs most of A_FF and fp64 cancellation costs 2-3 digits.
//
// Error-free transformations (Knuth two-sum, fma two-product) with explicit fma.  FP
// contraction is OFF for every TU that includes this header: HIP's default
// (-ffp-contract=fast) fused `s + a*b` in the Dot2 step into one fma while the product's
// error term was taken from the separately rounded a*b, which silently degraded the
// double-double prefix to fp64 accuracy on the device (caught by
// test_tnt_dd_and_prefix_dd_accuracy; tests/test_dd_host.py runs this header on the host).
#pragma once
#include <hip/hip_runtime.h>

#pragma clang fp contract(off)

struct gs_dd {
  double hi, lo;
};

__device__ __forceinline__ gs_dd dd_make(double hi, double lo = 0.0) { return {hi, lo}; }

// s + e = a + b exactly (any magnitudes)
__device__ __forceinline__ gs_dd dd_two_sum(double a, double b) {
  const double s = a + b;
  const double bb = s - a;
  return {s, (a - (s - bb)) + (b - bb)};
}
// same for |a| >= |b| (or a == 0)
__device__ __forceinline__ gs_dd dd_fast_two_sum(double a, double b) {
  const double s = a + b;
  return {s, b - (s - a)};
}
__device__ __forceinline__ gs_dd dd_add(gs_dd a, gs_dd b) {
  gs_dd s = dd_two_sum(a.hi, b.hi);
  const gs_dd t = dd_two_sum(a.lo, b.lo);
  s.lo += t.hi;
  s = dd_fast_two_sum(s.hi, s.lo);
  s.lo += t.lo;
  return dd_fast_two_sum(s.hi, s.lo);
}
__device__ __forceinline__ gs_dd dd_neg(gs_dd a) { return {-a.hi, -a.lo}; }
__device__ __forceinline__ gs_dd dd_sub(gs_dd a, gs_dd b) { return dd_add(a, dd_neg(b)); }
__device__ __forceinline__ gs_dd dd_add_d(gs_dd a, double b) {
  gs_dd s = dd_two_sum(a.hi, b);
  s.lo += a.lo;
  return dd_fast_two_sum(s.hi, s.lo);
}
__device__ __forceinline__ gs_dd dd_mul(gs_dd a, gs_dd b) {
  const double p = a.hi * b.hi;
  double e = fma(a.hi, b.hi, -p);
  e = fma(a.hi, b.lo, fma(a.lo, b.hi, e));
  return dd_fast_two_sum(p, e);
}
__device__ __forceinline__ gs_dd dd_mul_d(gs_dd a, double b) {
  const double p = a.hi * b;
  const double e = fma(a.lo, b, fma(a.hi, b, -p));
  return dd_fast_two_sum(p, e);
}
// a / b: one fp64 quotient, its dd residual, one correction
__device__ __forceinline__ gs_dd dd_div(gs_dd a, gs_dd b) {
  const double q1 = a.hi / b.hi;
  const gs_dd r = dd_sub(a, dd_mul_d(b, q1));
  const double q2 = r.hi / b.hi;
  const gs_dd r2 = dd_sub(r, dd_mul_d(b, q2));
  const double q3 = r2.hi / b.hi;
  return dd_add_d(dd_fast_two_sum(q1, q2), q3);
}
// sqrt(a), a > 0 (a <= 0 or NaN: NaN/0 propagate to the caller's pivot check)
__device__ __forceinline__ gs_dd dd_sqrt(gs_dd a) {
  const double x = sqrt(a.hi);
  const double p = x * x;
  const double e = fma(x, x, -p);
  const double r = ((a.hi - p) - e + a.lo) / (2.0 * x);
  return dd_fast_two_sum(x, r);
}
// log(a.hi + a.lo) to fp64 accuracy
__device__ __forceinline__ double dd_log(gs_dd a) { return log(a.hi) + a.lo / a.hi; }

// Dot2 accumulator (Ogita-Rump-Oishi): s + c carries a sum of exact products to ~u^2.
struct gs_dot2 {
  double s = 0.0, c = 0.0;
  __device__ __forceinline__ void init(gs_dd v) {
    s = v.hi;
    c = v.lo;
  }
  // += a * b for double-double a, b (the lo x lo term is below the result's precision)
  __device__ __forceinline__ void fma_dd(gs_dd a, gs_dd b) {
    const double p = a.hi * b.hi;
    const double pe = fma(a.hi, b.hi, -p);
    const gs_dd t = dd_two_sum(s, p);
    s = t.hi;
    c += t.lo + fma(a.hi, b.lo, fma(a.lo, b.hi, pe));
  }
  __device__ __forceinline__ void fma_ddd(gs_dd a, double b) {
    const double p = a.hi * b;
    const double pe = fma(a.hi, b, -p);
    const gs_dd t = dd_two_sum(s, p);
    s = t.hi;
    c += t.lo + fma(a.lo, b, pe);
  }
  __device__ __forceinline__ gs_dd get() const { return dd_fast_two_sum(s, c); }
};
