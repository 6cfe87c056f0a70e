// Power-law intrinsic red-noise Metropolis block, gfx950 fp64.
//
// Reference: PulsarBlockGibbs.update_red_params pulsar_gibbs.py:271-329 (steady state
// :312-319: 20 PTMCMCOneStep calls per sweep on the red-only likelihood) and
// get_lnlikelihood_red :549-566:
//   tau_k = (b_sin^2 + b_cos^2) / 2,  irn_k = phi_red(f_k; log10_A, gamma),  gw_k = 10^(2 rho_k)
//   lnL = sum_k lr_k - exp(lr_k),     lr_k = log tau_k - logaddexp(log irn_k, log gw_k).
// A power-law PSD is log-linear in its parameters: log irn_k = c_k + a_k log10_A + g_k gamma
// (host-probed from the signal's own get_phi), so a likelihood evaluation is one FMA chain,
// one logaddexp and one exp per frequency — no pow.
//
// Proposals restate PTMCMCSampler's symmetric jump mix (the dependency is absent and
// unpinned): SCAM along one eigenvector of the block covariance, AM along all of them, DE
// from a buffer of warm-up samples; SCAM/AM step scale 10 / 0.2 / 1 w.p. 0.03 / 0.07 / 0.9.
// anchor = 1 keeps the reference's semantics: its loop discards PTMCMCOneStep's returned
// (lnlike0, lnprob0) (:318-319), so every step of a block is accepted against the block's
// starting log-probability; anchor = 0 is the textbook chain (against the current state).
// Uniform priors: a proposal outside the bounds has lnprob = -inf (rejected); the other
// parameters' prior terms are constant within the block and cancel.
//
// Mapping: one wavefront per chain, lane l owns frequencies l, l + 64, ...; the sum is a
// butterfly reduction (every lane holds it, the MH decision is wave-uniform).
// Philox counters (slot 4s + j, sweep, chain, 0, GS_EV_REDMH) for step s:
//   j = 0: (u_kind, u_scale)  1: (u_a, u_b) direction / DE pair  2: normals (n1, n2)
//   j = 3: (u_acc, u_de).
#include "gibbs_common.h"
#include "gibbs_internal.h"

#pragma clang fp contract(off)  // proposals and sums rounded as the oracle restates them

namespace {

constexpr int RM_MAXK = 4;  // frequencies per lane (n_f <= 256)
constexpr int GS_EV_REDMH = 8;

struct RedFreq {
  double ltau[RM_MAXK], lgw[RM_MAXK], c[RM_MAXK], a[RM_MAXK], g[RM_MAXK];
  bool on[RM_MAXK];
};

__device__ __forceinline__ double lnirn(const RedFreq& F, int j, double la, double ga) {
  // (a_k la + c_k) + g_k ga, rounded step by step (no contraction), as the oracle computes it
  return gs_add_rn(gs_add_rn(gs_mul_rn(F.a[j], la), F.c[j]), gs_mul_rn(F.g[j], ga));
}

__device__ __forceinline__ double red_lnlike(const RedFreq& F, double la, double ga) {
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < RM_MAXK; ++j) {
    if (F.on[j]) {
      const double lr = F.ltau[j] - np_logaddexp(lnirn(F, j, la, ga), F.lgw[j]);
      s += lr - exp(lr);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  return s;
}

__global__ __launch_bounds__(256) void k_red_mh(RedMhArgs A) {
  const int wave = gs_wave_id(), lane = threadIdx.x & 63;
  const int64_t c = (int64_t)blockIdx.x * 4 + wave;
  if (c >= A.n_chain) return;  // whole wavefront exits together
  double* xc = A.x + c * A.ldx;
  const int colA = A.red_col[0], colG = A.red_col[1];
  double qa = xc[colA], qg = xc[colG];
  RedFreq F;
#pragma unroll
  for (int j = 0; j < RM_MAXK; ++j) {
    const int k = lane + 64 * j;
    F.on[j] = k < A.n_f;
    const int kk = F.on[j] ? k : 0;
    F.ltau[j] = log(A.tau[(int64_t)kk * A.n_chain + c]);
    F.lgw[j] = log(pow(10.0, 2.0 * xc[A.gw_col[kk]]));  // np.log(gw_sig.get_phi(params)[::2])
    F.c[j] = A.lnphi[kk];
    F.a[j] = A.lnphi[A.n_f + kk];
    F.g[j] = A.lnphi[2 * A.n_f + kk];
  }
  const double L0 = red_lnlike(F, qa, qg);
  double Lcur = L0;
  int acc = 0;
  if (A.nsteps > 0) {
    const double* J = A.jump;
    const double U00 = J[0], U01 = J[1], U10 = J[2], U11 = J[3], s0 = J[4], s1 = J[5];
    const double w_scam = J[6], w_am = J[7], lo0 = J[8], hi0 = J[9], lo1 = J[10], hi1 = J[11];
    const long long sw = gs_sweep(A.sweep, A.sweep_dev);
    const long long chain = A.chain_base + c;
    for (int s = 0; s < A.nsteps; ++s) {
      double u_kind, u_scale, u_a, u_b, n1, n2, u_acc, u_de;
      gs_uniform2(gs_counter(4 * s + 0, sw, chain, 0, GS_EV_REDMH), A.key, u_kind, u_scale);
      gs_uniform2(gs_counter(4 * s + 1, sw, chain, 0, GS_EV_REDMH), A.key, u_a, u_b);
      gs_normal2(gs_counter(4 * s + 2, sw, chain, 0, GS_EV_REDMH), A.key, n1, n2);
      gs_uniform2(gs_counter(4 * s + 3, sw, chain, 0, GS_EV_REDMH), A.key, u_acc, u_de);
      const double scale = u_scale > 0.97 ? 10.0 : (u_scale > 0.9 ? 0.2 : 1.0);
      double da, dg;
      if (u_kind < w_scam) {  // SCAM: one eigen-direction, cd = 2.4 / sqrt(2 * 1)
        const bool d1 = u_a >= 0.5;
        const double cd = 1.6970562748477141 * scale * (d1 ? s1 : s0) * n1;
        da = cd * (d1 ? U01 : U00);
        dg = cd * (d1 ? U11 : U10);
      } else if (u_kind < w_am) {  // AM: all directions, cd = 2.4 / sqrt(2 * ndim)
        const double cd = 1.2 * scale;
        const double z0 = n1 * s0, z1 = n2 * s1;
        da = cd * (U00 * z0 + U01 * z1);
        dg = cd * (U10 * z0 + U11 * z1);
      } else {  // DE: difference of two distinct buffer samples
        const int n = A.nde;
        const int i = min((int)(u_a * n), n - 1);
        int k = min((int)(u_b * (n - 1)), n - 2);
        if (k >= i) ++k;
        const double sc = u_de < 0.5 ? 1.0 : u_scale * 1.2;
        da = sc * (A.de[2 * i] - A.de[2 * k]);
        dg = sc * (A.de[2 * i + 1] - A.de[2 * k + 1]);
      }
      const double pa = qa + da, pg = qg + dg;
      const bool inb = pa >= lo0 && pa <= hi0 && pg >= lo1 && pg <= hi1;
      const double L1 = inb ? red_lnlike(F, pa, pg) : -__builtin_inf();
      const double ref = A.anchor ? L0 : Lcur;
      if (L1 - ref > log(u_acc)) {
        qa = pa;
        qg = pg;
        Lcur = L1;
        ++acc;
      }
    }
  }
  if (lane == 0) {
    xc[colA] = qa;
    xc[colG] = qg;
    if (A.lnl) A.lnl[c] = Lcur;
    if (A.n_acc) A.n_acc[c] = acc;
  }
  if (A.irn) {
#pragma unroll
    for (int j = 0; j < RM_MAXK; ++j)
      if (F.on[j]) A.irn[(int64_t)(lane + 64 * j) * A.n_chain + c] = exp(lnirn(F, j, qa, qg));
  }
}

}  // namespace

int launch_red_mh(hipStream_t s, const RedMhArgs& a) {
  hipLaunchKernelGGL(k_red_mh, dim3((unsigned)((a.n_chain + 3) / 4)), dim3(256), 0, s, a);
  return 0;
}
