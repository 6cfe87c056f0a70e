// Basis-ECORR block: the epoch columns of a basis-ECORR signal have a
// DIAGONAL block in TNT (every TOA belongs to at most one epoch), so Sigma = TNT +
// diag(phiinv) is reduced to the [timing model | free spectrum] columns R by eliminating
// the epochs first:
//     a_e = TNT_ee + 1/phi_e,  Sigma_R' = TNT_RR - B^T diag(1/a) B,  d_R' = d_R - B^T (d_E / a)
// (B = TNT[E, R]).  k_ecorr_schur forms Sigma_R', d_R' and the scalars of the
// marginalised likelihood for every chain's ECORR values; the existing prefix / lnlike /
// b-draw kernels then run on the R system, and k_ecorr_bdraw_e draws the epochs
// b_E | b_R ~ N((d_E - B b_R) / a, 1/a).  The Metropolis block is
// PulsarBlockGibbs.update_ecorr_params (pulsar_gibbs.py:409-486) on
// get_lnlikelihood_fullmarg (:569-610): k_ecorr_propose / k_ecorr_accept bracket one
// batched likelihood evaluation per step.
#include "gibbs_internal.h"

namespace {

typedef double gs_d4_t __attribute__((ext_vector_type(4)));

constexpr int EC_WAVES = 8;  // chains per workgroup (one wavefront each)
constexpr int EC_CH = 32;    // epochs per LDS chunk

__device__ __forceinline__ double ec_wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// 1/phi_k and log phi_k of backend k from log10_ecorr (phi = 10**(2 x), get_phiinv = 1/phi)
__device__ __forceinline__ void ec_phi(double x, double& inv, double& lg) {
  const double ph = pow(10.0, 2.0 * x);
  inv = 1.0 / ph;
  lg = log(ph);
}

// Batched ECORR Schur complement, one wavefront per chain, EC_WAVES chains per
// workgroup sharing every LDS chunk of Bx = [B | d_E] (EC_CH epochs x 16 NB columns).
// Per 4-epoch step a lane loads NB values of its epoch row, scales them by the chain's
// 1/a_e and issues NB (NB + 1) / 2 v_mfma_f64_16x16x4f64 into the lower tiles of
// [B | d_E]^T diag(1/a) [B | d_E]: rows < mR give B^T W B, row mR gives B^T W d_E and
// (mR, mR) gives sum d_E^2 / a.  Roofline: fp64 MFMA, 2 ne (16 NB)^2 / 2 flop per chain,
// Bx read once per workgroup from L2.
template <int NB>
__global__ __launch_bounds__(64 * EC_WAVES) void k_ecorr_schur(EcorrSchurArgs A) {
  extern __shared__ double lds[];
  __shared__ double wb[2][EC_WAVES][EC_CH];
  __shared__ double sinv[EC_WAVES][GS_WHITE_MAX_BK + 1], slog[EC_WAVES][GS_WHITE_MAX_BK + 1];
  constexpr int LDB = 16 * NB;
  constexpr int NT = NB * (NB + 1) / 2;
  const int tid = threadIdx.x, l = tid & 63, i = l & 15, k = l >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = blockIdx.x * EC_WAVES + w;
  const bool live = c < A.n_chain;
  const int ne = A.ne, mR = A.mR;
  if (l < A.n_bk) {
    double inv = 0.0, lg = 0.0;
    if (live) ec_phi(A.x[(int64_t)c * A.ldx + A.xcol[l]], inv, lg);
    sinv[w][l] = inv;
    slog[w][l] = lg;
  }
  __syncthreads();

  gs_d4_t acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = gs_d4_t{0.0, 0.0, 0.0, 0.0};
  double sla = 0.0, slp = 0.0;

  double reg[NB];
  double wreg = 0.0;
  auto load = [&](int e0) {
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const int idx = tid + 64 * EC_WAVES * q;  // EC_CH * LDB = 512 NB elements
      const int e = e0 + idx / LDB;
      reg[q] = (e < ne) ? A.Bx[(int64_t)e0 * LDB + idx] : 0.0;
    }
    wreg = 0.0;
    if (l < EC_CH && live) {
      const int e = e0 + l;
      if (e < ne) {
        const int kb = A.ebk[e];
        const double a = A.Dg[e] + sinv[w][kb];
        wreg = 1.0 / a;
        sla += log(a);
        slp += slog[w][kb];
      }
    }
  };
  auto store = [&](int buf) {
    double* dst = lds + buf * (EC_CH * LDB);
#pragma unroll
    for (int q = 0; q < NB; ++q) dst[tid + 64 * EC_WAVES * q] = reg[q];
    if (l < EC_CH) wb[buf][w][l] = wreg;
  };

  const int nch = (ne + EC_CH - 1) / EC_CH;
  load(0);
  store(0);
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    const int cb = ch & 1;
    if (ch + 1 < nch) load((ch + 1) * EC_CH);
    __builtin_amdgcn_sched_barrier(0);
    const double* cur = lds + cb * (EC_CH * LDB);
#pragma unroll
    for (int kk = 0; kk < EC_CH / 4; ++kk) {
      const double* row = cur + (4 * kk + k) * LDB + i;
      const double wv = wb[cb][w][4 * kk + k];
      double v[NB];
#pragma unroll
      for (int r = 0; r < NB; ++r) v[r] = row[16 * r];
#pragma unroll
      for (int r = 0; r < NB; ++r) {
        const double av = v[r] * wv;
#pragma unroll
        for (int j = 0; j <= r; ++j)
          acc[r * (r + 1) / 2 + j] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, v[j], acc[r * (r + 1) / 2 + j], 0, 0, 0);
      }
    }
    if (ch + 1 < nch) store(cb ^ 1);
    __syncthreads();
  }
  sla = ec_wave_sum(sla);
  slp = ec_wave_sum(slp);
  if (!live) return;

  double* out = A.TNT + (int64_t)c * mR * mR;
  double* dout = A.d + (int64_t)c * mR;
#pragma unroll
  for (int r = 0; r < NB; ++r) {
#pragma unroll
    for (int j = 0; j <= r; ++j) {
      const gs_d4_t v4 = acc[r * (r + 1) / 2 + j];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 16 * r + k + 4 * q, col = 16 * j + i;
        const double v = v4[q];
        if (row < mR && col <= row) {  // lower triangle only: exact symmetry
          const double s = A.A[(int64_t)row * mR + col] - v;
          out[(int64_t)row * mR + col] = s;
          out[(int64_t)col * mR + row] = s;
        } else if (row == mR && col < mR) {
          dout[col] = A.dR[col] - v;
        } else if (row == mR && col == mR) {
          A.aux[(int64_t)c * 4 + 1] = v;
        }
      }
    }
  }
  if (l == 0) {
    A.aux[(int64_t)c * 4 + 0] = sla;
    A.aux[(int64_t)c * 4 + 2] = slp;
    A.aux[(int64_t)c * 4 + 3] = 0.0;
  }
}

// scale = np.random.choice([0.1, 0.5, 1, 3, 10], p=[.1, .15, .5, .15, .1]) (pulsar_gibbs.py:430-433)
__device__ __forceinline__ double ec_scale(double u) {
  if (u < 0.1) return 0.1;
  if (u < 0.25) return 0.5;
  if (u < 0.75) return 1.0;
  if (u < 0.9) return 3.0;
  return 10.0;
}

// One Metropolis proposal per chain (pulsar_gibbs.py:458-462): scale, one ECORR parameter
// uniformly, q[par] += randn * (0.05 n_e) * scale.  xq = x with the jump applied;
// prop[c] = {x column, log U, inside prior, proposed value}.
__global__ __launch_bounds__(256) void k_ecorr_propose(EcorrMhArgs A) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= A.n_chain) return;
  double sc, z, u;
  int p;
  if (A.inj) {
    const double* q = A.inj + ((int64_t)A.step * A.n_chain + c) * 4;
    sc = q[0];
    p = (int)q[1];
    z = q[2];
    u = q[3];
  } else {
    const long long sw = gs_sweep(A.sweep, A.sweep_dev), gc = A.chain_base + c;
    const uint32_t s3 = 3u * (uint32_t)A.step;
    double u1, u2, v1, v2, u4;
    gs_uniform2(gs_counter(s3, sw, gc, 0, GS_EV_ECORR), A.key, u1, u2);
    gs_uniform2(gs_counter(s3 + 1, sw, gc, 0, GS_EV_ECORR), A.key, v1, v2);
    gs_uniform2(gs_counter(s3 + 2, sw, gc, 0, GS_EV_ECORR), A.key, u, u4);
    sc = ec_scale(u1);
    p = min((int)(u2 * A.n_e), A.n_e - 1);
    z = sqrt(-2.0 * log(1.0 - v1)) * cospi(2.0 * v2);
  }
  const double* xr = A.x + (int64_t)c * A.ldx;
  double* qr = A.xq + (int64_t)c * A.ldx;
  for (int j = 0; j < A.n_param; ++j) qr[j] = xr[j];
  const int col = A.ecol[p];
  const double qv = xr[col] + (z * (0.05 * A.n_e)) * sc;
  qr[col] = qv;
  double* pr = A.prop + (int64_t)c * 4;
  pr[0] = (double)col;
  pr[1] = log(u);
  pr[2] = (qv >= A.emin[p] && qv <= A.emax[p]) ? 1.0 : 0.0;  // Uniform prior (:613-617)
  pr[3] = qv;
}

// Metropolis decision (pulsar_gibbs.py:465-472): lnL = lnl_R + (sum d_E^2/a - sum log a -
// sum log phi_E) / 2 (the chain-independent constants cancel); -inf when a factor was not
// positive definite or the proposal left the prior.  init: only record lnL0 at x.
__global__ __launch_bounds__(256) void k_ecorr_accept(EcorrMhArgs A) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= A.n_chain) return;
  const double* ax = A.aux + (int64_t)c * 4;
  const bool pd = !(A.info && A.info[c]) && !(A.pinfo && A.pinfo[c]);
  const double l1 = pd ? A.lnl[c] + 0.5 * (ax[1] - ax[0] - ax[2]) : -INFINITY;
  if (A.init) {
    A.lnl0[c] = l1;
    return;
  }
  const double* pr = A.prop + (int64_t)c * 4;
  const double diff = (pr[2] != 0.0) ? l1 - A.lnl0[c] : -INFINITY;
  if (A.q_rec)
    for (int j = 0; j < A.n_e; ++j) A.q_rec[(int64_t)c * A.n_e + j] = A.xq[(int64_t)c * A.ldx + A.ecol[j]];
  if (diff > pr[1]) {
    A.x[(int64_t)c * A.ldx + (int)pr[0]] = pr[3];
    A.lnl0[c] = l1;
    if (A.n_acc) A.n_acc[c] += 1;
  }
}

// b_E | b_R (one thread per (chain, epoch)) and the scatter of b_R into b's original
// column order (threads ne .. ne + mR - 1).
__global__ __launch_bounds__(256) void k_ecorr_bdraw_e(EcorrBArgs A) {
  const int c = blockIdx.y;
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= A.ne + A.mR) return;
  if (A.chain_mask && !A.chain_mask[c]) return;  // gate (pulsar_gibbs.py:697-698)
  const double* bR = A.bR + (int64_t)c * A.ldbR;
  double* b = A.b + (int64_t)c * A.ldb;
  if (j >= A.ne) {
    b[A.rcol[j - A.ne]] = bR[j - A.ne];
    return;
  }
  const int e = j;
  double inv, lg;
  ec_phi(A.x[(int64_t)c * A.ldx + A.xcol[A.ebk[e]]], inv, lg);
  const double a = A.Dg[e] + inv;
  const double* row = A.Bx + (int64_t)e * A.ldbx;
  double s = row[A.mR];
  for (int t = 0; t < A.mR; ++t) s = fma(-row[t], bR[t], s);
  double z;
  if (A.z) {
    z = A.z[(int64_t)c * A.m + A.ecid[e]];
  } else {
    double n1, n2;
    gs_normal2(gs_counter((uint32_t)(e >> 1), gs_sweep(A.sweep, A.sweep_dev), A.chain_base + c, 0, A.event),
               A.key, n1, n2);
    z = (e & 1) ? n2 : n1;
  }
  b[A.ecid[e]] = s / a + z / sqrt(a);
}

template <int NB>
void launch_schur_nb(hipStream_t s, const EcorrSchurArgs& a) {
  static bool attr = false;
  const size_t lds = (size_t)2 * EC_CH * 16 * NB * sizeof(double);
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_ecorr_schur<NB>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL(k_ecorr_schur<NB>, dim3((unsigned)((a.n_chain + EC_WAVES - 1) / EC_WAVES)),
                     dim3(64 * EC_WAVES), lds, s, a);
}

}  // namespace

bool ecorr_nb_supported(int nb) { return nb >= 1 && nb <= 6; }  // NB 7, 8 spill

int launch_ecorr_schur(hipStream_t s, const EcorrSchurArgs& a) {
  switch (a.ldbx / 16) {
    case 1: launch_schur_nb<1>(s, a); break;
    case 2: launch_schur_nb<2>(s, a); break;
    case 3: launch_schur_nb<3>(s, a); break;
    case 4: launch_schur_nb<4>(s, a); break;
    case 5: launch_schur_nb<5>(s, a); break;
    case 6: launch_schur_nb<6>(s, a); break;
    case 7: launch_schur_nb<7>(s, a); break;
    case 8: launch_schur_nb<8>(s, a); break;
    default: return 1;
  }
  return 0;
}

int launch_ecorr_propose(hipStream_t s, const EcorrMhArgs& a) {
  hipLaunchKernelGGL(k_ecorr_propose, dim3((unsigned)((a.n_chain + 255) / 256)), dim3(256), 0, s, a);
  return 0;
}

int launch_ecorr_accept(hipStream_t s, const EcorrMhArgs& a) {
  hipLaunchKernelGGL(k_ecorr_accept, dim3((unsigned)((a.n_chain + 255) / 256)), dim3(256), 0, s, a);
  return 0;
}

int launch_ecorr_bdraw_e(hipStream_t s, const EcorrBArgs& a) {
  hipLaunchKernelGGL(k_ecorr_bdraw_e, dim3((unsigned)((a.ne + a.mR + 255) / 256), (unsigned)a.n_chain), dim3(256),
                     0, s, a);
  return 0;
}
