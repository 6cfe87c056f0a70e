// b|rho for large free-spectrum blocks (64 < NF <= 255; config 5: n_f = 100, NF = 200).
//
// Reference: PulsarBlockGibbs.update_b pulsar_gibbs.py:489-520 (same law as the
// SVD draw; see gibbs_bdraw.hip).  Same algorithm as the register-tile draw
// (gibbs_tile.h) -- upper Cholesky of the dF-augmented Schur block on 16 x 16 fp64
// MFMA tiles, diagonal tiles inverted by DPP column elimination, U^T and U_KK^-T
// stored for the backward solve -- with one difference: an NF = 200 block has 91
// upper tiles (182 KB), more than a wavefront's registers, so the tiles of each
// system live in a global workspace owned by the context (tile-major, element
// (s, lane) at s * 64 + lane: every tile load/store is 4 coalesced 512-byte rows,
// and each element is only ever written and read back by its own lane).
//
// One wavefront per system, BIG_WPB per workgroup, no inter-wave communication.
// The tile count is NT = NF / 16 + 1: the augmented column NF always has a slot
// (local index CP = NF % 16 of the last tile row, the template parameter).  In
// config 5 the sweep is dominated by the per-chain TNT (gs_white_tnt, fp64 MFMA):
// this draw is ~1 % of it.
//
// Normals: slot j of the Philox counter gives the packed normals z[2j], z[2j+1]
// of [z_F | z_M] (the NF <= 64 kernels use slot = lane for (z_F[lane], z_M[lane])).
#include "gibbs_common.h"
#include "gibbs_internal.h"
#include "gibbs_tile.h"

namespace {

constexpr int BIG_WPB = 4;
constexpr int BIG_NFMAX = 255;
constexpr int BIG_V = 272;  // per-wave vector slots (>= 16 NT)

// per-wave LDS: tb 272 | vb 64 | zb 320 | xb 272 | yb 272 | ph 272
constexpr int BIG_SCR = 272 + 64 + 320 + 3 * BIG_V;

__device__ __forceinline__ gs_d4 ld_tile(const double* __restrict__ ws, int tl, int lane) {
  const double* t = ws + (int64_t)tl * 256 + lane;
  gs_d4 v;
#pragma unroll
  for (int s = 0; s < 4; ++s) v[s] = t[64 * s];
  return v;
}

__device__ __forceinline__ void st_tile(double* __restrict__ ws, int tl, int lane, const gs_d4 v) {
  double* t = ws + (int64_t)tl * 256 + lane;
#pragma unroll
  for (int s = 0; s < 4; ++s) t[64 * s] = v[s];
}

template <int CP>
__global__ __launch_bounds__(64 * BIG_WPB) void k_bdraw_big(BdrawArgs A, double* wsp, int64_t ws_stride) {
  using namespace gtile;
  extern __shared__ double lds[];
  const int wave = gs_wave_id(), lane = threadIdx.x & 63;
  const int q = lane >> 4, c = lane & 15;
  const int64_t n_sys = (int64_t)A.n_psr * A.n_chain;
  const int64_t sys = (int64_t)blockIdx.x * BIG_WPB + wave;
  if (sys >= n_sys) return;  // no workgroup barriers below
  const int p = (int)(sys / A.n_chain), ch = (int)(sys % A.n_chain);
  if (A.chain_mask && A.chain_mask[A.mask_per_sys ? sys : (int64_t)ch] == 0) return;  // gate closed
  const int NF = A.NF, NMX = A.NMX, NT = NF / 16 + 1, LD = NF + 1;
  const int nM = __builtin_amdgcn_readfirstlane(A.nm[p]);  // uniform: SGPR
  double* ws = wsp + sys * ws_stride;
  double* scr = lds + wave * BIG_SCR;
  double* tb = scr;
  double* vb = tb + 272;
  double* zb = vb + 64;
  double* xb = zb + 320;
  double* yb = xb + BIG_V;
  double* ph = yb + BIG_V;
  const double* mb = A.model + (A.model_per_sys ? sys : (int64_t)p) * A.mstride;
  const double* S0 = mb;
  const double* G = mb + NF * LD + NF;
  const double* h = G + NMX * LD;
  const double* R = h + NMX;
  const int32_t* fidx = A.fidx + (int64_t)p * NF;
  const int32_t* midx = A.midx + (int64_t)p * NMX;

  // ---- per-system vectors into LDS: phiinv_F, [z_F | z_M]
  for (int f = lane; f < 16 * NT; f += 64) ph[f] = (f < NF) ? A.phiinv_F[(A.phi_per_chain ? (int64_t)ch : sys) * NF + f] : 1.0;
  if (A.z) {
    for (int f = lane; f < NF; f += 64) zb[f] = A.z[sys * A.ldb + fidx[f]];
    if (lane < nM) zb[NF + lane] = A.z[sys * A.ldb + midx[lane]];
  } else {
    for (int j = lane; 2 * j < NF + nM; j += 64) {
      double n1, n2;
      gs_normal2(gs_counter(j, gs_sweep(A.sweep, A.sweep_dev), A.chain_base + ch, p + A.psr_base, A.event), A.key, n1, n2);
      zb[2 * j] = n1;
      if (2 * j + 1 < NF + nM) zb[2 * j + 1] = n2;
    }
  }
  lds_fence();

  // ---- upper tiles of [[S0 + diag(phiinv_F), dF], [dF^T, 1]] (identity padding)
  for (int I = 0; I < NT; ++I)
    for (int J = I; J < NT; ++J) {
      gs_d4 v;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int r = 16 * I + 4 * s + q, col = 16 * J + c;
        int a = -1;
        if (r < NF && col < NF) a = r * LD + col;
        else if (r < NF && col == NF) a = r * LD + NF;  // dF[r] (gs_prefix)
        else if (r == NF && col < NF) a = col * LD + NF;
        double e = (a >= 0) ? S0[a] : 0.0;
        if (r == col) e += (r < NF) ? ph[r] : 1.0;
        v[s] = e;
      }
      st_tile(ws, tix(I, J, NT), lane, v);
    }

  // ---- factorisation
  int fail = 0;
  double ylast = 0.0;
  for (int K = 0; K < NT; ++K) {
    gs_d4 Ad = ld_tile(ws, tix(K, K, NT), lane), B;
    double rsd;
    if (K == NT - 1) {
      tile_elim<CP>(Ad, B, rsd, q, c);
      if (CP > 0) {
        const double yl = bcast_group_bp(Ad[CP >> 2], CP & 3, c);
        ylast = (c < CP) ? yl * rsd : 0.0;
      }
    } else {
      tile_elim<16>(Ad, B, rsd, q, c);
    }
    const unsigned long long badm = __ballot(!(rsd > 0.0 && rsd < __builtin_inf())) & 0xffffull;
    if (!fail && badm) fail = 16 * K + __ffsll((long long)badm);
    gs_d4 V;
#pragma unroll
    for (int s = 0; s < 4; ++s) V[s] = B[s] * rsd;
    for (int J = K + 1; J < NT; ++J) {
      const gs_d4 z = {0.0, 0.0, 0.0, 0.0};
      st_tile(ws, tix(K, J, NT), lane, mfma_tn(z, V, ld_tile(ws, tix(K, J, NT), lane)));
    }
    st_tile(ws, tix(K, K, NT), lane, transpose(V, tb, q, c));  // U_KK^-T for the backward solve
    for (int I = K + 1; I < NT; ++I) {
      const gs_d4 xk = ld_tile(ws, tix(K, I, NT), lane);
      for (int J = I; J < NT; ++J) {
        const int tl = tix(I, J, NT);
        st_tile(ws, tl, lane, mfma_tn_sub(ld_tile(ws, tl, lane), xk, ld_tile(ws, tix(K, J, NT), lane)));
      }
    }
    for (int J = K + 1; J < NT; ++J) {  // block row K final: keep U_KJ^T
      const int tl = tix(K, J, NT);
      st_tile(ws, tl, lane, transpose(ld_tile(ws, tl, lane), tb, q, c));
    }
  }

  // ---- y = U^-T dF: column CP of U_K,last (row CP of the stored transpose); last: ylast
  for (int K = 0; K + 1 < NT; ++K) {
    const gs_d4 ut = ld_tile(ws, tix(K, NT - 1, NT), lane);
    double sel = ut[0];
#pragma unroll
    for (int s = 1; s < 4; ++s) sel = ((CP >> 2) == s) ? ut[s] : sel;
    const double yk = bcast_group_bp(sel, CP & 3, c);
    if (q == 0) yb[16 * K + c] = yk;
  }
  if (q == 0) yb[16 * (NT - 1) + c] = ylast;
  lds_fence();

  // ---- backward: U x = y + z_F
  for (int K = NT - 1; K >= 0; --K) {
    double pacc = 0.0;
    for (int J = K + 1; J < NT; ++J) {
      const gs_d4 ut = ld_tile(ws, tix(K, J, NT), lane);
#pragma unroll
      for (int s = 0; s < 4; ++s) pacc = fma(ut[s], xb[16 * J + 4 * s + q], pacc);
    }
    pacc = qsum(pacc);
    const int i = 16 * K + c;
    const double w = yb[i] + ((i < NF) ? zb[i] : 0.0) - pacc;
    const gs_d4 sr = to_row(w, vb, q, c);
    const gs_d4 W = ld_tile(ws, tix(K, K, NT), lane);
    double p2 = 0.0;
#pragma unroll
    for (int s = 0; s < 4; ++s) p2 = fma(W[s], sr[s], p2);
    const double xk = qsum(p2);
    lds_fence();
    if (q == 0) xb[i] = (i < NF) ? xk : 0.0;
    lds_fence();
  }

  // ---- fixed-prior block: x_M = h + R z_M - G x_F (lane = row).  A failed factorisation
  // (non-PD Sigma, wave-uniform) keeps the previous b.
  if (fail) {
    if (A.info && lane == 0) A.info[sys] = fail;
    if (A.fail_count && lane == 0) A.fail_count[sys] += 1;
    return;
  }
  if (lane < nM) {
    double v = h[lane];
    for (int j = 0; j < nM; ++j) v = fma(R[lane * NMX + j], zb[NF + j], v);
    for (int f = 0; f < NF; ++f) v = fma(-G[lane * LD + f], xb[f], v);
    A.b[sys * A.ldb + midx[lane]] = v;
  }
  for (int f = lane; f < NF; f += 64) A.b[sys * A.ldb + fidx[f]] = xb[f];
  if (A.info && lane == 0) A.info[sys] = fail;
}

template <int CP>
void launch_big_cp(hipStream_t s, const BdrawArgs& a, double* ws, int64_t ws_stride) {
  const int64_t n_sys = (int64_t)a.n_psr * a.n_chain;
  const size_t lds = (size_t)BIG_WPB * BIG_SCR * sizeof(double);
  hipLaunchKernelGGL(k_bdraw_big<CP>, dim3((unsigned)((n_sys + BIG_WPB - 1) / BIG_WPB)), dim3(64 * BIG_WPB), lds, s,
                     a, ws, ws_stride);
}

}  // namespace

int64_t big_ws_doubles_per_sys(int NF) {
  const int NT = NF / 16 + 1;
  return (int64_t)NT * (NT + 1) / 2 * 256;
}

bool big_nf_supported(int NF) { return NF > 64 && NF <= BIG_NFMAX && (NF % 2) == 0; }

int launch_bdraw_big(hipStream_t s, const BdrawArgs& a, double* ws) {
  if (!big_nf_supported(a.NF)) return 1;
  const int64_t st = big_ws_doubles_per_sys(a.NF);
  switch (a.NF % 16) {
    case 0: launch_big_cp<0>(s, a, ws, st); break;
    case 2: launch_big_cp<2>(s, a, ws, st); break;
    case 4: launch_big_cp<4>(s, a, ws, st); break;
    case 6: launch_big_cp<6>(s, a, ws, st); break;
    case 8: launch_big_cp<8>(s, a, ws, st); break;
    case 10: launch_big_cp<10>(s, a, ws, st); break;
    case 12: launch_big_cp<12>(s, a, ws, st); break;
    default: launch_big_cp<14>(s, a, ws, st); break;
  }
  return 0;
}
