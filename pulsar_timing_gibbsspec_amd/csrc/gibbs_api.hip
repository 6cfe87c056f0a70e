// C-ABI of the MI355X Gibbs hot path (include/pulsar_gibbs.h), plus the TNT,
// prefix-factorisation and Philox kernels.
#include <stdio.h>

#include <string>

#include "gibbs_internal.h"

struct gs_ctx {
  int device;
  hipStream_t stream;
  uint64_t seed;
  int bcast;     // GS_OPT_BCAST
  int psr_base;  // GS_OPT_PSR_BASE: global index of this shard's pulsar 0 (RNG counters)
  int x_per_sys = 0;  // GS_OPT_X_PER_SYS
  int grid_exact = 0;  // GS_OPT_GRID_EXACT
  int brec_nc = 0;     // GS_OPT_BREC_CHAINS
  int phi_per_chain = 0;  // GS_OPT_PHI_PER_CHAIN
  int sweep_sched = 0;    // GS_OPT_SWEEP_SCHED
  int dbg_handoff = 0;    // GS_OPT_DEBUG_HANDOFF
  int last_shape = 0;     // GS_OPT_LAST_SWEEP_SHAPE (read only)
  const int64_t* sweep_dev = nullptr;  // gs_ctx_set_sweep_counter
  int32_t* fail_counts = nullptr;      // gs_ctx_set_fail_counts
  int32_t* grid_fallback = nullptr;    // gs_ctx_set_grid_fallback_counter
  double* bdraw_lnl = nullptr;         // gs_ctx_set_bdraw_lnl
  const double* bdraw_lnl_model = nullptr;
  double* ws = nullptr;  // tile workspace of the large-NF b-draw (grown on demand)
  size_t ws_bytes = 0;
};

namespace {

thread_local std::string g_err;

int fail_arg(int idx, const char* what) {
  g_err = std::string("argument ") + std::to_string(idx) + ": " + what;
  return idx;
}

int check_hip(hipError_t e, const char* where) {
  if (e == hipSuccess) return 0;
  g_err = std::string(where) + ": " + hipGetErrorString(e);
  return -(int)e;
}

int after_launch(const char* where) { return check_hip(hipGetLastError(), where); }

// the NF-dispatching launchers return 1 for an NF without an instantiation and 2 when the
// dynamic-LDS attribute could not be set (hipFuncSetAttribute)
int launch_rc(int rc, const char* kernel) {
  if (rc == 1) return fail_arg(4, "unsupported NF");
  if (rc == 2) {
    g_err = std::string(kernel) + ": hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed";
    return -(int)hipErrorInvalidValue;
  }
  return after_launch(kernel);
}

// grow the context workspace (large-NF b-draw tiles, prefix scratch) to `need` bytes
int ensure_ws(gs_ctx* ctx, size_t need) {
  if (need <= ctx->ws_bytes) return 0;
  int rc = check_hip(hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
  if (rc) return rc;
  if (ctx->ws) (void)hipFree(ctx->ws);
  ctx->ws = nullptr;
  ctx->ws_bytes = 0;
  rc = check_hip(hipMalloc((void**)&ctx->ws, need), "hipMalloc(context workspace)");
  if (rc) return rc;
  ctx->ws_bytes = need;
  return 0;
}

gs_key key_of(const gs_ctx* c) {
  gs_key k;
  k.k0 = (uint32_t)(c->seed & 0xffffffffu);
  k.k1 = (uint32_t)(c->seed >> 32);
  return k;
}

typedef double d4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------ TNT (a2)
// Blocked compensated accumulation: each MFMA chain sums one block of 64 TOAs from zero, and
// the block sums enter a two-sum (hi, lo) pair, so the rounding error grows with the block
// length rather than with n_toa (n_toa = 10^4 in configs[4]: a plain running sum was ~5x
// less accurate than numpy's blocked dgemm).  Once per model: accuracy over speed.
__device__ __forceinline__ void two_sum_acc(double& hi, double& lo, double x) {
  const double s = hi + x;
  const double bb = s - hi;
  lo += (hi - (s - bb)) + (x - bb);
  hi = s;
}

// grid (n_psr, nb*nb), nb = ceil(m_max/16); 4 wavefronts take alternate 64-TOA blocks.
// D[i][j] += sum_t (T[t][I0+i] / N[t]) T[t][J0+j] with v_mfma_f64_16x16x4f64:
// A lane l holds A[l&15][l>>4], B lane l holds B[l>>4][l&15];
// C/D lane l reg r holds D[(l>>4) + 4r][l&15].
__global__ __launch_bounds__(256) void k_tnt(const gs_tnt_desc* desc, int nb, const double* T,
                                             const double* Nv, const double* r, double* TNT) {
  __shared__ double red[3][8][64];
  const gs_tnt_desc D = desc[blockIdx.x];
  const int bi = blockIdx.y / nb, bj = blockIdx.y % nb;
  const int m = (int)D.m;
  if (bi * 16 >= m || bj * 16 >= m) return;
  const int w = gs_wave_id(), l = threadIdx.x & 63;
  const int i = l & 15, k = l >> 4;
  const int ci = bi * 16 + i, cj = bj * 16 + i;
  const double* Tp = T + D.T_off;
  const double* Np = Nv + D.toa_off;
  const int64_t n = D.n_toa;
  d4 hi = {0.0, 0.0, 0.0, 0.0}, lo = {0.0, 0.0, 0.0, 0.0};
  for (int64_t tb = (int64_t)w * 64; tb < n; tb += 256) {
    d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
    for (int s = 0; s < 16; ++s) {
      const int64_t t = tb + s * 4 + k;
      const bool ok = t < n;
      const double a = (ok && ci < m) ? Tp[t * m + ci] / Np[t] : 0.0;
      const double b = (ok && cj < m) ? Tp[t * m + cj] : 0.0;
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    }
    for (int q = 0; q < 4; ++q) {
      double h = hi[q], e = lo[q];
      two_sum_acc(h, e, acc[q]);
      hi[q] = h;
      lo[q] = e;
    }
  }
  if (w > 0) {
    for (int q = 0; q < 4; ++q) {
      red[w - 1][q][l] = hi[q];
      red[w - 1][4 + q][l] = lo[q];
    }
  }
  __syncthreads();
  if (w == 0) {
    for (int q = 0; q < 4; ++q) {
      double h = hi[q], e = lo[q];
      for (int u = 0; u < 3; ++u) {
        two_sum_acc(h, e, red[u][q][l]);
        e += red[u][4 + q][l];
      }
      const int row = bi * 16 + (l >> 4) + 4 * q, col = bj * 16 + (l & 15);
      if (row < m && col < m) TNT[D.tnt_off + (int64_t)row * m + col] = h + e;
    }
  }
  (void)r;
}

// d = T^T (r / N): grid (n_psr, ceil(m_max/64)), 4 wavefronts take alternate 64-TOA blocks,
// block sums compensated as in k_tnt.
__global__ __launch_bounds__(256) void k_tnr(const gs_tnt_desc* desc, const double* T,
                                             const double* Nv, const double* r, double* d) {
  __shared__ double red[2][4][64];
  const gs_tnt_desc D = desc[blockIdx.x];
  const int w = gs_wave_id(), l = threadIdx.x & 63;
  const int m = (int)D.m;
  const int j = blockIdx.y * 64 + l;
  double hi = 0.0, lo = 0.0;
  if (j < m) {
    const double* Tp = T + D.T_off;
    const double* rp = r + D.toa_off;
    const double* Np = Nv + D.toa_off;
    for (int64_t tb = (int64_t)w * 64; tb < D.n_toa; tb += 256) {
      const int64_t te = tb + 64 < D.n_toa ? tb + 64 : D.n_toa;
      double s = 0.0;
      for (int64_t t = tb; t < te; ++t) s = fma(Tp[t * m + j], rp[t] / Np[t], s);
      two_sum_acc(hi, lo, s);
    }
  }
  red[0][w][l] = hi;
  red[1][w][l] = lo;
  __syncthreads();
  if (w == 0 && j < m) {
    double h = red[0][0][l], e = red[1][0][l];
    for (int u = 1; u < 4; ++u) {
      two_sum_acc(h, e, red[0][u][l]);
      e += red[1][u][l];
    }
    d[D.d_off + j] = h + e;
  }
}

__global__ void k_philox(int64_t n, const uint32_t* ctr, uint32_t* out, gs_key key) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  gs_u4 c = {ctr[4 * i], ctr[4 * i + 1], ctr[4 * i + 2], ctr[4 * i + 3]};
  const gs_u4 w = philox4x32_10(c, key.k0, key.k1);
  out[4 * i] = w.x;
  out[4 * i + 1] = w.y;
  out[4 * i + 2] = w.z;
  out[4 * i + 3] = w.w;
}

// register-tile b draw / fused sweep / likelihood: any even NF <= 64 (one lane per column)
bool nf_supported(int NF) { return NF > 0 && NF <= 64 && (NF % 2) == 0; }

}  // namespace

// ====================================================================== C-ABI
extern "C" {

int gs_version(void) { return GS_ABI_VERSION; }

#ifndef GS_SRC_HASH
#define GS_SRC_HASH "unknown"
#endif
#ifndef GS_HIPCC_VER
#define GS_HIPCC_VER "unknown"
#endif
#ifndef GS_BUILD_STAMP
#define GS_BUILD_STAMP "unknown"
#endif
const char* gs_build_info(void) {
  return "sources " GS_SRC_HASH "; hipcc " GS_HIPCC_VER "; built " GS_BUILD_STAMP;
}

const char* gs_last_error(void) { return g_err.c_str(); }

int gs_ctx_create(int device, uint64_t seed, void* stream, gs_ctx** out) {
  if (!out) return fail_arg(4, "out is NULL");
  int rc = check_hip(hipSetDevice(device), "hipSetDevice");
  if (rc) return rc;
  gs_ctx* c = new gs_ctx;
  c->device = device;
  c->stream = (hipStream_t)stream;
  c->seed = seed;
  c->bcast = 3;
  c->psr_base = 0;
  *out = c;
  return 0;
}

int gs_ctx_destroy(gs_ctx* ctx) {
  if (ctx && ctx->ws) {
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(ctx->ws);
  }
  delete ctx;
  return 0;
}

int gs_ctx_set_stream(gs_ctx* ctx, void* stream) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  ctx->stream = (hipStream_t)stream;
  return 0;
}

int gs_ctx_set_seed(gs_ctx* ctx, uint64_t seed) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  ctx->seed = seed;
  return 0;
}

int gs_ctx_set_option(gs_ctx* ctx, int option, int value) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  switch (option) {
    case GS_OPT_BCAST:
      if (value < 0 || value > 3) return fail_arg(3, "GS_OPT_BCAST must be 0, 1, 2 or 3");
      ctx->bcast = value;
      return 0;
    case GS_OPT_PSR_BASE:
      if (value < 0 || value > (1 << 23)) return fail_arg(3, "GS_OPT_PSR_BASE out of range");
      ctx->psr_base = value;
      return 0;
    case GS_OPT_GRID_EXACT:
      if (value < 0 || value > 3) return fail_arg(3, "GS_OPT_GRID_EXACT must be 0, 1, 2 or 3");
      ctx->grid_exact = value;
      return 0;
    case GS_OPT_BREC_CHAINS:
      if (value < 0) return fail_arg(3, "GS_OPT_BREC_CHAINS must be >= 0");
      ctx->brec_nc = value;
      return 0;
    case GS_OPT_X_PER_SYS:
      if (value != 0 && value != 1) return fail_arg(3, "GS_OPT_X_PER_SYS must be 0 or 1");
      ctx->x_per_sys = value;
      return 0;
    case GS_OPT_PHI_PER_CHAIN:
      if (value != 0 && value != 1) return fail_arg(3, "GS_OPT_PHI_PER_CHAIN must be 0 or 1");
      ctx->phi_per_chain = value;
      return 0;
    case GS_OPT_SWEEP_SCHED:
      if (value < 0 || value > 3) return fail_arg(3, "GS_OPT_SWEEP_SCHED must be 0, 1, 2 or 3");
      ctx->sweep_sched = value;
      return 0;
    case GS_OPT_DEBUG_HANDOFF:
      if (value != 0 && value != 1) return fail_arg(3, "GS_OPT_DEBUG_HANDOFF must be 0 or 1");
      ctx->dbg_handoff = value;
      return 0;
    case GS_OPT_LAST_SWEEP_SHAPE:
      return fail_arg(2, "GS_OPT_LAST_SWEEP_SHAPE is read only");
    default:
      return fail_arg(2, "unknown option");
  }
}

int gs_ctx_get_option(gs_ctx* ctx, int option) {
  if (!ctx) return -1;
  if (option == GS_OPT_BCAST) return ctx->bcast;
  if (option == GS_OPT_PSR_BASE) return ctx->psr_base;
  if (option == GS_OPT_X_PER_SYS) return ctx->x_per_sys;
  if (option == GS_OPT_GRID_EXACT) return ctx->grid_exact;
  if (option == GS_OPT_BREC_CHAINS) return ctx->brec_nc;
  if (option == GS_OPT_PHI_PER_CHAIN) return ctx->phi_per_chain;
  if (option == GS_OPT_SWEEP_SCHED) return ctx->sweep_sched;
  if (option == GS_OPT_DEBUG_HANDOFF) return ctx->dbg_handoff;
  if (option == GS_OPT_LAST_SWEEP_SHAPE) return ctx->last_shape;
  return -1;
}

int gs_ctx_set_sweep_counter(gs_ctx* ctx, const int64_t* sweep_dev) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  ctx->sweep_dev = sweep_dev;
  return 0;
}

int gs_ctx_set_fail_counts(gs_ctx* ctx, int32_t* counts) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  ctx->fail_counts = counts;
  return 0;
}

int gs_ctx_set_grid_fallback_counter(gs_ctx* ctx, int32_t* counter) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  ctx->grid_fallback = counter;
  return 0;
}

int gs_ctx_set_bdraw_lnl(gs_ctx* ctx, double* lnl, const double* model) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if ((lnl == nullptr) != (model == nullptr)) return fail_arg(3, "lnl and model go together (both or neither)");
  ctx->bdraw_lnl = lnl;
  ctx->bdraw_lnl_model = model;
  return 0;
}

int gs_counter_add(gs_ctx* ctx, int64_t* counter, int64_t inc) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (!counter) return fail_arg(2, "counter is NULL");
  launch_counter_add(ctx->stream, counter, inc);
  return after_launch("k_counter_add");
}

int64_t gs_model_stride(int NF, int NMX) { return model_stride_doubles(NF, NMX); }

int gs_sweep_lds_bytes(int NF, int NMX) {  // the default (tile) variant: model block in the tile layout
  return (int)((model_tiled_doubles(NF, NMX) + (gs_tile_scr(NF) + 128) * GS_SWEEP_WPB) * 8);
}

int gs_tnt(gs_ctx* ctx, int n_psr, int m_max, const gs_tnt_desc* desc, const double* T,
           const double* Nvec, const double* r, double* TNT, double* d) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_psr < 0) return fail_arg(2, "n_psr < 0");
  if (m_max <= 0 || m_max > 4096) return fail_arg(3, "m_max out of range");
  if (!desc) return fail_arg(4, "desc is NULL");
  if (!T || !Nvec || !r) return fail_arg(5, "T/Nvec/r is NULL");
  if (n_psr == 0) return 0;
  const int nb = (m_max + 15) / 16;
  if (TNT) {
    hipLaunchKernelGGL(k_tnt, dim3(n_psr, nb * nb), dim3(256), 0, ctx->stream, desc, nb, T, Nvec, r, TNT);
    int rc = after_launch("k_tnt");
    if (rc) return rc;
  }
  if (d) {
    hipLaunchKernelGGL(k_tnr, dim3(n_psr, (m_max + 63) / 64), dim3(256), 0, ctx->stream, desc, T, Nvec, r, d);
    return after_launch("k_tnr");
  }
  return 0;
}

int gs_tnt_dd(gs_ctx* ctx, int n_psr, int m_max, const gs_tnt_desc* desc, const double* T, const double* Nvec,
              const double* r, double* TNT, double* TNT_lo, double* d, double* d_lo) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_psr < 0) return fail_arg(2, "n_psr < 0");
  if (m_max <= 0 || m_max > 4096) return fail_arg(3, "m_max out of range");
  if (!desc) return fail_arg(4, "desc is NULL");
  if (!T || !Nvec || !r) return fail_arg(5, "T/Nvec/r is NULL");
  if (n_psr == 0) return 0;
  return check_hip(launch_tnt_dd(ctx->stream, n_psr, m_max, desc, T, Nvec, r, TNT, TNT_lo, d, d_lo), "k_tnt_dd");
}

int gs_prefix_dd(gs_ctx* ctx, int n_psr, int n_chain, int NF, int NMX, const gs_prefix_desc* desc,
                 int64_t tnt_cstride, int64_t d_cstride, const double* TNT, const double* TNT_lo, const double* d,
                 const double* d_lo, const int32_t* fidx, const int32_t* midx, const double* phiinv_fixed,
                 double* model, int32_t* info) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_psr < 0) return fail_arg(2, "n_psr < 0");
  if (n_chain < 0) return fail_arg(3, "n_chain < 0");
  if (NF <= 0 || NF > 254 || (NF & 1)) return fail_arg(4, "NF must be even and <= 254");
  if (NMX < 0 || NMX > GS_NMX_WIDE) return fail_arg(5, "NMX must be in 0..128");
  if (!desc) return fail_arg(6, "desc is NULL");
  if (tnt_cstride < 0) return fail_arg(7, "tnt_cstride < 0");
  if (d_cstride < 0) return fail_arg(8, "d_cstride < 0");
  if (!TNT || !d || !fidx || !midx || !phiinv_fixed || !model) return fail_arg(9, "NULL array");
  if (n_psr == 0 || n_chain == 0) return 0;
  PrefixArgs a;
  a.n_psr = n_psr; a.n_chain = n_chain; a.NF = NF; a.NMX = NMX;
  a.tnt_cstride = tnt_cstride; a.d_cstride = d_cstride; a.mstride = model_stride_doubles(NF, NMX);
  a.desc = desc; a.TNT = TNT; a.TNT_lo = TNT_lo; a.d = d; a.d_lo = d_lo; a.phfix = phiinv_fixed;
  a.fidx = fidx; a.midx = midx; a.model = model; a.info = info;
  a.gscr = nullptr;
  a.gstride = prefix_scratch_doubles(NF, NMX);
  if (!prefix_scratch_in_lds(NF, NMX)) {
    const int rc = ensure_ws(ctx, (size_t)n_psr * n_chain * a.gstride * sizeof(double));
    if (rc) return rc;
    a.gscr = ctx->ws;
  }
  return check_hip(launch_prefix_dd(ctx->stream, a), "k_prefix_dd");
}

int gs_prefix_sys(gs_ctx* ctx, int n_psr, int n_chain, int NF, int NMX, const gs_prefix_desc* desc,
                  int64_t tnt_cstride, int64_t d_cstride, const double* TNT, const double* d,
                  const int32_t* fidx, const int32_t* midx, const double* phiinv_fixed,
                  double* model, int32_t* info) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (!TNT || !d || !fidx || !midx || !phiinv_fixed || !model) return fail_arg(9, "NULL array");
  return gs_prefix_dd(ctx, n_psr, n_chain, NF, NMX, desc, tnt_cstride, d_cstride, TNT, nullptr, d, nullptr, fidx,
                      midx, phiinv_fixed, model, info);
}

int gs_prefix(gs_ctx* ctx, int n_psr, int NF, int NMX, const gs_prefix_desc* desc,
              const double* TNT, const double* d, const int32_t* fidx, const int32_t* midx,
              const double* phiinv_fixed, double* model, int32_t* info) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_psr < 0) return fail_arg(2, "n_psr < 0");
  if (NF <= 0 || NF > 254 || (NF & 1)) return fail_arg(3, "NF must be even and <= 254");
  if (NMX < 0 || NMX > GS_NMX_WIDE) return fail_arg(4, "NMX must be in 0..128");
  if (!desc || !TNT || !d || !fidx || !midx || !phiinv_fixed || !model)
    return fail_arg(5, "NULL array");
  return gs_prefix_sys(ctx, n_psr, 1, NF, NMX, desc, 0, 0, TNT, d, fidx, midx, phiinv_fixed, model, info);
}

static int bdraw_impl(gs_ctx* ctx, int n_psr, int n_chain, int NF, int NMX, int ldb, const double* model,
                      const int32_t* fidx, const int32_t* midx, const int32_t* nm, const double* phiinv_F,
                      const double* z, int64_t sweep, int event, int64_t chain_base,
                      const int32_t* chain_mask, double* b, int32_t* info, int per_sys) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_psr < 0 || n_chain < 0) return fail_arg(2, "negative batch");
  const bool big = big_nf_supported(NF);
  if (!nf_supported(NF) && !big) return fail_arg(4, "NF must be even and <= 254");
  if (NMX < 0 || NMX > (big ? 64 : GS_NMX_WIDE))
    return fail_arg(5, "NMX must be in 0..128 (0..64 with NF > 64)");
  if (ldb < NF + 1) return fail_arg(6, "ldb too small");
  if (!model || !fidx || !midx || !nm || !phiinv_F || !b) return fail_arg(7, "NULL array");
  if (ctx->bdraw_lnl) return fail_arg(1, "the likelihood output (gs_ctx_set_bdraw_lnl) comes with gs_bdraw_tiled only");
  if (n_psr == 0 || n_chain == 0) return 0;
  if (big) {
    const size_t need = (size_t)n_psr * n_chain * big_ws_doubles_per_sys(NF) * sizeof(double);
    const int rc = ensure_ws(ctx, need);
    if (rc) return rc;
  }
  BdrawArgs a;
  a.n_psr = n_psr; a.n_chain = n_chain; a.NF = NF; a.NMX = NMX; a.ldb = ldb; a.event = event;
  a.mstride = model_stride_doubles(NF, NMX); a.sweep = sweep; a.chain_base = chain_base;
  a.sweep_dev = ctx->sweep_dev;
  a.model = model; a.fidx = fidx; a.midx = midx; a.nm = nm; a.chain_mask = chain_mask;
  a.phiinv_F = phiinv_F; a.z = z;
  a.b = b; a.info = info; a.key = key_of(ctx); a.bcast = ctx->bcast; a.psr_base = ctx->psr_base;
  a.fail_count = ctx->fail_counts;
  a.lnl = nullptr; a.lnl_model = nullptr; a.lnl_mstride = 0; a.persist = 0;
  a.model_per_sys = per_sys;
  a.mask_per_sys = ctx->x_per_sys;
  a.phi_per_chain = ctx->phi_per_chain;
  if (big) {
    launch_bdraw_big(ctx->stream, a, ctx->ws);
    return after_launch("k_bdraw_big");
  }
  return launch_rc(launch_bdraw(ctx->stream, a), "k_bdraw");
}

int gs_bdraw(gs_ctx* ctx, int n_psr, int n_chain, int NF, int NMX, int ldb, const double* model,
             const int32_t* fidx, const int32_t* midx, const int32_t* nm, const double* phiinv_F,
             const double* z, int64_t sweep, int event, int64_t chain_base, const int32_t* chain_mask,
             double* b, int32_t* info) {
  return bdraw_impl(ctx, n_psr, n_chain, NF, NMX, ldb, model, fidx, midx, nm, phiinv_F, z, sweep, event,
                    chain_base, chain_mask, b, info, 0);
}

int64_t gs_model_tiled_stride(int NF, int NMX) { return model_tiled_doubles(NF, NMX); }

int gs_model_tile(gs_ctx* ctx, int n_psr, int NF, int NMX, const double* model, const int32_t* nm, double* tiled) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_psr < 0) return fail_arg(2, "n_psr < 0");
  if (!nf_supported(NF)) return fail_arg(3, "NF must be even and <= 64");
  if (NMX < 0 || NMX > 64) return fail_arg(4, "NMX must be in 0..64");
  if (!model || !nm || !tiled) return fail_arg(5, "NULL array");
  if (n_psr == 0) return 0;
  launch_model_tile(ctx->stream, model, n_psr, NF, NMX, nm, tiled);
  return after_launch("k_model_tile");
}

int gs_bdraw_tiled(gs_ctx* ctx, int n_psr, int n_chain, int NF, int NMX, int ldb, const double* tiled,
                   const int32_t* fidx, const int32_t* midx, const int32_t* nm, const double* phiinv_F,
                   const double* z, int64_t sweep, int event, int64_t chain_base, const int32_t* chain_mask,
                   double* b, int32_t* info) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_psr < 0 || n_chain < 0) return fail_arg(2, "negative batch");
  if (!nf_supported(NF)) return fail_arg(4, "NF must be even and <= 64");
  if (NMX < 0 || NMX > 64) return fail_arg(5, "NMX must be in 0..64");
  if (ldb < NF + 1) return fail_arg(6, "ldb too small");
  if (!tiled || !fidx || !midx || !nm || !phiinv_F || !b) return fail_arg(7, "NULL array");
  if (n_psr == 0 || n_chain == 0) return 0;
  BdrawArgs a;
  a.n_psr = n_psr; a.n_chain = n_chain; a.NF = NF; a.NMX = NMX; a.ldb = ldb; a.event = event;
  a.mstride = model_tiled_doubles(NF, NMX); a.sweep = sweep; a.chain_base = chain_base;
  a.sweep_dev = ctx->sweep_dev;
  a.model = tiled; a.fidx = fidx; a.midx = midx; a.nm = nm; a.chain_mask = chain_mask;
  a.phiinv_F = phiinv_F; a.z = z;
  a.b = b; a.info = info; a.key = key_of(ctx); a.bcast = 3;  /* tile variant */ a.psr_base = ctx->psr_base;
  a.fail_count = ctx->fail_counts;
  a.lnl = ctx->bdraw_lnl; a.lnl_model = ctx->bdraw_lnl_model; a.lnl_mstride = model_stride_doubles(NF, NMX);
  a.persist = 0;
  a.model_per_sys = 0;
  a.mask_per_sys = ctx->x_per_sys;
  a.phi_per_chain = ctx->phi_per_chain;
  a.sched = ctx->sweep_sched;
  return launch_rc(launch_bdraw_tiled(ctx->stream, a, &ctx->last_shape), "k_bdraw_tiled");
}

int gs_bdraw_sys(gs_ctx* ctx, int n_psr, int n_chain, int NF, int NMX, int ldb, const double* model,
                 const int32_t* fidx, const int32_t* midx, const int32_t* nm, const double* phiinv_F,
                 const double* z, int64_t sweep, int event, int64_t chain_base, const int32_t* chain_mask,
                 double* b, int32_t* info) {
  return bdraw_impl(ctx, n_psr, n_chain, NF, NMX, ldb, model, fidx, midx, nm, phiinv_F, z, sweep, event,
                    chain_base, chain_mask, b, info, 1);
}

// ------------------------------------------------------------------ white noise (a10)
int gs_white_resid(gs_ctx* ctx, int n_psr, int n_chain, int64_t n_toa_max, int ldb,
                   const gs_tnt_desc* tdesc, const double* Tt, const double* r, const double* b,
                   int64_t ldy, double* y) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_psr < 0 || n_chain < 0) return fail_arg(2, "negative batch");
  if (n_toa_max < 0) return fail_arg(4, "n_toa_max < 0");
  if (ldb <= 0) return fail_arg(5, "ldb <= 0");
  if (!tdesc) return fail_arg(6, "tdesc is NULL");
  if (!Tt || !r || !b || !y) return fail_arg(7, "NULL array");
  if (ldy <= 0) return fail_arg(10, "ldy <= 0");
  if (n_psr == 0 || n_chain == 0 || n_toa_max == 0) return 0;
  const int64_t nmax = n_toa_max;
  WhiteResidArgs a;
  a.n_psr = n_psr; a.n_chain = n_chain; a.ldb = ldb; a.ldy = ldy; a.n_toa_max = nmax;
  a.tdesc = tdesc; a.Tt = Tt; a.r = r; a.b = b; a.y = y;
  launch_white_resid(ctx->stream, a);
  return after_launch("k_white_resid");
}

int gs_rho_analytic(gs_ctx* ctx, int n_psr, int n_chain, int NF, int ldb, const int32_t* fidx,
                    const double* b, const double* u, int64_t sweep, int64_t chain_base,
                    double rhomin, double rhomax, double* x, int ldx) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_psr < 0 || n_chain < 0) return fail_arg(2, "negative batch");
  if (NF <= 0 || (NF & 1)) return fail_arg(4, "NF must be even");
  if (!fidx || !b || !x) return fail_arg(6, "NULL array");
  if (!(rhomin > 0.0) || !(rhomax > rhomin)) return fail_arg(11, "need 0 < rhomin < rhomax");
  if (ldx < NF / 2) return fail_arg(14, "ldx too small");
  RhoArgs a;
  a.n_psr = n_psr; a.n_chain = n_chain; a.NF = NF; a.ldb = ldb; a.ldx = ldx; a.sweep = sweep;
  a.sweep_dev = ctx->sweep_dev;
  a.chain_base = chain_base; a.rhomin = rhomin; a.rhomax = rhomax; a.fidx = fidx; a.b = b;
  a.u = u; a.x = x; a.key = key_of(ctx); a.psr_base = ctx->psr_base;
  launch_rho_analytic(ctx->stream, a);
  return after_launch("k_rho_analytic");
}

int gs_sweep_freespec(gs_ctx* ctx, int n_psr, int n_chain, int NF, int NMX, int ldb,
                      const double* model, const int32_t* fidx, const int32_t* midx,
                      const int32_t* nm, double rhomin, double rhomax, int64_t chain_base,
                      double* x_state, double* b_state, int64_t it0, int n_sweeps, double* x_rec,
                      double* b_rec, const double* z0_inj, const double* z_inj,
                      const double* u_inj, int32_t* info) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_psr < 0 || n_chain < 0) return fail_arg(2, "negative batch");
  if (!nf_supported(NF)) return fail_arg(4, "NF must be even and <= 64");
  if (NMX < 0 || NMX > 64) return fail_arg(5, "NMX must be in 0..64");
  if (ldb < NF + 1) return fail_arg(6, "ldb too small");
  if (!model || !fidx || !midx || !nm) return fail_arg(7, "NULL model array");
  if (!(rhomin > 0.0) || !(rhomax > rhomin)) return fail_arg(11, "need 0 < rhomin < rhomax");
  if (!x_state || !b_state) return fail_arg(14, "NULL state");
  if (it0 < 0) return fail_arg(16, "it0 < 0");
  if (n_sweeps < 0) return fail_arg(17, "n_sweeps < 0");
  if (n_psr == 0 || n_chain == 0 || n_sweeps == 0) return 0;
  SweepArgs a;
  a.n_psr = n_psr; a.n_chain = n_chain; a.NF = NF; a.NMX = NMX; a.ldb = ldb; a.n_sweeps = n_sweeps;
  a.mstride = model_stride_doubles(NF, NMX); a.it0 = it0; a.chain_base = chain_base;
  a.rhomin = rhomin; a.rhomax = rhomax; a.model = model; a.fidx = fidx; a.midx = midx; a.nm = nm;
  a.x_state = x_state; a.b_state = b_state; a.x_rec = x_rec; a.b_rec = b_rec;
  a.z0_inj = z0_inj; a.z_inj = z_inj; a.u_inj = u_inj; a.info = info; a.key = key_of(ctx);
  a.fail_count = ctx->fail_counts;
  a.bcast = ctx->bcast; a.psr_base = ctx->psr_base;
  a.brec_nc = ctx->brec_nc < n_chain ? ctx->brec_nc : 0;
  a.sched = ctx->sweep_sched;
  a.dbg_handoff = ctx->dbg_handoff;
  return launch_rc(launch_sweep_freespec(ctx->stream, a, &ctx->last_shape), "k_sweep_freespec");
}

int gs_tau(gs_ctx* ctx, int n_psr, int n_chain, int NF, int ldb, const int32_t* fidx, const double* b,
           int half, double* tau) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_psr < 0 || n_chain < 0) return fail_arg(2, "negative batch");
  if (NF <= 0 || (NF & 1)) return fail_arg(4, "NF must be even");
  if (!fidx || !b || !tau) return fail_arg(6, "NULL array");
  TauArgs a;
  a.n_psr = n_psr; a.n_chain = n_chain; a.NF = NF; a.ldb = ldb; a.half = half; a.fidx = fidx; a.b = b;
  a.tau = tau;
  launch_tau(ctx->stream, a);
  return after_launch("k_tau");
}

static int grid_common(gs_ctx* ctx, GridArgs& a, int n_psr, int n_chain, int n_f, const double* tau,
                       const double* irn, int ngrid, const double* grid3, const double* u, int64_t sweep,
                       int64_t chain_base, double* x, int ldx, const int32_t* xcol, int32_t* idx_out) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_psr < 0 || n_chain < 0 || n_f < 0) return fail_arg(2, "negative batch");
  if (!tau) return fail_arg(5, "tau is NULL");
  if (ngrid <= 0) return fail_arg(7, "ngrid <= 0");
  if (!grid3) return fail_arg(8, "grid3 is NULL");
  if (!x || !xcol) return fail_arg(12, "x/xcol is NULL");
  a.n_psr = n_psr; a.n_chain = n_chain; a.n_f = n_f; a.ngrid = ngrid; a.ldx = ldx; a.sweep = sweep;
  a.sweep_dev = ctx->sweep_dev;
  a.chain_base = chain_base; a.tau = tau; a.irn = irn; a.grid3 = grid3; a.u = u; a.xcol = xcol; a.x = x;
  a.idx_out = idx_out; a.key = key_of(ctx); a.psr_base = ctx->psr_base;
  a.exact = ctx->grid_exact;
  a.n_fallback = ctx->grid_fallback;
  return 0;
}

int gs_rho_curn(gs_ctx* ctx, int n_psr, int n_chain, int n_f, const double* tau, const double* irn,
                int ngrid, const double* grid3, const double* u, int64_t sweep, int64_t chain_base,
                double* x, int ldx, const int32_t* xcol, int32_t* idx_out) {
  GridArgs a;
  int rc = grid_common(ctx, a, n_psr, n_chain, n_f, tau, irn, ngrid, grid3, u, sweep, chain_base, x, ldx,
                       xcol, idx_out);
  if (rc) return rc;
  launch_rho_curn(ctx->stream, a);
  return after_launch("k_rho_curn");
}

int gs_lnlike_marg(gs_ctx* ctx, int n_psr, int n_chain, int NF, int NMX, const double* model,
                   int model_per_sys, const int32_t* nm, const double* phiinv_F, double* lnl, int32_t* info) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_psr < 0 || n_chain < 0) return fail_arg(2, "negative batch");
  if (!nf_supported(NF)) return fail_arg(4, "NF must be even and <= 64");
  if (NMX < 0 || NMX > GS_NMX_WIDE) return fail_arg(5, "NMX must be in 0..128");
  if (!model || !nm || !phiinv_F || !lnl) return fail_arg(6, "NULL array");
  if (n_psr == 0 || n_chain == 0) return 0;
  LnlArgs a;
  a.n_psr = n_psr; a.n_chain = n_chain; a.NF = NF; a.NMX = NMX; a.model_per_sys = model_per_sys ? 1 : 0;
  a.model_global = NMX > 64;
  a.mstride = model_stride_doubles(NF, NMX); a.model = model; a.nm = nm; a.phiinv_F = phiinv_F;
  a.lnl = lnl; a.info = info; a.skip = nullptr;
  return launch_rc(launch_lnlike_marg(ctx->stream, a), "k_lnlike_marg");
}

int gs_lnlike_marg_gated(gs_ctx* ctx, int n_psr, int n_chain, int NF, int NMX, const double* model, const int32_t* nm,
                         const double* phiinv_F, const int32_t* gate, double* lnl, int32_t* info) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_psr < 0 || n_chain < 0) return fail_arg(2, "negative batch");
  if (!nf_supported(NF)) return fail_arg(4, "NF must be even and <= 64");
  if (NMX < 0 || NMX > GS_NMX_WIDE) return fail_arg(5, "NMX must be in 0..128");
  if (!model || !nm || !phiinv_F || !gate || !lnl) return fail_arg(6, "NULL array");
  if (n_psr == 0 || n_chain == 0) return 0;
  LnlArgs a;
  a.n_psr = n_psr; a.n_chain = n_chain; a.NF = NF; a.NMX = NMX; a.model_per_sys = 0;
  a.model_global = NMX > 64;
  a.mstride = model_stride_doubles(NF, NMX); a.model = model; a.nm = nm; a.phiinv_F = phiinv_F;
  a.lnl = lnl; a.info = info; a.skip = gate;
  return launch_rc(launch_lnlike_marg(ctx->stream, a), "k_lnlike_marg");
}

int gs_tau_sum(gs_ctx* ctx, int n_psr, int n_chain, int n_f, const double* tau, double* S) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_psr < 0 || n_chain < 0 || n_f < 0) return fail_arg(2, "negative batch");
  if (!tau || !S) return fail_arg(5, "NULL tau / S");
  launch_tau_sum(ctx->stream, n_psr, (int64_t)n_f * n_chain, tau, S);
  return after_launch("k_tau_sum");
}

int gs_tau_sum_fx(gs_ctx* ctx, int n_psr, int n_chain, int n_f, const double* tau, int e0, int64_t* acc,
                  int32_t* ovf) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_psr < 0 || n_chain < 0 || n_f < 0) return fail_arg(2, "negative batch");
  if (n_psr >= (1 << 15)) return fail_arg(2, "n_psr >= 32768 (int64 digit headroom)");
  if (!tau || !acc) return fail_arg(5, "NULL tau / acc");
  if (e0 < -1000 || e0 > 800) return fail_arg(6, "e0 out of range");
  launch_tau_sum_fx(ctx->stream, n_psr, (int64_t)n_f * n_chain, tau, e0, (long long*)acc, ovf);
  return after_launch("k_tau_sum_fx");
}

int gs_tau_sum_fx_b(gs_ctx* ctx, int n_psr, int n_chain, int NF, int ldb, const int32_t* fidx, const double* b,
                    int e0, int64_t* acc, int32_t* ovf) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_psr < 0 || n_chain < 0) return fail_arg(2, "negative batch");
  if (n_psr >= (1 << 15)) return fail_arg(2, "n_psr >= 32768 (int64 digit headroom)");
  if (NF <= 0 || NF > 64 || (NF & 1)) return fail_arg(4, "NF must be even and <= 64");
  if (ldb < NF) return fail_arg(5, "ldb < NF");
  if (!fidx || !b || !acc) return fail_arg(6, "NULL array");
  if (e0 < -1000 || e0 > 800) return fail_arg(8, "e0 out of range");
  TauArgs a;
  a.n_psr = n_psr; a.n_chain = n_chain; a.NF = NF; a.ldb = ldb; a.half = 0; a.fidx = fidx; a.b = b;
  a.tau = nullptr;
  launch_tau_sum_fx_b(ctx->stream, a, e0, (long long*)acc, ovf);
  return after_launch("k_tau_sum_fx_b");
}

int gs_fx_to_double(gs_ctx* ctx, int64_t n, int e0, const int64_t* acc, double* S) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n < 0) return fail_arg(2, "n < 0");
  if (e0 < -1000 || e0 > 800) return fail_arg(3, "e0 out of range");
  if (!acc || !S) return fail_arg(4, "NULL acc / S");
  launch_fx_to_double(ctx->stream, n, e0, (const long long*)acc, S);
  return after_launch("k_fx_to_double");
}

int gs_rho_curn_sum(gs_ctx* ctx, int n_psr, int n_chain, int n_f, const double* S, int ngrid,
                    const double* grid3, const double* u, int64_t sweep, int64_t chain_base, double* x,
                    int ldx, const int32_t* xcol, int32_t* idx_out) {
  if (ngrid > 64 * 32) return fail_arg(6, "ngrid > 2048");
  GridArgs a;
  int rc = grid_common(ctx, a, n_psr, n_chain, n_f, S, nullptr, ngrid, grid3, u, sweep, chain_base, x, ldx,
                       xcol, idx_out);
  if (rc) return rc;
  launch_rho_curn_sum(ctx->stream, a);
  return after_launch("k_rho_curn_sum");
}

int gs_rho_red(gs_ctx* ctx, int n_psr, int n_chain, int n_f, const double* tau, const double* gw,
               int ngrid, const double* grid3, const double* u, int64_t sweep, int64_t chain_base,
               double* x, int ldx, const int32_t* xcol, int32_t* idx_out) {
  if (!gw) return fail_arg(6, "gw is NULL");
  GridArgs a;
  int rc = grid_common(ctx, a, n_psr, n_chain, n_f, tau, gw, ngrid, grid3, u, sweep, chain_base, x, ldx,
                       xcol, idx_out);
  if (rc) return rc;
  launch_rho_red(ctx->stream, a);
  return after_launch("k_rho_red");
}

int gs_rho_gumbel(gs_ctx* ctx, int n_chain, int n_f, const double* tau, const double* irn, int ngrid,
                  const double* grid3, const double* u, int64_t sweep, int64_t chain_base, double* x,
                  int ldx, const int32_t* xcol, int32_t* idx_out) {
  if (!irn) return fail_arg(5, "irn is NULL");
  GridArgs a;
  int rc = grid_common(ctx, a, 1, n_chain, n_f, tau, irn, ngrid, grid3, u, sweep, chain_base, x, ldx, xcol,
                       idx_out);
  if (rc) return rc;
  launch_rho_gumbel(ctx->stream, a);
  return after_launch("k_rho_gumbel");
}

int gs_phi_from_x(gs_ctx* ctx, int n_chain, int ncol, const double* x, int ldx, const int32_t* cols,
                  double* out) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_chain < 0 || ncol < 0) return fail_arg(2, "negative size");
  if (!x || !cols || !out) return fail_arg(4, "NULL array");
  launch_phi_from_x(ctx->stream, n_chain, ncol, x, ldx, cols, out);
  return after_launch("k_phi_from_x");
}

int gs_pta_record(gs_ctx* ctx, int n_chain, int n_param, const double* x, double* x_rec, double* xlast) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_chain < 0 || n_param <= 0) return fail_arg(2, "bad size");
  if (!x || !xlast) return fail_arg(4, "NULL array");
  launch_pta_record(ctx->stream, n_chain, n_param, x, x_rec, xlast);
  return after_launch("k_pta_record");
}

int gs_pta_gate_phiinv(gs_ctx* ctx, int n_psr, int n_chain, int n_f, int n_param, const double* x,
                       const double* xlast, const int32_t* gw_col, const int32_t* red_col,
                       double* phiinv_F, int32_t* gate) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_psr < 0 || n_chain < 0 || n_f <= 0 || n_param <= 0) return fail_arg(2, "bad size");
  if (!x || !gw_col || !phiinv_F || !gate) return fail_arg(6, "NULL array");
  PtaGateArgs a;
  a.n_psr = n_psr; a.n_chain = n_chain; a.n_f = n_f; a.n_param = n_param; a.x = x; a.xlast = xlast;
  a.gw_col = gw_col; a.red_col = red_col; a.irn = nullptr; a.irn_pp = nullptr; a.phiinv_F = phiinv_F;
  a.gate = gate;
  launch_pta_gate_phiinv(ctx->stream, a);
  return after_launch("k_pta_gate_phiinv");
}

int gs_pta_gate_phiinv_irn(gs_ctx* ctx, int n_psr, int n_chain, int n_f, int n_param, const double* x,
                           const double* xlast, const int32_t* gw_col, const double* irn, double* phiinv_F,
                           int32_t* gate) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_psr < 0 || n_chain < 0 || n_f <= 0 || n_param <= 0) return fail_arg(2, "bad size");
  if (!x || !gw_col || !irn || !phiinv_F || !gate) return fail_arg(6, "NULL array");
  PtaGateArgs a;
  a.n_psr = n_psr; a.n_chain = n_chain; a.n_f = n_f; a.n_param = n_param; a.x = x; a.xlast = xlast;
  a.gw_col = gw_col; a.red_col = nullptr; a.irn = nullptr; a.irn_pp = irn; a.phiinv_F = phiinv_F; a.gate = gate;
  launch_pta_gate_phiinv(ctx->stream, a);
  return after_launch("k_pta_gate_phiinv");
}

int gs_phi_powerlaw(gs_ctx* ctx, int n_psr, int n_chain, int n_f, const double* x, int ldx, const int32_t* pl_col,
                    const double* lnphi, double* out) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_psr < 0 || n_chain < 0 || n_f <= 0) return fail_arg(2, "bad size");
  if (!x) return fail_arg(5, "x is NULL");
  if (ldx <= 0) return fail_arg(6, "ldx must be > 0");
  if (!pl_col || !lnphi || !out) return fail_arg(7, "NULL array");
  launch_phi_powerlaw(ctx->stream, n_psr, n_chain, n_f, x, ldx, pl_col, lnphi, out);
  return after_launch("k_phi_powerlaw");
}

int gs_hyper_mh(gs_ctx* ctx, int n_psr, int n_chain, int NF, int NMX, const double* model, const int32_t* nm,
                double* x, int ldx, const int32_t* gw_col, int n_h, const int32_t* hcol, const int32_t* hpsr,
                const double* hlo, const double* hhi, int red_kind, const int32_t* red_col, const int32_t* pl_col,
                const double* lnphi, double* lnl_p, int nsteps, int64_t sweep, int64_t chain_base,
                const double* inj, double* q_rec, int32_t* n_acc) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_psr <= 0 || n_chain < 0) return fail_arg(2, "bad batch");
  if (!nf_supported(NF)) return fail_arg(4, "NF must be even and <= 64");
  if (NMX < 0 || NMX > GS_NMX_WIDE) return fail_arg(5, "NMX must be in 0..128");
  if (!model || !nm) return fail_arg(6, "model/nm is NULL");
  if (!x) return fail_arg(8, "x is NULL");
  if (ldx <= 0 || ldx > 8192) return fail_arg(9, "ldx must be in 1..8192");
  if (!gw_col) return fail_arg(10, "gw_col is NULL");
  if (n_h <= 0) return fail_arg(11, "n_h must be > 0");
  if (!hcol || !hpsr || !hlo || !hhi) return fail_arg(12, "hyper tables are NULL");
  if (red_kind == 0 && !red_col) return fail_arg(17, "red_kind 0 needs red_col");
  if (red_kind == 1 && (!pl_col || !lnphi)) return fail_arg(18, "red_kind 1 needs pl_col and lnphi");
  if (red_kind != 0 && red_kind != 1) return fail_arg(16, "red_kind must be 0 or 1");
  if (!lnl_p) return fail_arg(20, "lnl_p is NULL");
  if (nsteps < 0 || nsteps > (1 << 20)) return fail_arg(21, "nsteps out of range");
  if (n_chain == 0 || nsteps == 0) return 0;
  HyperMhArgs a;
  a.n_psr = n_psr; a.n_chain = n_chain; a.NF = NF; a.NMX = NMX; a.ldx = ldx; a.n_h = n_h; a.nsteps = nsteps;
  a.red_kind = red_kind; a.mstride = model_stride_doubles(NF, NMX); a.sweep = sweep; a.chain_base = chain_base;
  a.sweep_dev = ctx->sweep_dev; a.key = key_of(ctx); a.model = model; a.nm = nm; a.gw_col = gw_col;
  a.hcol = hcol; a.hpsr = hpsr; a.red_col = red_col; a.pl_col = pl_col; a.hlo = hlo; a.hhi = hhi;
  a.lnphi = lnphi; a.inj = inj; a.x = x; a.lnl_p = lnl_p; a.q_rec = q_rec; a.n_acc = n_acc;
  return launch_rc(launch_hyper_mh(ctx->stream, a), "k_hyper_mh");
}

int gs_gate_phiinv_irn(gs_ctx* ctx, int n_chain, int n_f, int n_param, const double* x, const double* xlast,
                       const int32_t* gw_col, const double* irn, double* phiinv_F, int32_t* gate) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_chain < 0 || n_f <= 0 || n_param <= 0) return fail_arg(2, "bad size");
  if (!x || !gw_col || !irn || !phiinv_F || !gate) return fail_arg(5, "NULL array");
  PtaGateArgs a;
  a.n_psr = 1; a.n_chain = n_chain; a.n_f = n_f; a.n_param = n_param; a.x = x; a.xlast = xlast;
  a.gw_col = gw_col; a.red_col = nullptr; a.irn = irn; a.irn_pp = nullptr; a.phiinv_F = phiinv_F; a.gate = gate;
  launch_pta_gate_phiinv(ctx->stream, a);
  return after_launch("k_pta_gate_phiinv");
}

int gs_red_mh(gs_ctx* ctx, int n_chain, int n_f, int nsteps, int anchor, double* x, int ldx,
              const int32_t* red_col, const int32_t* gw_col, const double* tau, const double* lnphi,
              const double* jump, const double* de, int nde, int64_t sweep, int64_t chain_base, double* irn,
              double* lnl, int32_t* n_acc) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_chain < 0) return fail_arg(2, "n_chain < 0");
  if (n_f <= 0 || n_f > 256) return fail_arg(3, "n_f must be in 1..256");
  if (nsteps < 0 || nsteps > (1 << 20)) return fail_arg(4, "nsteps out of range");
  if (anchor != 0 && anchor != 1) return fail_arg(5, "anchor must be 0 or 1");
  if (!x) return fail_arg(6, "x is NULL");
  if (!red_col || !gw_col) return fail_arg(8, "red_col/gw_col is NULL");
  if (!tau || !lnphi) return fail_arg(10, "tau/lnphi is NULL");
  if (nsteps > 0 && !jump) return fail_arg(12, "jump is NULL");
  if (nde < 0 || (nde > 0 && !de)) return fail_arg(14, "bad DE buffer");
  if (n_chain == 0) return 0;
  RedMhArgs a;
  a.n_chain = n_chain; a.n_f = n_f; a.ldx = ldx; a.nsteps = nsteps; a.anchor = anchor; a.nde = nde;
  a.sweep = sweep; a.chain_base = chain_base; a.sweep_dev = ctx->sweep_dev; a.key = key_of(ctx);
  a.red_col = red_col; a.gw_col = gw_col; a.tau = tau; a.lnphi = lnphi; a.jump = jump; a.de = de;
  a.x = x; a.irn = irn; a.lnl = lnl; a.n_acc = n_acc;
  launch_red_mh(ctx->stream, a);
  return after_launch("k_red_mh");
}

int gs_philox(gs_ctx* ctx, int64_t n, const uint32_t* ctr, uint32_t* out) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n < 0) return fail_arg(2, "n < 0");
  if (!ctr || !out) return fail_arg(3, "NULL array");
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_philox, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, n, ctr, out,
                     key_of(ctx));
  return after_launch("k_philox");
}


int gs_white_mh(gs_ctx* ctx, int n_psr, int n_chain, const gs_white_desc* wdesc, const int32_t* wcol,
                const int32_t* wkind, const int32_t* wbk, const double* wmin, const double* wmax,
                const double* sigma2, const double* y, int64_t ldy, double* x, int ldx, int n_steps,
                const int32_t* nsteps_chain, int64_t sweep, int64_t chain_base, const double* inj,
                double* q_rec, int32_t* n_acc) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_psr < 0 || n_chain < 0) return fail_arg(2, "negative batch");
  if (!wdesc) return fail_arg(4, "wdesc is NULL");
  if (!wcol || !wkind || !wbk || !wmin || !wmax) return fail_arg(5, "NULL parameter table");
  if (!sigma2 || !y) return fail_arg(10, "NULL sigma2 / y");
  if (ldy <= 0) return fail_arg(12, "ldy <= 0");
  if (!x || ldx <= 0) return fail_arg(13, "x / ldx");
  if (n_steps < 0) return fail_arg(15, "n_steps < 0");
  if (n_psr == 0 || n_chain == 0) return 0;
  WhiteMhArgs a;
  a.x_per_sys = ctx->x_per_sys;
  a.n_psr = n_psr; a.n_chain = n_chain; a.ldx = ldx; a.n_steps = n_steps; a.psr_base = ctx->psr_base;
  a.ldy = ldy; a.sweep = sweep; a.chain_base = chain_base;
  a.sweep_dev = ctx->sweep_dev;
  a.wdesc = wdesc; a.wcol = wcol; a.wkind = wkind; a.wbk = wbk; a.nsteps_chain = nsteps_chain;
  a.wmin = wmin; a.wmax = wmax; a.sigma2 = sigma2; a.y = y; a.inj = inj;
  a.x = x; a.q_rec = q_rec; a.n_acc = n_acc; a.key = key_of(ctx);
  launch_white_mh(ctx->stream, a);
  return after_launch("k_white_mh");
}

int gs_white_tnt(gs_ctx* ctx, int n_psr, int n_chain, int m_max, const gs_tnt_desc* tdesc,
                 const gs_white_desc* wdesc, const int32_t* wcol, const int32_t* wkind,
                 const int32_t* wbk, const double* T, const double* sigma2, const int32_t* bk,
                 const double* r, const double* x, int ldx, int64_t tnt_cstride, int64_t d_cstride,
                 double* TNT, double* d) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_psr < 0 || n_chain < 0) return fail_arg(2, "negative batch");
  if (m_max <= 0 || m_max > 4096) return fail_arg(4, "m_max out of range");
  if (!tdesc) return fail_arg(5, "tdesc is NULL");
  if (!wdesc) return fail_arg(6, "wdesc is NULL");
  if (!wcol || !wkind || !wbk) return fail_arg(7, "NULL parameter table");
  if (!T || !sigma2 || !bk || !r) return fail_arg(10, "NULL T / sigma2 / bk / r");
  if (!x || ldx <= 0) return fail_arg(14, "x / ldx");
  if (tnt_cstride < 0 || d_cstride < 0) return fail_arg(16, "negative chain stride");
  if (!TNT || !d) return fail_arg(18, "NULL TNT / d");
  if (n_psr == 0 || n_chain == 0) return 0;
  WhiteTntArgs a;
  a.x_per_sys = ctx->x_per_sys;
  a.n_psr = n_psr; a.n_chain = n_chain; a.m_max = m_max; a.ldx = ldx;
  a.tnt_cstride = tnt_cstride; a.d_cstride = d_cstride; a.tdesc = tdesc; a.wdesc = wdesc;
  a.wcol = wcol; a.wkind = wkind; a.wbk = wbk; a.bk = bk; a.T = T; a.sigma2 = sigma2; a.r = r; a.x = x;
  a.TNT = TNT; a.d = d;
  launch_white_tnt(ctx->stream, a);
  return after_launch("k_white_tnt");
}

// ------------------------------------------------------------------ basis ECORR
int gs_ecorr_schur(gs_ctx* ctx, int n_chain, int mR, int ne, int ldbx, const double* Bx, const double* Dg,
                   const int32_t* ebk, int n_bk, const int32_t* xcol, const double* x, int ldx,
                   const double* A, const double* dR, double* TNT, double* d, double* aux) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_chain < 0) return fail_arg(2, "n_chain < 0");
  if (mR <= 0) return fail_arg(3, "mR <= 0");
  if (ne < 0) return fail_arg(4, "ne < 0");
  if (ldbx % 16 || ldbx < mR + 1 || !ecorr_nb_supported(ldbx / 16) || ldbx > 16 * ((mR + 1 + 15) / 16))
    return fail_arg(5, "ldbx must be 16 ceil((mR + 1) / 16) <= 128");
  if (!Bx || !Dg || !ebk) return fail_arg(6, "NULL Bx / Dg / ebk");
  if (n_bk <= 0 || n_bk > GS_WHITE_MAX_BK) return fail_arg(9, "n_bk must be in 1..15");
  if (!xcol || !x || ldx <= 0) return fail_arg(10, "xcol / x / ldx");
  if (!A || !dR || !TNT || !d || !aux) return fail_arg(13, "NULL A / dR / TNT / d / aux");
  if (n_chain == 0) return 0;
  EcorrSchurArgs a;
  a.n_chain = n_chain; a.mR = mR; a.ne = ne; a.ldbx = ldbx; a.ldx = ldx; a.n_bk = n_bk;
  a.Bx = Bx; a.Dg = Dg; a.A = A; a.dR = dR; a.x = x; a.ebk = ebk; a.xcol = xcol;
  a.TNT = TNT; a.d = d; a.aux = aux;
  launch_ecorr_schur(ctx->stream, a);
  return after_launch("k_ecorr_schur");
}

int gs_ecorr_prefix(gs_ctx* ctx, int n_chain, int NF, int NMX, int nM, int ne, int ldbx, const double* Bx,
                    const double* Dg, const int32_t* ebk, int n_bk, const int32_t* xcol, const double* x,
                    int ldx, const double* Ap, const double* phiinv_F, double* model, double* aux,
                    double* lnl, int32_t* info, int64_t bx_cstride, int64_t dg_cstride, int64_t ap_cstride) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_chain < 0) return fail_arg(2, "n_chain < 0");
  if (NF != 20 && NF != 40 && NF != 60) return fail_arg(3, "NF must be 20, 40 or 60");
  if (nM <= 0 || nM > 16 || NMX < nM || NMX > 64) return fail_arg(5, "need 1 <= nM <= 16, nM <= NMX <= 64");
  if (ne < 0) return fail_arg(6, "ne < 0");
  if (ldbx != 16 * (1 + (NF + 1 + 15) / 16)) return fail_arg(7, "ldbx must be 16 (1 + ceil((NF + 1) / 16))");
  if (!Bx || !Dg || !ebk) return fail_arg(8, "NULL Bx / Dg / ebk");
  if (n_bk <= 0 || n_bk > GS_WHITE_MAX_BK) return fail_arg(11, "n_bk must be in 1..15");
  if (!xcol || !x || ldx <= 0) return fail_arg(12, "xcol / x / ldx");
  if (!Ap || !aux) return fail_arg(15, "NULL Ap / aux");
  if (lnl ? !phiinv_F : !model) return fail_arg(16, "likelihood mode needs phiinv_F, block mode needs model");
  if (n_chain == 0) return 0;
  EcorrPrefixArgs a = {};
  a.n_chain = n_chain; a.NF = NF; a.NMX = NMX; a.nM = nM; a.ne = ne; a.ldbx = ldbx; a.ldx = ldx; a.n_bk = n_bk;
  a.mstride = model_stride_doubles(NF, NMX);
  a.Bx = Bx; a.Dg = Dg; a.Ap = Ap; a.x = x; a.ebk = ebk; a.xcol = xcol; a.model = model; a.aux = aux; a.info = info;
  a.phiinv_F = phiinv_F; a.lnl = lnl;
  if (bx_cstride < 0 || dg_cstride < 0 || ap_cstride < 0) return fail_arg(20, "negative per-chain stride");
  if ((bx_cstride == 0) != (ap_cstride == 0) || (bx_cstride == 0) != (dg_cstride == 0))
    return fail_arg(20, "per-chain strides must be all zero or all nonzero");
  a.bx_cs = bx_cstride; a.dg_cs = dg_cstride; a.ap_cs = ap_cstride;
  if (launch_ecorr_prefix(ctx->stream, a)) return fail_arg(7, "unsupported ldbx");
  return after_launch("k_ecorr_prefix");
}

int gs_ecorr_lnl_state(gs_ctx* ctx, int n_chain, int NF, int NMX, int nM, int ne, int ldbx, const double* Bx,
                       const double* Dg, const int32_t* ebk, int n_bk, const int32_t* xcol, const int32_t* eoff,
                       const double* x, const double* x_old, const double* prop, int ldx, const double* Ap,
                       const double* phiinv_F, double* tbuf, int32_t* tidx, double* aux, double* lnl, int32_t* info,
                       int64_t bx_cstride, int64_t dg_cstride, int64_t ap_cstride) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_chain < 0) return fail_arg(2, "n_chain < 0");
  if (NF != 20 && NF != 40 && NF != 60) return fail_arg(3, "NF must be 20, 40 or 60");
  if (nM <= 0 || nM > 16 || NMX < nM || NMX > 64) return fail_arg(5, "need 1 <= nM <= 16, nM <= NMX <= 64");
  if (ne < 0) return fail_arg(6, "ne < 0");
  if (ldbx != 16 * (1 + (NF + 1 + 15) / 16)) return fail_arg(7, "ldbx must be 16 (1 + ceil((NF + 1) / 16))");
  if (!Bx || !Dg || !ebk) return fail_arg(8, "NULL Bx / Dg / ebk");
  if (n_bk <= 0 || n_bk > GS_WHITE_MAX_BK) return fail_arg(11, "n_bk must be in 1..15");
  if (!xcol || !x || ldx <= 0) return fail_arg(12, "xcol / x / ldx");
  if (x_old && (!prop || !eoff)) return fail_arg(14, "an incremental step needs prop and eoff");
  if (!x_old && !Ap) return fail_arg(17, "a full evaluation needs Ap");
  if (!phiinv_F || !aux || !lnl) return fail_arg(19, "NULL phiinv_F / aux / lnl");
  if (!tbuf || !tidx) return fail_arg(20, "NULL tbuf / tidx");
  if (bx_cstride < 0 || dg_cstride < 0 || ap_cstride < 0) return fail_arg(25, "negative per-chain stride");
  if ((bx_cstride == 0) != (dg_cstride == 0) || (!x_old && (bx_cstride == 0) != (ap_cstride == 0)))
    return fail_arg(25, "per-chain strides must be all zero or all nonzero");
  if (n_chain == 0) return 0;
  EcorrPrefixArgs a = {};
  a.n_chain = n_chain; a.NF = NF; a.NMX = NMX; a.nM = nM; a.ne = ne; a.ldbx = ldbx; a.ldx = ldx; a.n_bk = n_bk;
  a.mstride = model_stride_doubles(NF, NMX);
  a.Bx = Bx; a.Dg = Dg; a.Ap = Ap; a.x = x; a.ebk = ebk; a.xcol = xcol; a.model = nullptr; a.aux = aux;
  a.info = info; a.phiinv_F = phiinv_F; a.lnl = lnl;
  a.bx_cs = bx_cstride; a.dg_cs = dg_cstride; a.ap_cs = ap_cstride;
  a.xold = x_old; a.prop = prop; a.eoff = eoff; a.tbuf = tbuf; a.tidx = tidx;
  if (launch_ecorr_prefix(ctx->stream, a)) return fail_arg(7, "unsupported ldbx");
  return after_launch("k_ecorr_prefix");
}

int gs_ecorr_epoch_sums(gs_ctx* ctx, int n_chain, const gs_white_desc* wdesc, const int32_t* wcol,
                        const int32_t* wkind, const int32_t* wbk, const double* x, int ldx, const double* T, int m,
                        const double* sigma2, const int32_t* bk, const double* r, int ne, int kb, int dcol,
                        const int32_t* colmap, const int32_t* eptr, const int32_t* etoa, const double* eu,
                        double* Bx, double* Dg) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_chain < 0) return fail_arg(2, "n_chain < 0");
  if (!wdesc || !wcol || !wkind || !wbk) return fail_arg(3, "NULL white tables");
  if (!x || ldx <= 0) return fail_arg(7, "x / ldx");
  if (!T || m <= 0) return fail_arg(9, "T / m");
  if (!sigma2 || !bk || !r) return fail_arg(11, "NULL sigma2 / bk / r");
  if (ne < 0 || kb <= 0 || dcol < 0 || dcol >= kb) return fail_arg(14, "ne / kb / dcol");
  if (!colmap || !eptr || !etoa || !eu) return fail_arg(17, "NULL colmap / epoch lists");
  if (!Bx || !Dg) return fail_arg(21, "NULL Bx / Dg");
  if (n_chain == 0 || ne == 0) return 0;
  EcorrSumArgs a = {};
  a.w.n_psr = 1; a.w.n_chain = n_chain; a.w.m_max = m; a.w.ldx = ldx; a.w.x_per_sys = 0;
  a.w.wdesc = wdesc; a.w.wcol = wcol; a.w.wkind = wkind; a.w.wbk = wbk; a.w.bk = bk;
  a.w.T = T; a.w.sigma2 = sigma2; a.w.r = r; a.w.x = x;
  a.n_chain = n_chain; a.ne = ne; a.kb = kb; a.dcol = dcol;
  a.colmap = colmap; a.eptr = eptr; a.etoa = etoa; a.eu = eu; a.Bx = Bx; a.Dg = Dg;
  launch_ecorr_epoch_sums(ctx->stream, a);
  return after_launch("k_ecorr_epoch_sums");
}

int gs_ecorr_gather(gs_ctx* ctx, int n_chain, int m, int ne, int kb, const int32_t* ecid, const int32_t* colmap,
                    const double* phm, const double* TNT, int64_t tnt_cstride, const double* d,
                    int64_t d_cstride, double* Bx, double* Dg, double* Ap) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_chain < 0 || m <= 0 || ne < 0) return fail_arg(2, "n_chain / m / ne");
  if (kb <= 16 || kb % 16) return fail_arg(5, "kb must be a multiple of 16 above 16");
  if (!ecid || !colmap || !phm) return fail_arg(6, "NULL ecid / colmap / phm");
  if (!TNT || !d || tnt_cstride < (int64_t)m * m || d_cstride < m) return fail_arg(9, "TNT / d / strides");
  if (!Bx || !Dg || !Ap) return fail_arg(13, "NULL Bx / Dg / Ap");
  if (n_chain == 0) return 0;
  EcorrGatherArgs a;
  a.n_chain = n_chain; a.m = m; a.ne = ne; a.kb = kb; a.nM = 16; a.tnt_cstride = tnt_cstride;
  a.d_cstride = d_cstride; a.TNT = TNT; a.d = d; a.phm = phm; a.ecid = ecid; a.colmap = colmap;
  a.Bx = Bx; a.Dg = Dg; a.Ap = Ap;
  launch_ecorr_gather(ctx->stream, a);
  return after_launch("k_ecorr_gather");
}

int gs_ecorr_propose(gs_ctx* ctx, int n_chain, int n_e, const int32_t* ecol, const double* emin,
                     const double* emax, const double* x, int ldx, int n_param, double* xq, int step,
                     int64_t sweep, int64_t chain_base, const double* inj, double* prop) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_chain < 0) return fail_arg(2, "n_chain < 0");
  if (n_e <= 0) return fail_arg(3, "n_e <= 0");
  if (!ecol || !emin || !emax) return fail_arg(4, "NULL ecol / emin / emax");
  if (!x || ldx <= 0 || n_param <= 0 || n_param > ldx) return fail_arg(7, "x / ldx / n_param");
  if (!xq || !prop) return fail_arg(10, "NULL xq / prop");
  if (step < 0) return fail_arg(11, "step < 0");
  if (n_chain == 0) return 0;
  EcorrMhArgs a = {};
  a.n_chain = n_chain; a.n_e = n_e; a.ldx = ldx; a.n_param = n_param; a.step = step;
  a.sweep = sweep; a.chain_base = chain_base; a.sweep_dev = ctx->sweep_dev; a.key = key_of(ctx);
  a.ecol = ecol; a.emin = emin; a.emax = emax; a.inj = inj;
  a.x = const_cast<double*>(x); a.xq = xq; a.prop = prop;
  launch_ecorr_propose(ctx->stream, a);
  return after_launch("k_ecorr_propose");
}

int gs_ecorr_accept(gs_ctx* ctx, int n_chain, int n_e, const int32_t* ecol, int init, const double* lnl,
                    const int32_t* info, const int32_t* pinfo, const double* aux, const double* prop,
                    const double* xq, double* x, int ldx, double* lnl0, double* q_rec, int32_t* n_acc) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_chain < 0) return fail_arg(2, "n_chain < 0");
  if (n_e <= 0 || !ecol) return fail_arg(3, "n_e / ecol");
  if (!lnl || !aux) return fail_arg(6, "NULL lnl / aux");
  if (!init && (!prop || !xq || !x || ldx <= 0)) return fail_arg(10, "prop / xq / x / ldx");
  if (!lnl0) return fail_arg(14, "NULL lnl0");
  if (n_chain == 0) return 0;
  EcorrMhArgs a = {};
  a.next_step = -1;
  a.n_chain = n_chain; a.n_e = n_e; a.ldx = ldx; a.init = init ? 1 : 0;
  a.ecol = ecol; a.lnl = lnl; a.info = info; a.pinfo = pinfo; a.aux = aux;
  a.prop = const_cast<double*>(prop); a.xq = const_cast<double*>(xq); a.x = x; a.lnl0 = lnl0;
  a.q_rec = q_rec; a.n_acc = n_acc;
  launch_ecorr_accept(ctx->stream, a);
  return after_launch("k_ecorr_accept");
}

int gs_ecorr_accept_propose(gs_ctx* ctx, int n_chain, int n_e, const int32_t* ecol, int init, const double* lnl,
                            const int32_t* info, const int32_t* pinfo, const double* aux, double* prop,
                            double* xq, double* x, int ldx, double* lnl0, double* q_rec, int32_t* n_acc,
                            const double* emin, const double* emax, int n_param, int next_step, int64_t sweep,
                            int64_t chain_base, const double* inj) {
  return gs_ecorr_accept_propose2(ctx, n_chain, n_e, ecol, init, lnl, info, pinfo, aux, prop, xq, x, ldx, lnl0,
                                  q_rec, n_acc, emin, emax, n_param, next_step, sweep, chain_base, inj, nullptr);
}

int gs_ecorr_accept_propose2(gs_ctx* ctx, int n_chain, int n_e, const int32_t* ecol, int init, const double* lnl,
                             const int32_t* info, const int32_t* pinfo, const double* aux, double* prop,
                             double* xq, double* x, int ldx, double* lnl0, double* q_rec, int32_t* n_acc,
                             const double* emin, const double* emax, int n_param, int next_step, int64_t sweep,
                             int64_t chain_base, const double* inj, int32_t* tidx) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_chain < 0) return fail_arg(2, "n_chain < 0");
  if (n_e <= 0 || !ecol) return fail_arg(3, "n_e / ecol");
  if (!lnl || !aux) return fail_arg(6, "NULL lnl / aux");
  if (!prop || !xq || !x || ldx <= 0) return fail_arg(10, "prop / xq / x / ldx");
  if (!lnl0) return fail_arg(14, "NULL lnl0");
  if (next_step >= 0 && (!emin || !emax || n_param <= 0 || n_param > ldx))
    return fail_arg(17, "emin / emax / n_param");
  if (n_chain == 0) return 0;
  EcorrMhArgs a = {};
  a.n_chain = n_chain; a.n_e = n_e; a.ldx = ldx; a.init = init ? 1 : 0; a.next_step = next_step;
  a.ecol = ecol; a.lnl = lnl; a.info = info; a.pinfo = pinfo; a.aux = aux;
  a.prop = prop; a.xq = xq; a.x = x; a.lnl0 = lnl0; a.q_rec = q_rec; a.n_acc = n_acc;
  a.n_param = n_param; a.emin = emin; a.emax = emax; a.inj = inj;
  a.sweep = sweep; a.chain_base = chain_base; a.sweep_dev = ctx->sweep_dev; a.key = key_of(ctx);
  a.tidx = tidx;
  launch_ecorr_accept(ctx->stream, a);
  return after_launch("k_ecorr_accept");
}

int gs_ecorr_bdraw_e(gs_ctx* ctx, int n_chain, int mR, int ne, int ldbx, const double* Bx, const double* Dg,
                     const int32_t* ebk, const int32_t* xcol, const double* x, int ldx, const double* bR,
                     int ldbR, const int32_t* ecid, const int32_t* rcol, int m, const double* z,
                     int64_t sweep, int event, int64_t chain_base, const int32_t* chain_mask, double* b,
                     int ldb, int64_t bx_cstride, int64_t dg_cstride, int dcol, const int32_t* jmap) {
  if (!ctx) return fail_arg(1, "ctx is NULL");
  if (n_chain < 0 || mR <= 0 || ne < 0) return fail_arg(2, "n_chain / mR / ne");
  if (ldbx < mR + 1 || ldbx > 128) return fail_arg(5, "ldbx must be in [mR + 1, 128]");
  if (dcol < 0 || dcol >= ldbx || !jmap) return fail_arg(26, "dcol / jmap");
  if (bx_cstride < 0 || dg_cstride < 0) return fail_arg(24, "negative per-chain stride");
  if (!Bx || !Dg || !ebk || !xcol) return fail_arg(6, "NULL Bx / Dg / ebk / xcol");
  if (!x || ldx <= 0) return fail_arg(10, "x / ldx");
  if (!bR || ldbR < mR) return fail_arg(12, "bR / ldbR");
  if (!ecid || !rcol) return fail_arg(14, "NULL ecid / rcol");
  if (m != mR + ne) return fail_arg(16, "m != mR + ne");
  if (!b || ldb < m) return fail_arg(22, "b / ldb");
  if (n_chain == 0) return 0;
  EcorrBArgs a;
  a.n_chain = n_chain; a.mR = mR; a.ne = ne; a.ldbx = ldbx; a.ldx = ldx; a.ldbR = ldbR; a.m = m; a.ldb = ldb;
  a.event = event; a.sweep = sweep; a.chain_base = chain_base; a.sweep_dev = ctx->sweep_dev; a.key = key_of(ctx);
  a.Bx = Bx; a.Dg = Dg; a.x = x; a.bR = bR; a.z = z; a.ebk = ebk; a.xcol = xcol; a.ecid = ecid; a.rcol = rcol;
  a.chain_mask = chain_mask; a.b = b;
  a.bx_cs = bx_cstride; a.dg_cs = dg_cstride; a.dcol = dcol; a.jmap = jmap;
  launch_ecorr_bdraw_e(ctx->stream, a);
  return after_launch("k_ecorr_bdraw_e");
}

}  // extern "C"
