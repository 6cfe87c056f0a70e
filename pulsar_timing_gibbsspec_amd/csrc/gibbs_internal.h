// Internal launch-argument structs shared by the kernel TUs and the C-ABI TU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pulsar_gibbs.h"
#include "gibbs_common.h"

// Wavefronts (systems) per workgroup of the b-draw / sweep kernels: the
// workgroup shares one LDS copy of its pulsar's model block.
#ifndef GS_SWEEP_WPB
#define GS_SWEEP_WPB 4
#endif
// ... of the one-draw-per-launch b|rho kernel (k_bdraw: every PTA sweep stages each pulsar's
// model block once per workgroup)
#ifndef GS_BDRAW_WPB
#define GS_BDRAW_WPB 4
#endif

// fixed-prior (timing-model) columns per pulsar: up to 64 everywhere (lane per row), up to
// GS_NMX_WIDE in gs_prefix / gs_bdraw with NF <= 64 (k_prefix_wide: L_M in LDS, 128 KB)
#define GS_NMX_WIDE 128

// model block: S0 | dF | G | h | R | aux[2] (aux: sum log diag L_M, |L_M^-1 d_M|^2)
__host__ __device__ inline int64_t model_aux_offset(int NF, int NMX) {
  return (int64_t)NF * (NF + 1) + NF + (int64_t)NMX * (NF + 1) + NMX + (int64_t)NMX * NMX;
}
__host__ __device__ inline int64_t model_stride_doubles(int NF, int NMX) {
  const int64_t s = model_aux_offset(NF, NMX) + 2;
  return (s + 1) & ~int64_t(1);  // 16-byte multiple
}

// The fused sweep's LDS copy of a model block in the register-tile layout (gibbs_tile.h
// ModelTiled): S' (NT(NT+1)/2 tiles: the augmented, identity-padded Schur block), G' (nP x NT
// tiles), R' (nP(nP+1)/2 tiles), each tile 4 registers x 64 lanes, then h (NMX, even) -- or, for
// NMX > 16, S' followed by the row-major G | h | R (model_tiled_fix).
// NT = NF/16 + 1 tile rows, nP = ceil(NMX/16) fixed-block chunks.
__host__ __device__ inline int model_tiled_nt(int NF) { return NF / 16 + 1; }
__host__ __device__ inline int model_tiled_np(int NMX) { return (NMX + 15) / 16; }
__host__ __device__ inline int64_t model_tiled_g_offset(int NF) {
  const int NT = model_tiled_nt(NF);
  return (int64_t)NT * (NT + 1) / 2 * 256;
}
__host__ __device__ inline int64_t model_tiled_r_offset(int NF, int NMX) {
  return model_tiled_g_offset(NF) + (int64_t)model_tiled_np(NMX) * model_tiled_nt(NF) * 256;
}
__host__ __device__ inline int64_t model_tiled_h_offset(int NF, int NMX) {
  const int nP = model_tiled_np(NMX);
  return model_tiled_r_offset(NF, NMX) + (int64_t)nP * (nP + 1) / 2 * 256;
}
// With more than 16 timing-model columns the fixed block stays row-major (G | h | R exactly as in
// the model block, right after S'): two 16-row chunks of mostly-zero G'/R' tiles would take the
// block past the LDS budget of 3 workgroups per CU (nm = 17 in configs[2]/[3]: 43 KB tiled vs
// 30 KB S' + row-major G/h/R).
__host__ __device__ inline bool model_tiled_fix(int NMX) { return NMX <= 16; }
// The fixed-block layout of ONE pulsar's block in a batch with NMX columns at most: a pulsar with
// nM <= 16 takes the tiled fixed block of a 16-column model even when NMX > 16 (configs[2]/[3]: 43
// of the 45 pulsars have nM <= 16, two have 17), so only the pulsars that need it read G and R
// row-major.  The block size covers both layouts.
__host__ __device__ inline int model_tiled_layout(int NMX, int nM) { return NMX <= 16 ? NMX : (nM <= 16 ? 16 : NMX); }
__host__ __device__ inline int64_t model_tiled_doubles(int NF, int NMX) {
  const int nf = NMX <= 16 ? NMX : 16;
  const int64_t fix = model_tiled_h_offset(NF, nf) + ((nf + 1) & ~1);
  if (model_tiled_fix(NMX)) return fix;
  const int64_t n = model_tiled_g_offset(NF) + (int64_t)NMX * (NF + 1) + NMX + (int64_t)NMX * NMX;
  const int64_t rm = (n + 1) & ~int64_t(1);
  return rm > fix ? rm : fix;
}

// gs_prefix / gs_prefix_sys / gs_prefix_dd (gibbs_prefix.hip)
struct PrefixArgs {
  int n_psr, n_chain, NF, NMX;
  int64_t tnt_cstride, d_cstride, mstride;
  int64_t gstride;  // doubles per system of gscr
  const gs_prefix_desc* desc;
  const double *TNT, *TNT_lo, *d, *d_lo, *phfix;  // lo parts may be NULL (= 0)
  const int32_t *fidx, *midx;
  double* model;
  int32_t* info;
  double* gscr;  // global scratch (NULL: LDS)
};
int64_t prefix_scratch_doubles(int NF, int NMX);
bool prefix_scratch_in_lds(int NF, int NMX);
hipError_t launch_prefix_dd(hipStream_t s, const PrefixArgs& a);
hipError_t launch_tnt_dd(hipStream_t s, int n_psr, int m_max, const gs_tnt_desc* desc, const double* T,
                         const double* Nvec, const double* r, double* TNT, double* TNT_lo, double* d, double* d_lo);

struct LnlArgs {
  int n_psr, n_chain, NF, NMX, model_per_sys;
  int model_global;  // shared model block read from global memory (too large for LDS)
  int64_t mstride;
  const double* model;
  const int32_t* nm;
  const double* phiinv_F;
  double* lnl;
  int32_t* info;
  const int32_t* skip;  // chains c with skip[c] != 0 are left as they are (gs_lnlike_marg_gated), or NULL
};
int launch_lnlike_marg(hipStream_t s, const LnlArgs& a);

// PTA red-noise hyper-parameter Metropolis block (gs_hyper_mh, gibbs_bdraw.hip)
struct HyperMhArgs {
  int n_psr, n_chain, NF, NMX, ldx, n_h, nsteps, red_kind;
  int64_t mstride, sweep, chain_base;
  const int64_t* sweep_dev;
  gs_key key;
  const double* model;  // per-pulsar prefix model blocks (row-major), read from global / L2
  const int32_t *nm, *gw_col, *hcol, *hpsr, *red_col, *pl_col;
  const double *hlo, *hhi, *lnphi, *inj;
  double *x, *lnl_p, *q_rec;
  int32_t* n_acc;
};
int launch_hyper_mh(hipStream_t s, const HyperMhArgs& a);

struct BdrawArgs {
  int n_psr, n_chain, NF, NMX, ldb, event, bcast, psr_base;
  int model_per_sys;  // 1: model block per (pulsar, chain) system, read from global
  int mask_per_sys;   // chain_mask indexed by system (GS_OPT_X_PER_SYS)
  int phi_per_chain;  // phiinv_F holds one row per chain, shared by every pulsar (GS_OPT_PHI_PER_CHAIN)
  int64_t mstride, sweep, chain_base;
  const int64_t* sweep_dev;  // ctx sweep counter (graph replay) or NULL
  const double* model;
  const int32_t *fidx, *midx, *nm, *chain_mask;
  const double *phiinv_F, *z;
  double* b;
  int32_t* info;
  int32_t* fail_count;  // gs_ctx_set_fail_counts: failed draws per system (b kept), or NULL
  double* lnl;             // gs_ctx_set_bdraw_lnl: lnL of each drawn system (k_bdraw_tiled), or NULL
  const double* lnl_model;  // ... with the model constants from these row-major blocks
  int64_t lnl_mstride;
  int persist;  // k_bdraw_tiled: 0 = one workgroup per 16 chains of a pulsar, G = G persistent workgroups
  int sched = 0;  // gs_bdraw_tiled: GS_OPT_SWEEP_SCHED (0 cost model, 2 one chain per wave, 3 two)
  gs_key key;
};

struct SweepArgs {
  int n_psr, n_chain, NF, NMX, ldb, n_sweeps, bcast, psr_base;
  int brec_nc;  // GS_OPT_BREC_CHAINS: 0 = b_rec holds every system, K = chains c < K only
  int sched;    // GS_OPT_SWEEP_SCHED
  int dbg_handoff;  // GS_OPT_DEBUG_HANDOFF (test only)
  int64_t mstride, it0, chain_base;
  double rhomin, rhomax;
  const double* model;
  const int32_t *fidx, *midx, *nm;
  double *x_state, *b_state, *x_rec, *b_rec;
  const double *z0_inj, *z_inj, *u_inj;
  int32_t* info;
  int32_t* fail_count;  // gs_ctx_set_fail_counts: failed draws per system (b kept), or NULL
  gs_key key;
};

struct RhoArgs {
  int n_psr, n_chain, NF, ldb, ldx, psr_base;
  int64_t sweep, chain_base;
  const int64_t* sweep_dev;  // ctx sweep counter (graph replay) or NULL
  double rhomin, rhomax;
  const int32_t* fidx;
  const double *b, *u;
  double* x;
  gs_key key;
};

// *shape: the workgroup shape launched (GS_OPT_LAST_SWEEP_SHAPE: 1 hand-off, 2 one chain per wave, 3 two)
int launch_sweep_freespec(hipStream_t s, const SweepArgs& a, int* shape);
int launch_bdraw(hipStream_t s, const BdrawArgs& a);
// *shape: 2 one chain per wave (k_bdraw_tiled), 3 two chains per wave (k_bdraw_pair)
int launch_bdraw_tiled(hipStream_t s, const BdrawArgs& a, int* shape);
int launch_model_tile(hipStream_t s, const double* model, int n_psr, int NF, int NMX, const int32_t* nm,
                      double* tiled);
// large free-spectrum blocks (64 < NF <= 255), tiles in a context-owned workspace
bool big_nf_supported(int NF);
int64_t big_ws_doubles_per_sys(int NF);
int launch_bdraw_big(hipStream_t s, const BdrawArgs& a, double* ws);
int launch_rho_analytic(hipStream_t s, const RhoArgs& a);

struct TauArgs {
  int n_psr, n_chain, NF, ldb, half;
  const int32_t* fidx;
  const double* b;
  double* tau;
};

struct GridArgs {
  int n_psr, n_chain, n_f, ngrid, ldx, psr_base;
  int exact;  // GS_OPT_GRID_EXACT: 1 numpy's operation order (bit-exact pdfs); 0 certified f32 /
              // f64 two-level draw (red grid); 2 the f64 wave kernels
  int32_t* n_fallback;  // gs_ctx_set_grid_fallback_counter: rows redone in f64, or NULL
  int64_t sweep, chain_base;
  const int64_t* sweep_dev;  // ctx sweep counter (graph replay) or NULL
  const double *tau, *irn, *grid3, *u;
  const int32_t* xcol;
  double* x;
  int32_t* idx_out;
  gs_key key;
};

int launch_counter_add(hipStream_t s, int64_t* counter, int64_t inc);
int launch_tau_sum(hipStream_t s, int n_psr, int64_t nrow, const double* tau, double* S);
int launch_tau_sum_fx(hipStream_t s, int n_psr, int64_t nrow, const double* tau, int e0, long long* acc, int* ovf);
int launch_fx_to_double(hipStream_t s, int64_t nrow, int e0, const long long* acc, double* S);
int launch_tau_sum_fx_b(hipStream_t s, const TauArgs& a, int e0, long long* acc, int* ovf);
int launch_rho_curn_sum(hipStream_t s, const GridArgs& a);

struct PtaGateArgs {
  int n_psr, n_chain, n_f, n_param;
  const double *x, *xlast;
  const int32_t *gw_col, *red_col;
  const double* irn;  // [n_f x n_chain] power-law red phi added to every pulsar's phi, or NULL
  const double* irn_pp;  // [n_psr x n_f x n_chain] per-pulsar red phi (gs_pta_gate_phiinv_irn), or NULL
  double* phiinv_F;
  int32_t* gate;
};

int launch_tau(hipStream_t s, const TauArgs& a);
int launch_rho_curn(hipStream_t s, const GridArgs& a);
int launch_rho_red(hipStream_t s, const GridArgs& a);
int launch_rho_gumbel(hipStream_t s, const GridArgs& a);
int launch_phi_from_x(hipStream_t s, int n_chain, int ncol, const double* x, int ldx, const int32_t* cols,
                      double* out);
int launch_pta_record(hipStream_t s, int n_chain, int n_param, const double* x, double* x_rec, double* xlast);
int launch_pta_gate_phiinv(hipStream_t s, const PtaGateArgs& a);
int launch_phi_powerlaw(hipStream_t s, int n_psr, int n_chain, int n_f, const double* x, int ldx,
                        const int32_t* pl_col, const double* lnphi, double* out);

struct WhiteMhArgs {
  int n_psr, n_chain, ldx, n_steps, psr_base;
  int x_per_sys;  // GS_OPT_X_PER_SYS
  int64_t ldy, sweep, chain_base;
  const int64_t* sweep_dev;  // ctx sweep counter (graph replay) or NULL
  const gs_white_desc* wdesc;
  const int32_t *wcol, *wkind, *wbk, *nsteps_chain;
  const double *wmin, *wmax, *sigma2, *y, *inj;
  double *x, *q_rec;
  int32_t* n_acc;
  gs_key key;
};

struct WhiteResidArgs {
  int n_psr, n_chain, ldb;
  int64_t ldy, n_toa_max;
  const gs_tnt_desc* tdesc;
  const double *Tt, *r, *b;
  double* y;
};

struct WhiteTntArgs {
  int n_psr, n_chain, m_max, ldx;
  int x_per_sys;  // GS_OPT_X_PER_SYS
  int64_t tnt_cstride, d_cstride;
  const gs_tnt_desc* tdesc;
  const gs_white_desc* wdesc;
  const int32_t *wcol, *wkind, *wbk, *bk;
  const double *T, *sigma2, *r, *x;
  double *TNT, *d;
};

int launch_white_mh(hipStream_t s, const WhiteMhArgs& a);

// ECORR operands with white noise sampled: epoch segment sums (gibbs_white.hip)
struct EcorrSumArgs {
  WhiteTntArgs w;  // white tables, x, T (row-major n_toa x m), sigma2, bk, r of pulsar 0
  int n_chain, ne, kb, dcol;
  const int32_t *colmap, *eptr, *etoa;
  const double* eu;
  double *Bx, *Dg;
};
int launch_ecorr_epoch_sums(hipStream_t s, const EcorrSumArgs& a);

// power-law red-noise Metropolis block (gibbs_red.hip)
struct RedMhArgs {
  int n_chain, n_f, ldx, nsteps, anchor, nde;
  int64_t sweep, chain_base;
  const int64_t* sweep_dev;
  gs_key key;
  const int32_t *red_col, *gw_col;
  const double *tau, *lnphi, *jump, *de;
  double *x, *irn, *lnl;
  int32_t* n_acc;
};
int launch_red_mh(hipStream_t s, const RedMhArgs& a);
int launch_white_resid(hipStream_t s, const WhiteResidArgs& a);
int launch_white_tnt(hipStream_t s, const WhiteTntArgs& a);

// basis-ECORR block (gibbs_ecorr.hip)
struct EcorrSchurArgs {
  int n_chain, mR, ne, ldbx, ldx, n_bk;
  const double *Bx, *Dg, *A, *dR, *x;
  const int32_t *ebk, *xcol;
  double *TNT, *d, *aux;
};
struct EcorrMhArgs {
  int n_chain, n_e, ldx, n_param, step, init;
  int next_step;  // k_ecorr_accept: propose step next_step afterwards (< 0: no)
  int64_t sweep, chain_base;
  const int64_t* sweep_dev;
  gs_key key;
  const int32_t* ecol;
  const double *emin, *emax, *inj, *lnl, *aux;
  const int32_t *info, *pinfo;
  double *x, *xq, *prop, *lnl0, *q_rec;
  int32_t* n_acc;
  int32_t* tidx;  // incremental ECORR state: flipped on acceptance (NULL: none)
};
struct EcorrBArgs {
  int n_chain, mR, ne, ldbx, ldx, ldbR, m, ldb, event, dcol;
  int64_t sweep, chain_base, bx_cs, dg_cs;  // per-chain strides of Bx / Dg (0: shared)
  const int32_t* jmap;                      // Bx column -> index into bR (-1: skip)
  const int64_t* sweep_dev;
  gs_key key;
  const double *Bx, *Dg, *x, *bR, *z;
  const int32_t *ebk, *xcol, *ecid, *rcol, *chain_mask;
  double* b;
};
struct EcorrPrefixArgs {
  int n_chain, NF, NMX, nM, ne, ldbx, ldx, n_bk;
  int64_t mstride, bx_cs, dg_cs, ap_cs;  // per-chain strides of Bx / Dg / Ap (0: shared)
  const double *Bx, *Dg, *Ap, *x;
  const double* phiinv_F;  // likelihood mode (lnl != NULL): [n_chain x NF]
  const int32_t *ebk, *xcol;
  double *model, *aux, *lnl;
  int32_t* info;
  // stored state T = Ap - P (gs_ecorr_lnl_state): tbuf [2][n_chain][NT x 256], tidx [n_chain] the
  // current slot; xold != NULL: incremental step from the state at xold to x (prop: the proposal
  // records, eoff: per-backend epoch offsets)
  const double *xold, *prop;
  const int32_t* eoff;
  double* tbuf;
  int32_t* tidx;
};
int launch_ecorr_prefix(hipStream_t s, const EcorrPrefixArgs& a);
struct EcorrGatherArgs {
  int n_chain, m, ne, kb, nM;
  int64_t tnt_cstride, d_cstride;
  const double *TNT, *d, *phm;
  const int32_t *ecid, *colmap;
  double *Bx, *Dg, *Ap;
};
int launch_ecorr_gather(hipStream_t s, const EcorrGatherArgs& a);
bool ecorr_nb_supported(int nb);
int launch_ecorr_schur(hipStream_t s, const EcorrSchurArgs& a);
int launch_ecorr_propose(hipStream_t s, const EcorrMhArgs& a);
int launch_ecorr_accept(hipStream_t s, const EcorrMhArgs& a);
int launch_ecorr_bdraw_e(hipStream_t s, const EcorrBArgs& a);
