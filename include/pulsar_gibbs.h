/*
 * pulsar_gibbs.h — C-ABI of the MI355X free-spectrum Gibbs hot path.
 *
 * The reference (astrolamb/pulsar_timing_gibbsspec) is pure Python over
 * numpy/scipy; it has no native boundary.  These entry points replace the
 * L2 -> L3 arithmetic of its samplers and are bound by
 * ctypes from pulsar_timing_gibbsspec_amd/_lib.py.  Each entry cites the
 * reference code it replaces.
 *
 * Conventions
 *   - every array argument is caller-owned DEVICE memory (fp64 unless noted),
 *     row-major, with the leading dimensions given;
 *   - a "system" is one (pulsar p, chain c) pair, sys = p * n_chain + c;
 *   - calls are asynchronous on the context's stream; a context is not
 *     thread-safe (one host thread per context);
 *   - return 0 on success, a negative HIP error code (-hipError_t) on a
 *     runtime failure, or a positive 1-based index of the offending argument;
 *     gs_last_error() describes the last failure of the calling thread;
 *   - per-system `info` (int32, may be NULL): 0 = ok, k > 0 = the k-th leading
 *     minor of Sigma was not positive definite (maps to the reference's
 *     LinAlgError branch, pulsar_gibbs.py:511, and to the -inf likelihood at
 *     pulsar_gibbs.py:603-604).
 *
 * Random numbers: device Philox4x32-10, key = the context seed, counter =
 *   (slot, sweep, global chain id, (global pulsar << 8) | event).  Any draw can be
 *   replaced by injected values (parity mode) by passing a non-NULL array.
 */
#ifndef PULSAR_GIBBS_H
#define PULSAR_GIBBS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GS_ABI_VERSION 1

/* Philox event ids (counter word 3, low 8 bits) */
enum {
  GS_EV_B0 = 1,     /* first b draw of a run, from xs   (pulsar_gibbs.py:661-662) */
  GS_EV_RHO = 2,    /* rho|b uniforms                    (pulsar_gibbs.py:215)     */
  GS_EV_B = 3,      /* gated b draw                      (pulsar_gibbs.py:697-698) */
  GS_EV_RED = 4,    /* per-pulsar red grid-CDF uniforms  (pta_gibbs.py:271)        */
  GS_EV_CURN = 5,   /* common grid-CDF uniforms          (pta_gibbs.py:209)        */
  GS_EV_GUMBEL = 6, /* Gumbel-max uniforms               (pulsar_gibbs.py:233)     */
  GS_EV_WHITE = 7,  /* white-noise MH draws              (pulsar_gibbs.py:377-398) */
  GS_EV_REDMH = 8,  /* power-law red-noise MH draws      (pulsar_gibbs.py:312-319) */
  GS_EV_ECORR = 9,  /* basis-ECORR MH draws              (pulsar_gibbs.py:458-470) */
  GS_EV_ECORR_B = 10, /* epoch coefficients of a gated b draw (b_E | b_R)          */
  GS_EV_ECORR_B0 = 11, /* epoch coefficients of the first b draw                   */
  GS_EV_HYPER = 12, /* PTA red hyper-parameter MH draws  (pta_gibbs.py:319-340)     */
  GS_EV_USER = 16   /* first id free for callers                                    */
};

/* Context options (gs_ctx_set_option) */
enum {
  GS_OPT_BCAST = 1,   /* b-draw factorisation variant: 0 = lane-row, v_readlane -> SGPR;
                         1 = lane-row, LDS broadcast; 2 = lane-row, v_readlane in batches
                         of 8 SGPR pairs; 3 = 16x16 fp64 MFMA tiles (default) */
  GS_OPT_PSR_BASE = 2, /* global index of this context's pulsar 0 (Philox counters of a
                         pulsar-sharded run); default 0 */
  GS_OPT_X_PER_SYS = 3, /* 0 (default): x holds one row per chain (a PTA's parameter vector,
                         pta_gibbs.py); 1: one row per (pulsar, chain) system, row
                         p * n_chain + c (independent pulsars, each its own
                         PulsarBlockGibbs, config 5).  Read by gs_white_mh, gs_white_tnt;
                         with 1, gs_bdraw*'s chain_mask and gs_white_mh's nsteps_chain
                         are indexed by system too. */
  GS_OPT_GRID_EXACT = 4, /* grid conditionals: 1 = numpy's operation order (sequential product
                         of per-pulsar pdfs, sequential cumsum: bit-identical pdfs); 2 = the f64
                         wave kernels (log-space product, one rcp per four ratios, short exp:
                         pdfs equal to ~1e-15 relative); 0 (default) = as 2, except gs_rho_red
                         and gs_rho_curn_sum (ngrid <= 1024): every point in f32 with a per-row
                         error certificate, rows whose index the certificate cannot prove redone
                         with 2's f64 arithmetic (indices of exact arithmetic, as 2's), 16 lanes
                         per row; 3 = as 0 with the round-3 certified red kernel (64 lanes per
                         row, one compare per point) and 2's CURN-from-sums kernel */
  GS_OPT_BREC_CHAINS = 5, /* gs_sweep_freespec b_rec: 0 (default) = every system, row
                         sweep * n_psr * n_chain + p * n_chain + c; K > 0 = chains c < K of
                         each pulsar only, compact rows (sweep * n_psr + p) * K + c (the
                         reference's bchain is chain 0: K = 1 puts n_psr rows per sweep on
                         the host instead of staging every chain's b in HBM) */
  GS_OPT_PHI_PER_CHAIN = 6, /* 1: gs_bdraw*'s phiinv_F holds ONE row per chain (n_chain x NF),
                         shared by every pulsar -- the CURN sweep without per-pulsar red noise,
                         whose phiinv is the common spectrum alone (pta_gibbs.py:512-548); 0
                         (default): one row per (pulsar, chain) system */
  GS_OPT_SWEEP_SCHED = 7, /* gs_sweep_freespec's workgroup shape (tile variant; same draws): 0
                         (default) = chosen by a cost model of the launch; 1 = 12-wave workgroups
                         of 16 chains, each trio of waves running a 13th..16th chain in thirds of
                         the sweeps (every wave draws 4/3 chains: n_psr x n_chain = 4096 fills the
                         3072 wave slots of 3 waves/SIMD in one round); 2 = 4-wave workgroups,
                         one chain per wave; 3 = two chains per wave (NF = 60 tile variant with
                         device Philox, even chain counts; else as 0), both chains' draws sharing
                         the diagonal-tile eliminations at 2 waves/SIMD.  gs_bdraw_tiled
                         follows it too (3: two chains per wave where NF = 60, no lnL output is
                         attached and the chain count is even; otherwise one chain per wave).
                         The 12-wave shape is used only when its LDS (model
                         block + 12 waves' scratch, save, park and hand-off slots) fits the
                         device's per-workgroup limit; otherwise the 4-wave shape runs.  A
                         hand-off that does not arrive within the bounded wait (or arrives from a
                         chain already marked failed) is never read: the chain's remaining sweeps
                         are skipped, nothing stale is recorded, and its info is set to -1. */
  GS_OPT_DEBUG_HANDOFF = 8, /* test only: 1 = workgroup 0's first trio never publishes its first
                         hand-off (and the wait is shortened), so the 13th chain of workgroup 0
                         must end with info = -1 */
  GS_OPT_LAST_SWEEP_SHAPE = 9 /* read only (gs_ctx_get_option): the workgroup shape the context's
                         last gs_sweep_freespec or gs_bdraw_tiled launch ran -- 1 = 12-wave
                         hand-off, 2 = one chain per wave, 3 = two chains per wave, 0 = none yet */
};

typedef struct gs_ctx gs_ctx;

/* Ragged-batch descriptor for gs_tnt (one per pulsar, int64 fields, device). */
typedef struct {
  int64_t n_toa;   /* TOAs of this pulsar                                   */
  int64_t m;       /* basis columns                                          */
  int64_t T_off;   /* element offset of T (n_toa x m, row-major) in T       */
  int64_t toa_off; /* element offset into Nvec / r                          */
  int64_t tnt_off; /* element offset of TNT (m x m) in TNT                  */
  int64_t d_off;   /* element offset of d (m) in d                          */
} gs_tnt_desc;

/* Per-pulsar descriptor for gs_prefix (device). */
typedef struct {
  int64_t m;       /* basis columns                                         */
  int64_t n_fixed; /* fixed-prior columns nM (m - NF), 0 < nM <= NMX        */
  int64_t tnt_off; /* element offset of TNT (m x m) in TNT                  */
  int64_t d_off;   /* element offset of d (m) in d                          */
} gs_prefix_desc;

int gs_version(void);
/* Build stamp: "sources <hash of every .hip/.h source>; hipcc <HIP version>; built <UTC time> on
 * <host>" (not an ABI entry the reference has; a provenance check for the shipped library). */
const char* gs_build_info(void);
const char* gs_last_error(void);

int gs_ctx_create(int device, uint64_t seed, void* hip_stream, gs_ctx** out);
int gs_ctx_destroy(gs_ctx* ctx);
int gs_ctx_set_stream(gs_ctx* ctx, void* hip_stream);
int gs_ctx_set_seed(gs_ctx* ctx, uint64_t seed);
int gs_ctx_set_option(gs_ctx* ctx, int option, int value);
int gs_ctx_get_option(gs_ctx* ctx, int option); /* -1 on unknown option / NULL ctx */

/*
 * Graph replay of sweeps (a8): Philox counters use sweep + *sweep_dev when a device-side
 * sweep counter is attached (NULL detaches), so a captured sequence of launches draws
 * fresh numbers on every replay; gs_counter_add(counter, inc) advances it on the stream
 * (captured with the sweep).  Attach before capturing.
 */
int gs_ctx_set_sweep_counter(gs_ctx* ctx, const int64_t* sweep_dev);
/*
 * Non-positive-definite Sigma inside a run (the reference's LinAlgError branch,
 * pulsar_gibbs.py:507-516): every b-draw kernel (gs_bdraw*, gs_sweep_freespec) keeps the
 * system's previous b when its factorisation fails -- no NaN enters the chain state -- and
 * reports the first failing pivot in info.  With a per-system counter array attached
 * (int32 [n_sys], device, NULL detaches), each failed draw also adds 1 to counts[sys], so a
 * caller can surface failures as they happen.  The counts persist across calls.
 */
int gs_ctx_set_fail_counts(gs_ctx* ctx, int32_t* counts);
int gs_counter_add(gs_ctx* ctx, int64_t* counter, int64_t inc);
/* int32 device counter (NULL detaches) incremented by the grid rows the certified f32 draw had to
   redo in f64 (GS_OPT_GRID_EXACT = 0). */
int gs_ctx_set_grid_fallback_counter(gs_ctx* ctx, int32_t* counter);
/* Likelihood by-product of the b draw (NULL, NULL detaches): while attached, gs_bdraw_tiled also
   writes lnl[p * n_chain + c] for every system -- gs_lnlike_marg's value at the same phiinv_F, bit
   for bit (the same factorisation; the model constants aux[2] from the row-major gs_prefix blocks
   `model`, one per pulsar); a system whose chain_mask entry is 0 keeps its b and still gets its
   lnl (the likelihood-mode factorisation on the already staged block).  The PTA red-noise
   Metropolis block starts from these (pta_gibbs.py:689-704: the gated draw at the end of a sweep factorises exactly the systems the
   next sweep's block starts from), instead of re-factorising every (pulsar, chain).  gs_bdraw /
   gs_bdraw_sys refuse to run while it is attached. */
int gs_ctx_set_bdraw_lnl(gs_ctx* ctx, double* lnl, const double* model);

/* Doubles per pulsar in a model buffer (see gs_prefix). */
int64_t gs_model_stride(int NF, int NMX);
/* Dynamic LDS bytes per workgroup of the fused sweep (tile variant, 4-wave workgroups) for
 * (NF, NMX); the 12-wave hand-off workgroups of GS_OPT_SWEEP_SCHED take more. */
int gs_sweep_lds_bytes(int NF, int NMX);

/*
 * (a2) TNT = T^T N^-1 T, d = T^T N^-1 r for a ragged batch of pulsars.
 * Replaces pulsar_gibbs.py:500-502 (also :584-586) and pta_gibbs.py:523-526.
 * fp64 MFMA (v_mfma_f64_16x16x4f64), split over TOAs.
 */
int gs_tnt(gs_ctx* ctx, int n_psr, int m_max, const gs_tnt_desc* desc,
           const double* T, const double* Nvec, const double* r, double* TNT, double* d);
/*
 * Same in double-double: TNT + TNT_lo and d + d_lo equal T^T N^-1 T and T^T N^-1 r of the
 * fp64 inputs to ~1e-30 relative (exact products, compensated sums; TNT exactly symmetric).
 * TNT_lo / d_lo may be NULL.  Feed the pairs to gs_prefix_dd: the fp64 rounding of TNT is,
 * relative to the Schur block the draw factorises, a perturbation of up to ~1e-9 at 10^4
 * TOAs.  VALU work; once per noise state.
 */
int gs_tnt_dd(gs_ctx* ctx, int n_psr, int m_max, const gs_tnt_desc* desc, const double* T,
              const double* Nvec, const double* r, double* TNT, double* TNT_lo, double* d, double* d_lo);

/*
 * Fixed-prior prefix of the Cholesky of Sigma = TNT + diag(phiinv), with the
 * fixed-prior columns (timing model; phiinv constant across sweeps) ordered
 * first and the NF free-spectrum columns (gwid, pulsar_gibbs.py:90-105) last.
 * Writes, per pulsar p, at model + p * gs_model_stride(NF, NMX):
 *   S0 [NF x (NF+1)]  Schur complement TNT_FF - W^T W  (row stride NF+1)
 *   dF [NF]           d_F - W^T L_M^-1 d_M
 *   G  [NMX x (NF+1)] L_M^-T W  (row stride NF+1)
 *   h  [NMX]          L_M^-T L_M^-1 d_M
 *   R  [NMX x NMX]    L_M^-T  (upper)
 *   aux[2]            sum log diag L_M, |L_M^-1 d_M|^2  (gs_lnlike_marg)
 * fidx: [n_psr x NF] column index of each free-spectrum column (gwid);
 * midx: [n_psr x NMX] column index of each fixed-prior column;
 * phiinv_fixed: [n_psr x NMX] their (constant) phiinv (1e-40 for the TM).
 * L_M, W = L_M^-1 A_MF, e, S0 and dF are computed in double-double (the fp64 Schur
 * complement cancels 2-3 digits) and rounded; G, h, R in fp64.
 */
int gs_prefix(gs_ctx* ctx, int n_psr, int NF, int NMX, const gs_prefix_desc* desc,
              const double* TNT, const double* d, const int32_t* fidx, const int32_t* midx,
              const double* phiinv_fixed, double* model, int32_t* info);

/*
 * (a1, a5) Batched b|rho draw: Sigma = TNT + diag(phiinv) -> Cholesky ->
 * b = Sigma^-1 d + L^-T z for n_psr x n_chain systems, one wavefront each.
 * NF = 20, 40, 60: register tiles; even NF in 66..254 (config 5: 200): tiles in a
 * workspace the context allocates on first use (NF/16+1)(NF/16+2)/2 * 2 KB per
 * system; Philox slot j then gives the packed normals 2j, 2j+1 of [z_F | z_M].
 * Replaces PulsarBlockGibbs.update_b (pulsar_gibbs.py:489-520) and
 * PTABlockGibbs.update_b (pta_gibbs.py:512-548).
 * phiinv_F: [n_sys x NF] phiinv of the free-spectrum columns (fidx order);
 * nm: [n_psr] fixed-prior column count; z: [n_sys x ldb] injected normals
 * indexed by ORIGINAL column (NULL: Philox, event `event`, sweep `sweep`);
 * chain_mask: [n_chain] ([n_sys] under GS_OPT_X_PER_SYS) or NULL; masked systems keep b (the
 * b-update gate, pta_gibbs.py:703).  b: [n_sys x ldb] output in original column order.
 */
int gs_bdraw(gs_ctx* ctx, int n_psr, int n_chain, int NF, int NMX, int ldb,
             const double* model, const int32_t* fidx, const int32_t* midx, const int32_t* nm,
             const double* phiinv_F, const double* z, int64_t sweep, int event,
             int64_t chain_base, const int32_t* chain_mask, double* b, int32_t* info);

/*
 * Register-tile copies of n_psr shared model blocks (NF <= 64, NMX <= 64) for gs_bdraw_tiled:
 * per pulsar p, at tiled + p * gs_model_tiled_stride(NF, NMX), the augmented Schur block, -G and
 * R as 16x16 tiles in the MFMA C layout (4 registers x 64 lanes each) and h.  Once per model
 * (white-noise) state, after gs_prefix / gs_prefix_dd; the values are copies (G negated), so
 * gs_bdraw_tiled's draws equal gs_bdraw's bit for bit.
 */
int64_t gs_model_tiled_stride(int NF, int NMX);
int gs_model_tile(gs_ctx* ctx, int n_psr, int NF, int NMX, const double* model, const int32_t* nm,
                  double* tiled);
/* gs_bdraw on gs_model_tile's blocks (the register-tile variant whatever GS_OPT_BCAST says):
 * same arguments and results, the model staged in the layout the draw loads lane-linearly. */
int gs_bdraw_tiled(gs_ctx* ctx, int n_psr, int n_chain, int NF, int NMX, int ldb,
                   const double* tiled, const int32_t* fidx, const int32_t* midx, const int32_t* nm,
                   const double* phiinv_F, const double* z, int64_t sweep, int event,
                   int64_t chain_base, const int32_t* chain_mask, double* b, int32_t* info);

/*
 * (a3) rho|b analytic draw: tau_k = (b_sin^2 + b_cos^2)/2 over fidx,
 * truncated inverse-gamma inverse CDF, x = 0.5 log10 rho.
 * Replaces pulsar_gibbs.py:206-216,236.  u: [n_sys x NF/2] injected U(0,1)
 * (NULL: Philox event GS_EV_RHO).  x: [n_sys x ldx] output (first NF/2 cols).
 */
int gs_rho_analytic(gs_ctx* ctx, int n_psr, int n_chain, int NF, int ldb, const int32_t* fidx,
                    const double* b, const double* u, int64_t sweep, int64_t chain_base,
                    double rhomin, double rhomax, double* x, int ldx);

/*
 * (a8) Fused free-spectrum sweep for independent chains (configs 1-3):
 * n_sweeps iterations of PulsarBlockGibbs.sample's loop body
 * (pulsar_gibbs.py:656-698): record (x, b) before the update, first b draw
 * from xs when the global sweep index is 0, analytic rho|b, the all(xnew !=
 * x_old[-1]) gate, b|rho — with each wavefront's state kept in registers.
 * x_state [n_sys x NF/2] log10 rho, b_state [n_sys x ldb]: read at entry,
 * written at exit.  x_rec [n_sweeps x n_sys x NF/2], b_rec [n_sweeps x n_sys x ldb]
 * (either may be NULL).  z0_inj [n_sys x ldb], z_inj [n_sweeps x n_sys x ldb],
 * u_inj [n_sweeps x n_sys x NF/2]: injected draws or NULL.  info [n_sys].
 */
int gs_sweep_freespec(gs_ctx* ctx, int n_psr, int n_chain, int NF, int NMX, int ldb,
                      const double* model, const int32_t* fidx, const int32_t* midx,
                      const int32_t* nm, double rhomin, double rhomax, int64_t chain_base,
                      double* x_state, double* b_state, int64_t it0, int n_sweeps,
                      double* x_rec, double* b_rec, const double* z0_inj, const double* z_inj,
                      const double* u_inj, int32_t* info);
/* (x_rec / b_rec may be pinned host memory: the kernel then writes the history straight to
   the host over PCIe, readable after the call's work completes.) */

/*
 * tau[p][k][c] = b_sin^2 + b_cos^2 over fidx (pta_gibbs.py:194-195, 259-260), or
 * half of it when half != 0 (pulsar_gibbs.py:208-209).  tau: [n_psr x NF/2 x n_chain].
 */
int gs_tau(gs_ctx* ctx, int n_psr, int n_chain, int NF, int ldb, const int32_t* fidx, const double* b,
           int half, double* tau);

/*
 * Grid conditionals.  grid3 = [rho_g | log rho_g | 0.5 log10 rho_g] (3 x ngrid, host numpy,
 * rho_g = 10**linspace(log10 rhomin, log10 rhomax, ngrid)).  Draws write
 * x[c * ldx + xcol[...]] = 0.5 log10 rho_g[idx] and, if idx_out != NULL, the index.
 * One lane per (chain, frequency) row walks the grid serially: numpy's order of
 * operations (sequential product over pulsars, sequential cumsum, cdf / max,
 * searchsorted(side='left') - 1 with -1 -> last point) is reproduced exactly.
 *
 * (a6) common free spectrum, product over pulsars (pta_gibbs.py:181-214):
 *   tau, irn [n_psr x n_f x n_chain] (irn NULL = no intrinsic red noise),
 *   u [n_chain x n_f] or NULL (Philox GS_EV_CURN); xcol [n_f].
 */
int gs_rho_curn(gs_ctx* ctx, int n_psr, int n_chain, int n_f, const double* tau, const double* irn,
                int ngrid, const double* grid3, const double* u, int64_t sweep, int64_t chain_base,
                double* x, int ldx, const int32_t* xcol, int32_t* idx_out);
/*
 *  Marginalised likelihood get_lnlikelihood_fullmarg (pulsar_gibbs.py:569-610,
 * pta_gibbs.py:577-621) for n_psr x n_chain systems from the prefix model blocks (one per
 * pulsar, or per system with model_per_sys): lnl[sys] = 1/2 (d^T Sigma^-1 d - log det Sigma)
 * + 1/2 sum_F log phiinv_F, -inf (and info > 0) if Sigma is not positive definite.  The
 * reference's value adds the model constants -1/2 (sum log N + r^T N^-1 r) + 1/2 sum_M log
 * phiinv_M.  NF = 20, 40, 60.
 */
int gs_lnlike_marg(gs_ctx* ctx, int n_psr, int n_chain, int NF, int NMX, const double* model,
                   int model_per_sys, const int32_t* nm, const double* phiinv_F, double* lnl, int32_t* info);
/* gs_lnlike_marg (shared model blocks) for the chains a gated b draw skipped: only systems of
   chains c with gate[c] == 0 are evaluated; the others keep their lnl (and info).  Ranks the
   chains with a workgroup ballot scan so only workgroups with work stage a model block (for a
   b draw without the lnl output, e.g. the row-major gs_bdraw path). */
int gs_lnlike_marg_gated(gs_ctx* ctx, int n_psr, int n_chain, int NF, int NMX, const double* model, const int32_t* nm,
                         const double* phiinv_F, const int32_t* gate, double* lnl, int32_t* info);

/*
 * (a6, sufficient statistic) CURN without per-pulsar red noise: the common pdf depends on
 * tau only through S[k][c] = sum_p tau[p][k][c] (pta_gibbs.py:194-205 with irn = 0), so a
 * pulsar-sharded run all-reduces S instead of gathering tau.
 * gs_tau_sum: S [n_f x n_chain] = sum over the n_psr local pulsars (sequential order).
 * gs_rho_curn_sum: the grid-CDF draw of pta_gibbs.py:181-214 from S and the GLOBAL
 * pulsar count n_psr, in log space (log pdf = -n_psr log rho_g - S / (2 rho_g));
 * equal to gs_rho_curn up to pdf rounding (1e-15 relative).  ngrid <= 2048.
 */
int gs_tau_sum(gs_ctx* ctx, int n_psr, int n_chain, int n_f, const double* tau, double* S);
/*
 * The tau sums in exact fixed point, for a pulsar-sharded run whose exchange must not depend on
 * the number of shards or the collective's reduction order (shard counts 1/2/4/8
 * give identical chains).  gs_tau_sum_fx: acc [3 x n_f x n_chain] int64 = the 48-bit digits of
 * sum_p floor(tau_p / 2^e0) (every tau truncated to the grid 2^e0, exact integer sums; n_psr <
 * 2^15), ovf (int32, may be NULL) set to 1 for a negative / non-finite tau or one >= 2^(e0+144).
 * Digits of several shards add as int64 (all-reduce SUM, any order) to the digits of the whole
 * array.  gs_fx_to_double: S [n] (n = n_f x n_chain) from summed digits, rounded the same way on
 * every rank.  PTAChains uses e0 = floor(log2 rhomin) - 64.
 */
int gs_tau_sum_fx(gs_ctx* ctx, int n_psr, int n_chain, int n_f, const double* tau, int e0, int64_t* acc,
                  int32_t* ovf);
int gs_fx_to_double(gs_ctx* ctx, int64_t n, int e0, const int64_t* acc, double* S);
/* gs_tau followed by gs_tau_sum_fx in one pass over b (tau never stored): the same digits.
   NF <= 64 (one lane per free-spectrum column; a workgroup per chain). */
int gs_tau_sum_fx_b(gs_ctx* ctx, int n_psr, int n_chain, int NF, int ldb, const int32_t* fidx, const double* b,
                    int e0, int64_t* acc, int32_t* ovf);
int gs_rho_curn_sum(gs_ctx* ctx, int n_psr, int n_chain, int n_f, const double* S, int ngrid,
                    const double* grid3, const double* u, int64_t sweep, int64_t chain_base, double* x,
                    int ldx, const int32_t* xcol, int32_t* idx_out);

/*
 * (a7) per-pulsar red free spectrum conditioned on phi_gw (pta_gibbs.py:252-276):
 *   tau [n_psr x n_f x n_chain], gw [n_f x n_chain] = phi_gw of the sin columns,
 *   u [n_chain x n_psr x n_f] or NULL (Philox GS_EV_RED); xcol [n_psr x n_f].
 */
int gs_rho_red(gs_ctx* ctx, int n_psr, int n_chain, int n_f, const double* tau, const double* gw,
               int ngrid, const double* grid3, const double* u, int64_t sweep, int64_t chain_base,
               double* x, int ldx, const int32_t* xcol, int32_t* idx_out);
/*
 * (a4) single pulsar with intrinsic red noise: grid + Gumbel-max (pulsar_gibbs.py:218-234).
 *   tau (half convention), irn [n_f x n_chain]; u [n_chain x n_f x ngrid] U(0,1) behind the
 *   Gumbels (G = -log(-log1p(-u))) or NULL (Philox GS_EV_GUMBEL); xcol [n_f].
 */
int gs_rho_gumbel(gs_ctx* ctx, int n_chain, int n_f, const double* tau, const double* irn, int ngrid,
                  const double* grid3, const double* u, int64_t sweep, int64_t chain_base, double* x,
                  int ldx, const int32_t* xcol, int32_t* idx_out);

/*
 *  Power-law intrinsic red noise, single pulsar (PulsarBlockGibbs with a red
 * signal, pulsar_gibbs.py:271-329, 549-566).  One wavefront per chain.
 * gs_red_mh: nsteps Metropolis steps on (log10_A, gamma) = x[c][red_col[0]], x[c][red_col[1]]
 *   under the red-only likelihood get_lnlikelihood_red (:549-566)
 *     lnL = sum_k lr_k - exp(lr_k),  lr_k = log tau_k - logaddexp(log irn_k, log 10^(2 x[c][gw_col[k]]))
 *   with log irn_k = lnphi[k] + lnphi[n_f + k] log10_A + lnphi[2 n_f + k] gamma (the power law,
 *   log-linear; lnphi [3 x n_f] probed on the host from the signal's get_phi) and tau
 *   [n_f x n_chain] in the half convention (gs_tau half = 1).  Proposals (symmetric):
 *   jump[12] = {U00, U01, U10, U11, sqrt S0, sqrt S1, P(SCAM), P(SCAM) + P(AM), lo_A, hi_A,
 *   lo_gamma, hi_gamma} (U, S: SVD of the block's proposal covariance; the remainder of the
 *   probability is the DE jump over de [nde x 2], nde >= 2 when used).  anchor = 1: every step
 *   is accepted against the block's starting lnL (the reference discards PTMCMCOneStep's
 *   returned state, :318-319); anchor = 0: against the current state.  Outputs: x (in place),
 *   irn [n_f x n_chain] = phi_red at the final state (or NULL), lnl [n_chain] = lnL at the final
 *   state (or NULL), n_acc [n_chain] accepted steps (or NULL).  nsteps = 0 evaluates only.
 *   Philox event GS_EV_REDMH, slots 4 s .. 4 s + 3 of step s.  n_f <= 256.
 * gs_gate_phiinv_irn: gs_pta_gate_phiinv for one pulsar with phi_F = 10**(2 x_gw) + irn
 *   (enterprise sums the phis of signals sharing the Fourier basis).
 */
int gs_red_mh(gs_ctx* ctx, int n_chain, int n_f, int nsteps, int anchor, double* x, int ldx,
              const int32_t* red_col, const int32_t* gw_col, const double* tau, const double* lnphi,
              const double* jump, const double* de, int nde, int64_t sweep, int64_t chain_base, double* irn,
              double* lnl, int32_t* n_acc);
int gs_gate_phiinv_irn(gs_ctx* ctx, int n_chain, int n_f, int n_param, const double* x, const double* xlast,
                       const int32_t* gw_col, const double* irn, double* phiinv_F, int32_t* gate);

/* out[j][c] = 10**(2 x[c * ldx + cols[j]]): free-spectrum phi (sin column) from log10 rho. */
int gs_phi_from_x(gs_ctx* ctx, int n_chain, int ncol, const double* x, int ldx, const int32_t* cols,
                  double* out);

/*
 * PTA sweep plumbing (PTABlockGibbs.sample, pta_gibbs.py:664-704):
 * gs_pta_record: x_rec[c] = x[c] (may be NULL), xlast[c] = x[c][n_param-1];
 * gs_pta_gate_phiinv: gate[c] = all(x[c] != xlast[c]) (xlast NULL: gate = 1) and
 *   phiinv_F[(p * n_chain + c) x 2 n_f] = 1 / (10**(2 x_gw) + 10**(2 x_red,p)) repeated
 *   over (sin, cos); gw_col [n_f], red_col [n_psr x n_f] or NULL.
 */
int gs_pta_record(gs_ctx* ctx, int n_chain, int n_param, const double* x, double* x_rec, double* xlast);
int gs_pta_gate_phiinv(gs_ctx* ctx, int n_psr, int n_chain, int n_f, int n_param, const double* x,
                       const double* xlast, const int32_t* gw_col, const int32_t* red_col,
                       double* phiinv_F, int32_t* gate);
/* gs_pta_gate_phiinv with the per-pulsar red phi given: phi = 10**(2 x_gw) + irn[p][k][c]
 * (irn [n_psr x n_f x n_chain], e.g. gs_phi_powerlaw's power-law red noise, pta_gibbs.py:518-519). */
int gs_pta_gate_phiinv_irn(gs_ctx* ctx, int n_psr, int n_chain, int n_f, int n_param, const double* x,
                           const double* xlast, const int32_t* gw_col, const double* irn, double* phiinv_F,
                           int32_t* gate);

/*
 * PTA red-noise hyper-parameters (PTABlockGibbs, redsample='mh', the reference's default;
 * pta_gibbs.py:278-340 with get_lnlikelihood :577-621).
 * gs_phi_powerlaw: out [n_psr x n_f x n_chain] = power-law red phi at the sin columns,
 *   exp((a_pk log10_A_p + c_pk) + g_pk gamma_p) (red_sig[p].get_phi(params)[::2], :198), with
 *   (log10_A_p, gamma_p) = x[c][pl_col[2p]], x[c][pl_col[2p+1]] and lnphi [n_psr x 3 x n_f] =
 *   (c, a, g) (a power-law PSD is log-linear in its parameters; host-probed from get_phi).
 * gs_hyper_mh: nsteps single-parameter Metropolis steps per chain, one wavefront each:
 *   scale = choice([.1, .5, 1, 3, 10], p=[.1, .15, .5, .15, .1]), j = choice(n_h), q[hcol[j]] +=
 *   randn * (0.05 n_h) * scale, accept if lnL(q) - lnL(x) > log(rand), lnL the summed
 *   marginalised likelihood.  Parameter j belongs to pulsar hpsr[j], so only that pulsar's term
 *   is re-evaluated: lnl_p [n_psr x n_chain] holds every pulsar's phi-dependent lnL at x (seed it
 *   with gs_lnlike_marg on the phiinv of x) and is updated in place.  A proposal outside [hlo[j],
 *   hhi[j]] (uniform prior) is rejected without a likelihood.  hpsr[j] = -1: parameter j belongs to
 *   a pulsar this call does not hold (pulsar-sharded run: every rank draws the same steps from the
 *   chain-level Philox counters and applies those of its own pulsars); its steps are skipped.
 *   Red phi of pulsar p: red_kind 0 =
 *   free spectrum 10**(2 x[red_col[p][k]]) (red_col [n_psr x n_f]); 1 = power law (pl_col,
 *   lnphi as above).  phi = 10**(2 x[gw_col[k]]) + red (the common spectrum is held fixed in the
 *   block).  inj [nsteps x n_chain x 4] = (scale, j, randn, rand) per step, or NULL (Philox event
 *   12, slots 3 s .. 3 s + 2).  q_rec [nsteps x n_chain x 3] = (j, proposed value, accepted) or
 *   NULL; n_acc [n_chain] accepted steps or NULL.  model: gs_prefix blocks, one per pulsar.
 */
int gs_phi_powerlaw(gs_ctx* ctx, int n_psr, int n_chain, int n_f, const double* x, int ldx, const int32_t* pl_col,
                    const double* lnphi, double* out);
int gs_hyper_mh(gs_ctx* ctx, int n_psr, int n_chain, int NF, int NMX, const double* model, const int32_t* nm,
                double* x, int ldx, const int32_t* gw_col, int n_h, const int32_t* hcol, const int32_t* hpsr,
                const double* hlo, const double* hhi, int red_kind, const int32_t* red_col, const int32_t* pl_col,
                const double* lnphi, double* lnl_p, int nsteps, int64_t sweep, int64_t chain_base,
                const double* inj, double* q_rec, int32_t* n_acc);

/* ------------------------------------------------------------------------
 * (a10) White-noise Metropolis block and the per-chain TNT it forces
 * (PulsarBlockGibbs.update_white_params pulsar_gibbs.py:332-406,
 * get_lnlikelihood_white :523-546, TNT recompute :500-502 / :664-665).
 *
 * N_i = efac_k^2 (sigma_i^2 + 10^(2 log10_t2equad_k)) + 10^(2 log10_tnequad_k) for the
 * backend k of TOA i (absent parameters: efac 1, equads 0).  TOAs of a pulsar are
 * stored grouped by backend (the likelihood is a sum, so the order is free);
 * y / sigma2 / r / bk rows use the pulsar's toa_off.  Per-chain arrays of TOAs
 * (y) are chain-major with leading dimension ldy (>= total TOAs).
 */
#define GS_WHITE_MAX_BK 15 /* backends per pulsar  */
#define GS_WHITE_MAX_W 32  /* white parameters per pulsar */
enum { GS_WHITE_EFAC = 0, GS_WHITE_TNEQUAD = 1, GS_WHITE_T2EQUAD = 2 };

typedef struct {
  int64_t n_toa;   /* TOAs of this pulsar                                          */
  int64_t toa_off; /* element offset into sigma2 / bk / r and each chain's y row    */
  int64_t w_off;   /* offset of this pulsar's parameters in the wcol/wkind/... tables */
  int32_t n_bk;    /* backends (<= GS_WHITE_MAX_BK)                                */
  int32_t n_w;     /* white parameters (<= GS_WHITE_MAX_W)                         */
  int32_t bk_off[GS_WHITE_MAX_BK + 1]; /* first TOA of each backend group; [n_bk] = n_toa */
} gs_white_desc;

/*
 * y = r - T b per (pulsar, chain) (pulsar_gibbs.py:534-535).  tdesc: the gs_tnt_desc
 * array with T_off indexing Tt, the COLUMN-major (m x n_toa) copy of T.
 * y: [n_chain x ldy], system (p, c) at y + c * ldy + toa_off.  n_toa_max: largest n_toa.
 */
int gs_white_resid(gs_ctx* ctx, int n_psr, int n_chain, int64_t n_toa_max, int ldb,
                   const gs_tnt_desc* tdesc, const double* Tt, const double* r, const double* b,
                   int64_t ldy, double* y);

/*
 * n_steps single-parameter Metropolis steps per (pulsar, chain) on the pulsar's
 * white parameters (pulsar_gibbs.py:373-404): scale from {0.1,0.5,1,3,10} w.p.
 * {.1,.15,.5,.15,.1}, one parameter uniformly, jump z * (0.05 n_w) * scale, Uniform
 * prior [wmin, wmax] (inclusive), accept if dlnL > log U.  One wavefront per system;
 * a step only re-sums the TOAs of the backend it touches.
 * wcol/wkind/wbk [sum n_w] int32: x column, GS_WHITE_* kind, backend; wmin/wmax [sum n_w].
 * x: [n_chain x ldx] read and updated in place.  nsteps_chain [n_chain] (NULL: n_steps).
 * inj [n_steps x n_sys x 4] (scale value, parameter index within the pulsar's list,
 * normal, uniform) or NULL (Philox GS_EV_WHITE, sweep `sweep`).
 * q_rec [n_steps x n_sys x GS_WHITE_MAX_W] proposals q[wind] (short_chain, :390) or NULL;
 * n_acc [n_sys] accepted steps or NULL.
 */
int gs_white_mh(gs_ctx* ctx, int n_psr, int n_chain, const gs_white_desc* wdesc,
                const int32_t* wcol, const int32_t* wkind, const int32_t* wbk, const double* wmin,
                const double* wmax, const double* sigma2, const double* y, int64_t ldy, double* x,
                int ldx, int n_steps, const int32_t* nsteps_chain, int64_t sweep, int64_t chain_base,
                const double* inj, double* q_rec, int32_t* n_acc);

/*
 * Per-chain TNT = T^T N_c^-1 T and d = T^T N_c^-1 r with N_c from the chain's white
 * parameters in x (pulsar_gibbs.py:495-502).  T row-major as in gs_tnt (tdesc T_off);
 * system (p, c) writes TNT + tdesc[p].tnt_off + c * tnt_cstride (m x m, full) and
 * d + tdesc[p].d_off + c * d_cstride.  bk [total TOAs] int32 backend of each TOA.
 */
int gs_white_tnt(gs_ctx* ctx, int n_psr, int n_chain, int m_max, const gs_tnt_desc* tdesc,
                 const gs_white_desc* wdesc, const int32_t* wcol, const int32_t* wkind,
                 const int32_t* wbk, const double* T, const double* sigma2, const int32_t* bk,
                 const double* r, const double* x, int ldx, int64_t tnt_cstride, int64_t d_cstride,
                 double* TNT, double* d);

/*
 * gs_prefix for per-chain systems: system (p, c) reads TNT + desc[p].tnt_off +
 * c * tnt_cstride, d + desc[p].d_off + c * d_cstride and writes its model block at
 * model + (p * n_chain + c) * gs_model_stride(NF, NMX).
 */
int gs_prefix_sys(gs_ctx* ctx, int n_psr, int n_chain, int NF, int NMX, const gs_prefix_desc* desc,
                  int64_t tnt_cstride, int64_t d_cstride, const double* TNT, const double* d,
                  const int32_t* fidx, const int32_t* midx, const double* phiinv_fixed,
                  double* model, int32_t* info);

/*
 * gs_prefix_sys from a double-double TNT / d (gs_tnt_dd): TNT_lo, d_lo at the same offsets and
 * strides as TNT, d, or NULL (= gs_prefix_sys).  TNT full (symmetric), as for gs_prefix.
 */
int gs_prefix_dd(gs_ctx* ctx, int n_psr, int n_chain, int NF, int NMX, const gs_prefix_desc* desc,
                 int64_t tnt_cstride, int64_t d_cstride, const double* TNT, const double* TNT_lo,
                 const double* d, const double* d_lo, const int32_t* fidx, const int32_t* midx,
                 const double* phiinv_fixed, double* model, int32_t* info);

/* gs_bdraw with one model block per system (model + sys * gs_model_stride). */
int gs_bdraw_sys(gs_ctx* ctx, int n_psr, int n_chain, int NF, int NMX, int ldb,
                 const double* model, const int32_t* fidx, const int32_t* midx, const int32_t* nm,
                 const double* phiinv_F, const double* z, int64_t sweep, int event,
                 int64_t chain_base, const int32_t* chain_mask, double* b, int32_t* info);

/* ------------------------------------------------------------------------
 *  Basis ECORR, single pulsar, n_chain chains
 * (PulsarBlockGibbs.update_ecorr_params pulsar_gibbs.py:409-486 on get_lnlikelihood_fullmarg
 * :569-610; the b draw of update_b :489-520 with the epoch columns; the sweep order of
 * pta_gibbs_freespec.ipynb's sampler: ECORR block, rho|b, gated b).
 *
 * The ne epoch columns E (ecid) of a basis-ECORR signal have a diagonal TNT block, so the
 * ECORR state enters only through a_e = TNT_ee + 1/phi_e, phi_e = 10**(2 x[c][xcol[ebk[e]]]).
 * R = the other mR columns in increasing order (rcol).  Caller-built, chain-independent:
 *   Bx [ne x ldbx] rows [TNT[e, R] | d_e | 0 ...], ldbx = 16 ceil((mR + 1) / 16) <= 128;
 *   Dg [ne] = TNT_ee;  A [mR x mR] = TNT_RR;  dR [mR] = d_R;  ebk [ne] backend of each epoch;
 *   xcol [n_bk] x column of each backend's log10_ecorr (n_bk <= GS_WHITE_MAX_BK).
 * gs_ecorr_schur: per chain TNT [c][mR x mR] = A - B^T diag(1/a) B, d [c][mR] = dR - B^T (d_E/a),
 *   aux [c][4] = {sum log a, sum d_E^2 / a, sum log phi_E, 0}.  The marginalised likelihood is
 *   then gs_lnlike_marg on the R system (gs_prefix_sys of TNT, d) + (aux1 - aux0 - aux2) / 2
 *   + the model constants.
 * gs_ecorr_propose: one Metropolis proposal per chain at step `step` (:458-462): the ECORR
 *   columns of xq = those of x with x[ecol[p]] += z (0.05 n_e) scale (other columns of xq are
 *   not written); prop [n_chain x 4] scratch.  inj [steps x n_chain x 4]
 *   (scale value, parameter index, normal, uniform) or NULL (Philox GS_EV_ECORR).
 *   emin/emax [n_e]: the Uniform prior of each ECORR parameter.
 * gs_ecorr_accept: lnL1 = lnl + (aux1 - aux0 - aux2)/2 (-inf if info or pinfo is nonzero);
 *   init = 1 stores lnL1 in lnl0 (the block's starting value); otherwise accepts
 *   (x[c][col] = proposed value, lnl0 = lnL1, n_acc += 1) when lnL1 - lnl0 > log U and the
 *   proposal is inside the prior (:465-472).  q_rec [n_chain x n_e] = q[eind] or NULL.
 * gs_ecorr_bdraw_e: b_E = (d_E - B b_R)/a + z/sqrt(a) and b[rcol[j]] = bR[j]: the full b
 *   (Bx column t multiplies bR[jmap[t]], skipped when jmap[t] < 0; d_E is column dcol; with the
 *   gs_ecorr_schur layout jmap = 0..mR-1, dcol = mR)
 *   [n_chain x ldb] in original column order from the R draw bR [n_chain x ldbR] (gs_bdraw_sys
 *   on the Schur systems).  z [n_chain x m] injected normals by original column, or NULL
 *   (Philox event `event`: GS_EV_ECORR_B / GS_EV_ECORR_B0).  chain_mask as in gs_bdraw.
 */
int gs_ecorr_schur(gs_ctx* ctx, int n_chain, int mR, int ne, int ldbx, const double* Bx, const double* Dg,
                   const int32_t* ebk, int n_bk, const int32_t* xcol, const double* x, int ldx,
                   const double* A, const double* dR, double* TNT, double* d, double* aux);
/*
 * gs_ecorr_prefix: gs_ecorr_schur + gs_prefix_sys fused (no per-chain TNT in HBM): writes each
 * chain's model block (gs_prefix layout, model + c * gs_model_stride(NF, NMX)) and aux [c][4]
 * as gs_ecorr_schur.  Columns reordered [M | F | d]: Bx [ne x ldbx] rows
 * [TNT[e, M] (nM <= 16, zero-padded to 16) | TNT[e, F] (fidx order, NF) | d_e | 0 ...];
 * Ap [ldbx x ldbx] the same ordering of TNT with phiinv_M added on the M diagonal, d as row and
 * column 16 + NF, (d, d) = 0 and 1 on the padded M diagonal; ldbx = 16 (1 + ceil((NF + 1) / 16))
 * in {48, 64, 80} (NF = 20, 40, 60); 1 on every padded diagonal.  info [c] > 0: the k-th pivot failed.
 * Likelihood mode (lnl != NULL; model unused, may be NULL): phiinv_F [n_chain x NF] (fidx order)
 * is added and the F block factored in registers; lnl [c] = (d^T Sigma^-1 d - log det S_R -
 * ... ) / 2 in gs_ecorr_accept's convention with aux [c][1] = 0 (lnL = lnl + (aux1 - aux0 -
 * aux2) / 2 + constants), so one launch per Metropolis step replaces gs_ecorr_prefix +
 * gs_lnlike_marg.
 */
int gs_ecorr_prefix(gs_ctx* ctx, int n_chain, int NF, int NMX, int nM, int ne, int ldbx, const double* Bx,
                    const double* Dg, const int32_t* ebk, int n_bk, const int32_t* xcol, const double* x,
                    int ldx, const double* Ap, const double* phiinv_F, double* model, double* aux,
                    double* lnl, int32_t* info, int64_t bx_cstride, int64_t dg_cstride, int64_t ap_cstride);
/*
 * gs_ecorr_lnl_state: gs_ecorr_prefix's likelihood mode with a stored per-chain state, for the
 * Metropolis steps of update_ecorr_params (pulsar_gibbs.py:456-484; the reference re-factors the full
 * system per step).  tbuf [2][n_chain][NT x 256] doubles (NT = the 16 x 16 tiles of the [M | F | d]
 * upper triangle, (ldbx / 16) (ldbx / 16 + 1) / 2), tidx [n_chain] the chain's current slot.
 *   x_old == NULL: full evaluation at x (as gs_ecorr_prefix), T = Ap - P(x) stored in slot tidx[c].
 *   x_old != NULL: one step from the state at x_old to the proposal x, which moves one backend's
 *     ECORR parameter (column prop[c * 4], gs_ecorr_propose's record): only that backend's epochs
 *     are re-weighted, T(x) = T(x_old) - sum_{e of the backend} (1/a_e(x) - 1/a_e(x_old)) Bx_e^T Bx_e,
 *     read from slot tidx[c] and written to slot tidx[c] ^ 1.  Epochs must be grouped by backend:
 *     eoff [n_bk + 1] the first epoch of each backend (eoff[n_bk] = ne); Ap is not read.
 * lnl / aux / info as gs_ecorr_prefix's likelihood mode.  gs_ecorr_accept_propose2 with tidx adopts
 * the proposal's slot on acceptance.  Equal to the full evaluation to rounding (tests); the host
 * re-evaluates from Ap at every Metropolis block's start.
 */
int gs_ecorr_lnl_state(gs_ctx* ctx, int n_chain, int NF, int NMX, int nM, int ne, int ldbx, const double* Bx,
                       const double* Dg, const int32_t* ebk, int n_bk, const int32_t* xcol, const int32_t* eoff,
                       const double* x, const double* x_old, const double* prop, int ldx, const double* Ap,
                       const double* phiinv_F, double* tbuf, int32_t* tidx, double* aux, double* lnl, int32_t* info,
                       int64_t bx_cstride, int64_t dg_cstride, int64_t ap_cstride);
/*
 * White noise sampled with ECORR (per-chain N): Bx / Dg / Ap differ per chain.  gs_ecorr_gather
 * builds them from per-chain TNT [c][m x m] (tnt_cstride) and d [c][m] (d_cstride), e.g.
 * gs_white_tnt's output: Bx [c][ne x kb], Dg [c][ne], Ap [c][kb x kb] with colmap [kb] = the
 * original column of each reordered column, -1 for padding (1 on the Ap diagonal), -2 for d;
 * phm [16] = phiinv of the fixed-prior columns (added on the Ap diagonal of the first 16).
 * Pass the per-chain strides (ne kb, ne, kb kb) to gs_ecorr_prefix / gs_ecorr_bdraw_e.
 */
/*
 * gs_ecorr_epoch_sums: the per-chain [B | d_E] rows and epoch diagonal straight from the TOAs
 * (white noise sampled): Bx [c][e][j] = sum_{q in eptr[e]..eptr[e+1]} eu[q] T[etoa[q]][colmap[j]]
 * / N_c, column dcol = sum eu r / N_c, Dg [c][e] = sum eu^2 / N_c, N_c from chain c's white
 * parameters in x (the gs_white_mh / gs_white_tnt tables of one pulsar; T row-major
 * n_toa x m, TOAs in the order of sigma2 / bk / r).  With the epoch columns of T being
 * quantisation indicators this equals TNT[ecid[e], colmap[j]] of the full SYRK.
 */
int gs_ecorr_epoch_sums(gs_ctx* ctx, int n_chain, const gs_white_desc* wdesc, const int32_t* wcol,
                        const int32_t* wkind, const int32_t* wbk, const double* x, int ldx, const double* T, int m,
                        const double* sigma2, const int32_t* bk, const double* r, int ne, int kb, int dcol,
                        const int32_t* colmap, const int32_t* eptr, const int32_t* etoa, const double* eu,
                        double* Bx, double* Dg);
int gs_ecorr_gather(gs_ctx* ctx, int n_chain, int m, int ne, int kb, const int32_t* ecid, const int32_t* colmap,
                    const double* phm, const double* TNT, int64_t tnt_cstride, const double* d,
                    int64_t d_cstride, double* Bx, double* Dg, double* Ap);
int gs_ecorr_propose(gs_ctx* ctx, int n_chain, int n_e, const int32_t* ecol, const double* emin,
                     const double* emax, const double* x, int ldx, int n_param, double* xq, int step,
                     int64_t sweep, int64_t chain_base, const double* inj, double* prop);
int gs_ecorr_accept(gs_ctx* ctx, int n_chain, int n_e, const int32_t* ecol, int init, const double* lnl,
                    const int32_t* info, const int32_t* pinfo, const double* aux, const double* prop,
                    const double* xq, double* x, int ldx, double* lnl0, double* q_rec, int32_t* n_acc);
/* gs_ecorr_accept followed, in the same launch, by gs_ecorr_propose's proposal for step
 * next_step (< 0: none) from the updated x: one launch per Metropolis step. */
int gs_ecorr_accept_propose(gs_ctx* ctx, int n_chain, int n_e, const int32_t* ecol, int init, const double* lnl,
                            const int32_t* info, const int32_t* pinfo, const double* aux, double* prop,
                            double* xq, double* x, int ldx, double* lnl0, double* q_rec, int32_t* n_acc,
                            const double* emin, const double* emax, int n_param, int next_step, int64_t sweep,
                            int64_t chain_base, const double* inj);
/* gs_ecorr_accept_propose that also flips tidx [c] (gs_ecorr_lnl_state's slot) on acceptance
 * (tidx == NULL: identical to gs_ecorr_accept_propose). */
int gs_ecorr_accept_propose2(gs_ctx* ctx, int n_chain, int n_e, const int32_t* ecol, int init, const double* lnl,
                             const int32_t* info, const int32_t* pinfo, const double* aux, double* prop,
                             double* xq, double* x, int ldx, double* lnl0, double* q_rec, int32_t* n_acc,
                             const double* emin, const double* emax, int n_param, int next_step, int64_t sweep,
                             int64_t chain_base, const double* inj, int32_t* tidx);
int gs_ecorr_bdraw_e(gs_ctx* ctx, int n_chain, int mR, int ne, int ldbx, const double* Bx, const double* Dg,
                     const int32_t* ebk, const int32_t* xcol, const double* x, int ldx, const double* bR,
                     int ldbR, const int32_t* ecid, const int32_t* rcol, int m, const double* z,
                     int64_t sweep, int event, int64_t chain_base, const int32_t* chain_mask, double* b,
                     int ldb, int64_t bx_cstride, int64_t dg_cstride, int dcol, const int32_t* jmap);

/*
 * Philox4x32-10 test hook: out[i] = the 4 words for counter
 * (ctr[4*i..4*i+3]) under the context key.  ctr/out: [n x 4] uint32.
 */
int gs_philox(gs_ctx* ctx, int64_t n, const uint32_t* ctr, uint32_t* out);

#ifdef __cplusplus
}
#endif
#endif /* PULSAR_GIBBS_H */
