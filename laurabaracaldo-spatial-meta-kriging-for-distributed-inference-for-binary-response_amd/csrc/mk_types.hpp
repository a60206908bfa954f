// Device-resident state of one batch of subsets (one GPU's shard).
//
// HBM layout (S local subsets, q outcomes, n_pad = roundup(max n_s + 1, 128)):
//   coords  [S][2][n_pad]            SoA x | y (padding 0)
//   y, wt   [S][Np]                  Np = n_pad*q, location-major (i*q + a), padding 0
//   X       [S][p][Np]               column-major design
//   eta, w  [S][Np]
//   L       [S*q][2][n_pad^2]        accepted / candidate lower Cholesky factors of R_h
//                                    (row n_s of a candidate holds u_h: bordered solve -> z)
//   Winv    [S*q][2][nt][128^2]      inverses of the diagonal 128-tiles of each factor
//   W       [S*q][n_pad^2]           W_h = L_h^-1 of the accepted factor (lower, column-major)
//   QB      [S*q][nt][128^2]         diagonal 128-tiles of R_h^-1 = W'W (rows < n_s)
//   u, z    [S][q][n_pad]            u = (I (x) A^-1) w, z_h = W_h u_h  (so u_h'R_h^-1 u_h = |z_h|^2)
//   Z       [S][q][q][n_pad]         Z_{h,c} = W_h u_c (q > 1 only)
//   bacc,zc [S][q][n_pad]            lookahead: border-solve partial sums, z'_h = L'_h^-1 u_h
//   Y       [S*q][n_pad^2]           lookahead: inverse-level scratch (else the free factor slot)
//   PT, XK  [S*q][n_pad][n_test_pad] kriging: P^T = rho(obs, test) and X = W P^T
// All matrices of one (subset, outcome) pair are contiguous; every kernel finds
// its pair from blockIdx and the cur[] slot table, so no host round trip is
// needed between the steps of an iteration.
#pragma once
#include "mk_common.hpp"

#define MK_QMAX 4
#define MK_CD_SPLIT 8        // k_inv_copydiag: workgroups per 128-tile (kernel and launch grid)
#define MK_QUANT_MAX 16384   // kept samples per quantile summary (k_quantiles sorts them in 128 KB of LDS)

namespace mk {

struct Model {
  int S, q, p, n_pad, Np, nt, ntri, n_theta, cov_model;
  int link;                               // MK_LINK_LOGIT | MK_LINK_PROBIT
  int o_A, o_phi, o_nu, o_w, n_mh_max;   // MH parameter offsets (spBayes order)
  int n_batch, batch_length, n_samples, kept0, n_kept;
  int n_test, n_test_pad, ntt;
  int subset_base;                        // global index of local subset 0
  int S_all;                              // subsets of the whole shard (stride of the kept-state records)
  int t_off;                              // global index of test site 0 (tiled kriging; 0 when fused)
  uint64_t seed;
  double accept_rate;
  double phi_a[MK_QMAX], phi_b[MK_QMAX], nu_a[MK_QMAX], nu_b[MK_QMAX];
  double iw_df, iw_S[MK_QMAX * MK_QMAX];
  // data
  const int* n_s;
  const double* coords;
  const double* y;
  const double* wt;
  const double* X;
  const double* coords_test;   // [2][n_test_pad]
  const double* span;          // [S] bounding-box diagonal of the subset's sites (Matern tables)
  const double* span_pt;       // [S] bound on the subset-to-test-site distances (Matern kriging tables)
  double* chtab;               // [S*q][MK_CH_TAB] Matern: Chebyshev tables of the pairs' candidates (k_matern_table)
  double* chtab_p;             // [S*q][MK_CH_TAB] Matern: tables of the current (phi, nu), kriging (k_matern_table_list)
  // state
  double* beta;      // [S][p]
  double* theta;     // [S][n_theta]: A lower-tri (log diag) | logit phi | logit nu
  double* w;         // [S][Np]
  double* eta;       // [S][Np]
  double* tune;      // [S][n_mh_max]  log proposal sd
  double* acc;       // [S][n_mh_max]  accept counts within the current batch
  double* u;         // [S][q][n_pad]
  double* z;         // [S][q][n_pad]
  double* Z;         // [S][q][q][n_pad]
  double* logdetR;   // [S][q]
  double* quad;      // [S][q]      u_h' R_h^-1 u_h at the current state
  double* A_full;    // [S][q*q]    current A (col-major)
  double* Ainv;      // [S][q*q]
  int* dirty;        // [S*q]
  // candidate scratch
  double* ld_part;   // [S*q][nt]   logdet partials of the candidate factor (per (subset, outcome) pair)
  double* quad_c;    // [S*q]
  int* info;         // [S*q]
  // sweep scratch
  double* sw_delta;  // [S][Np]
  double* sw_dll;    // [S][Np]
  double* sw_logu;   // [S][Np]
  int* sw_acc;       // [S][Np]
  // outputs
  double* samples;     // [S][n_samples][P]   reported columns beta | K | phi | nu
  double* acc_hist;    // [S][n_batch][p+n_theta+1]  per-batch accept rates (last = mean over w)
  double* w_samples;   // [S][n_samples][Np] or null
  double* s_pred;      // [S][q][n_test_pad]  kriging variance reduction for the current (phi, nu)
  double* s_part;      // [S*q][nt][n_test_pad]
  double* PT;          // [S*q][n_pad][n_test_pad]
  double* XK;          // [S*q][n_test_pad][n_pad]  column t = W rho_t
  double* w_pred;      // [S][n_kept][q*n_test]   (tiled kriging: q*tile)
  // kept chain states for tiled kriging: [n_kept][S_all][...]
  double* kz;          // z_h = W_h u_h   (q*n_pad)
  double* kth;         // theta           (n_theta)
  double* kA;          // A               (q*q)
  // lookahead schedule (mk_api.hip): border solve of the candidate factored ahead of its iteration
  double* bacc;        // [S][q][n_pad]     right-looking partial sums of the border solve
  double* zc;          // [S][q][n_pad]     z'_h = L'_h^-1 u_h of the candidate
  int* la_nu;          // [S*q]             Matern: 1 where this iteration's nu step accepted (k_nu_border)
  int P;               // reported columns
};

struct MatSet {
  double* L;
  double* Winv;
  double* W;   // [S*q][ld*ld] inverse factor (persistent)
  double* Q;   // [S*q][ld*ld] full inverse (parity-test entry point only)
  double* QB;  // [S*q][nt][128*128] diagonal tiles of the inverse
  int* cur;    // [S*q]
  double* Y;   // [S*q][ld*ld] inverse-level scratch (lookahead schedule; else the free factor slot)
  int ld, nt, q;
};

// phi-interpolated tiled kriging (mk_mcmc.hip section 11, mk_api.hip predict_tile_cheb)
#define MK_CHEB_MAX 32      // Chebyshev nodes per subset at most
#define MK_CHEB_CHECKS 3    // exact check values per subset and tile: the kept range's ends and middle
#define MK_CHEB_CHECKS_MAX 5
struct ChebK {
  const double* Sn;     // [slot][S][T_pad]  exact s at the nodes (slots < nc[s]) and the check points
  const double* nphi;   // [slot][S]         the slots' phi (as the candidate assembly computed it)
  const double* wts;    // [S][MK_CHEB_MAX]  barycentric weights
  const int* nc;        // [S]               nodes
  int nchk;             // check slots per subset (after the nodes)
  long T_pad;
};

__device__ inline long mat_elems(const MatSet& m) { return (long)m.ld * m.ld; }
__device__ inline double* mat_slot(const MatSet& m, int sh, int slot) {
  return m.L + ((long)sh * 2 + slot) * mat_elems(m);
}
__device__ inline double* winv_slot(const MatSet& m, int sh, int slot, int k) {
  return m.Winv + (((long)sh * 2 + slot) * m.nt + k) * (MK_NB * MK_NB);
}
__device__ inline Key subset_key(const Model& md, int s) { return make_key(md.seed, (uint32_t)(md.subset_base + s)); }

// XCD-aware block -> (entry, tile) map.  Blocks are dealt round-robin over the 8 XCDs
// (block b runs on XCD b % 8); the S*T work items are cut into 8 contiguous chunks and XCD x
// takes chunk x in order, so the tiles of one entry (subset) run on one XCD and share its L2
// (its shared panel is fetched once), and every XCD gets an equal share however few entries
// are active (a short list of changed subsets no longer leaves XCDs idle).  S is the number of
// ACTIVE entries; the grid (xcd_grid of the maximum) covers any S up to that maximum.  Speed
// only; any placement is correct.
__device__ inline bool xcd_map(int S, int T, int* s, int* t) {
  const int W = S * T, C = (W + 7) >> 3;
  const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
  if (j >= C) return false;
  const int w = x * C + j;
  if (w >= W) return false;
  *s = w / T;
  *t = w % T;
  return true;
}
__host__ inline int xcd_grid(int S, int T) { return 8 * ((S + 7) / 8) * T; }


}  // namespace mk
