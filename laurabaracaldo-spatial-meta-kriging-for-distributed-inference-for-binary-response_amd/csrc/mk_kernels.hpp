// Kernel declarations shared by the launch code (mk_api.hip).
#pragma once
#include "mk_types.hpp"
#include "mk_corr.hpp"

namespace mk {
inline int xcd_grid_h(int S, int T) { return 8 * ((S + 7) / 8) * T; }
// mk_linalg.hip
template <int MODEL>
__global__ void k_cov_candidate(Model md, MatSet ms, int h0, int hc, int which, int iter, const int* slist, const int* scount);
// the candidate kernel specialised for the session's covariance model
typedef void (*CovCandidateKernel)(Model, MatSet, int, int, int, int, const int*, const int*);
inline CovCandidateKernel cov_candidate_kernel(int model) {
  return model == MK_COV_EXPONENTIAL ? k_cov_candidate<MK_COV_EXPONENTIAL> : k_cov_candidate<MK_COV_MATERN>;
}
template <int TM, int TN = TM>
__global__ void k_chol_update(MatSet ms, int S, int h0, int hc, int k, int ia, int ib, int j0, int j1,
                              const int* slist, const int* scount);
template <int TM>
__global__ void k_chol_trsm(MatSet ms, int S, int h0, int hc, int k, int ia, int ib, const int* slist,
                            const int* scount);
int pv_grid(int max_entries, int nt, int ntt);   // k_pred_var's grid (mk_linalg.hip)
template <int TM>
__global__ void k_chol_update_trsm(MatSet ms, int S, int h0, int hc, int k, int ia, int ib, int j0, int extra,
                                   const int* slist, const int* scount);
__global__ void k_chol_diag(MatSet ms, const int* n_s, int h0, int hc, int k, double* ld_part, double* quad_c, int* info,
                            const int* slist, const int* scount, int cj0, int cj1);
__global__ void k_inv_copydiag(MatSet ms, const int* list, const int* count);
template <int TM>
__global__ void k_inv_level(MatSet ms, const int* list, const int* count, int sz, int phase);
__global__ void k_lauum(MatSet ms, const int* n_s, const int* list, const int* count);
__global__ void k_qblocks(MatSet ms, const int* n_s, const int* list, const int* count);
__global__ void k_take_border(Model md, MatSet ms, const int* list, const int* count, const double* zc);
__global__ void k_cand_border(Model md, MatSet ms, int h0, int hc);
__global__ void k_pred_draw_runs(Model md, const double* kz, const double* kA, int k_lo, const int* plist,
                                 const int* pcount, const int* run_start, int j_end);
__global__ void k_run_start(const int* plist, const int* pcount, int* run_start, int j);
__global__ void k_border_step(Model md, MatSet ms, int k);
__global__ void k_nu_border(Model md, MatSet ms);
__global__ void k_border_quad(Model md);
__global__ void k_trmv_Z(Model md, MatSet ms);
template <int MODEL>
__global__ void k_pred_PT(Model md, const int* list, const int* count);
__global__ void k_pred_PT_matern(Model md, const int* list, const int* count);
__global__ void k_matern_table(Model md, int h0, int hc, int which, int iter, const int* slist, const int* scount);
__global__ void k_matern_table_list(Model md, const int* list, const int* count);
typedef void (*PredPTKernel)(Model, const int*, const int*);
inline PredPTKernel pred_PT_kernel(int model) {
  return model == MK_COV_EXPONENTIAL ? k_pred_PT<MK_COV_EXPONENTIAL> : k_pred_PT<MK_COV_MATERN>;
}
template <bool GEN>
__global__ void k_pred_var(Model md, MatSet ms, const int* list, const int* count);
__global__ void k_pred_var_reduce(Model md, int nt, const int* list, const int* count);
// mk_mcmc.hip
__global__ void k_beta(Model md, int iter);
__global__ void k_Aphase(Model md, int iter);
__global__ void k_theta_mh(Model md, MatSet ms, int h0, int hc, int which, int iter);
__global__ void k_dirty_list(Model md, int force, int* list_inv, int* count_inv, int* list_pred, int* count_pred);
template <int Q>
__global__ void k_sweep(Model md, MatSet ms, int iter, const int* adm, int* fb);
template <int Q>
__global__ void k_sweep_mg(Model md, MatSet ms, int iter, double* part, int* cnt, int* xcc, int* err, int* adm, int spins_max);
template <int Q, int KR, int P, int HH, int LN>
__global__ void k_sweep_site(Model md, MatSet ms, int iter);
// its dynamic LDS: the sites' proposal / likelihood difference / accept draw + the accept flags
inline size_t sweep_site_lds_bytes(int ns_max, int q, int lean = 0) { return (size_t)ns_max * q * (lean ? 4 : 3) * 8 + (size_t)ns_max * 4; }
// the one-pass site sweep (kr 1: n_pad <= 2048, four row pairs per thread; 2: <= 4096, eight); NULL
// where its registers would spill (q = 3 with kr = 2, q = 4): the 64-site-block kernels run there
// q = 1: the lean pair form (two sites per barrier, fused-multiply-add dots, no row masks beyond the
// one upper element a pair loads; lean 1: the border row dropped by a factor; 2: for shards whose
// n_s are all even, no border element in a loaded pair); q = 2, 3: one site per barrier, masked.
inline const void* sweep_site_kernel(int q, int kr, int lean = 1) {
  if (q == 1) {
    if (kr == 1)
      return lean == 1 ? (const void*)k_sweep_site<1, 4, 2, 0, 1> : (const void*)k_sweep_site<1, 4, 2, 0, 2>;
    return lean == 1 ? (const void*)k_sweep_site<1, 8, 2, 0, 1> : (const void*)k_sweep_site<1, 8, 2, 0, 2>;
  }
  switch (q) {
    case 2: return kr == 1 ? (const void*)k_sweep_site<2, 4, 1, 0, 0> : (const void*)k_sweep_site<2, 8, 1, 0, 0>;
    case 3: return kr == 1 ? (const void*)k_sweep_site<3, 4, 1, 0, 0> : nullptr;
    default: return nullptr;
  }
}
template <int Q>
__global__ void k_sweep_step(Model md, MatSet ms, int iter, int B, double* part);
inline const void* sweep_step_kernel(int q) {
  switch (q) {
    case 1: return (const void*)k_sweep_step<1>;
    case 2: return (const void*)k_sweep_step<2>;
    case 3: return (const void*)k_sweep_step<3>;
    default: return (const void*)k_sweep_step<4>;
  }
}
// the sweep kernels specialised for the session's number of outcomes
inline const void* sweep_kernel(int q, bool mg) {
  switch (q) {
    case 1: return mg ? (const void*)k_sweep_mg<1> : (const void*)k_sweep<1>;
    case 2: return mg ? (const void*)k_sweep_mg<2> : (const void*)k_sweep<2>;
    case 3: return mg ? (const void*)k_sweep_mg<3> : (const void*)k_sweep<3>;
    default: return mg ? (const void*)k_sweep_mg<4> : (const void*)k_sweep<4>;
  }
}
__global__ void k_record(Model md, int iter);
__global__ void k_record_w(Model md, int iter);
__global__ void k_adapt(Model md, int b);
__global__ void k_pred_draw(Model md, int iter, int kidx);
__global__ void k_quantiles(const double* data, long subset_stride, long row_stride, int n_rows, int n_cols,
                            const double* probs, int n_probs, double* out);
__global__ void k_combine(const double* grids, int K, long G, double* out, int mean);
__global__ void k_record_kept(Model md, int kidx);
__global__ void k_kept_dirty(Model md, const double* th_prev, int* slist, int* scount, int* plist, int* pcount);
__global__ void k_flip_pairs(MatSet ms, const int* plist, const int* pcount);
__global__ void k_kept_phi(Model md, const double* th, int n, double* phis);
__global__ void k_krig_g(Model md, MatSet ms, const double* z, double* Gt, int j, int nkp);
__global__ void k_cheb_check(Model md, ChebK c, unsigned long long* err);
__global__ void k_kt_snap(Model md, double* zs, double* phis, double* As);
__global__ void k_pred_tab_draw(Model md, ChebK c, const double* g, const double* coords, const double* phis,
                                const double* As, int iter, int kidx);
__global__ void k_pred_cheb_draw(Model md, ChebK c, const double* Gt, const double* phit, const double* coords,
                                 const double* kA, int k_lo, int nkp);
// mk_post.hip
__global__ void k_weiszfeld(const double* grids, int K, int L, long C, int max_iter, double tol, double* out, int* iters);
__global__ void k_post_index(uint64_t seed, int samplesize, int n_levels, int* idx);
__global__ void k_post_interp(const double* grid, int L, long C, const int* idx, int S, const int* lo, const int* hi,
                              const int* mode, const double* t, double* out);
__global__ void k_post_prob(const double* sample_par, int S, const double* x_test, long C, int p, const double* sample_w,
                            int link, double* pout);
__global__ void k_glm_pass(const double* yprop, const double* wt, const double* X, long n, int p, const double* coef,
                           int mode, int link, double* part);
// mk_init.hip
__global__ void k_init_state(Model md);
__global__ void k_theta_init(Model md, MatSet ms, int h0, int hc);
__global__ void k_load_plain(MatSet ms, const double* A, int n, int S);
__global__ void k_extract_candidate(MatSet ms, int n, int S, double* out);
__global__ void k_extract_L(MatSet ms, int n, int S, double* L, int inv_slot_mode);
}  // namespace mk
