// Batched covariance assembly, blocked left-looking Cholesky and explicit
// inverse for every (subset, outcome) correlation matrix on the GPU.
//
// Replaces the spBayes internals behind spMvGLM (MK.R:80-84): spCovLT-style
// covariance assembly + LAPACK dpotrf/dpotri.
//
// Cholesky (lower, NB = 128, nt tiles per side), for panel k = 0..nt-1:
//   k_chol_update : C(i,k) -= L(i,0:k) L(k,0:k)^T        for i >= k   (MFMA GEMM, K = 128k)
//   k_chol_diag   : factor C(k,k) in LDS, invert it (Winv_k), logdet partial,
//                   read the bordered row (quadratic form u' R^-1 u)
//   k_chol_trsm   : L(i,k) = C(i,k) Winv_k^T                for i > k    (MFMA GEMM, K = 128)
// Inverse of an accepted factor, W = L^-1: diagonal tiles from the Winv of the
//   factorisation (k_inv_copydiag), then recursive doubling over block pairs
//   (k_inv_level: W_BT = -W_BB L_BT W_TT, log2(nt) levels x 2 MFMA GEMM launches)
// then the diagonal 128-tiles of R^-1 = W'W (k_qblocks) for the latent sweep;
// the full W'W (k_lauum) only serves the parity-test entry point.
// Kriging (kept iterations): P^T = rho(obs, test) materialised once per changed
// (phi, nu) (k_pred_PT) and X = W P^T (k_pred_var, MFMA) give both the variance
// reduction |X_t|^2 and, every kept iteration, the mean X_t . z.
#include "mk_gemm.hpp"
#include "mk_types.hpp"
#include "mk_corr.hpp"

namespace mk {

// ---------------------------------------------------------------- covariance
// Candidate correlation matrix of outcome h for every subset, lower tiles only:
//   R[i][j] = rho(|s_i - s_j|; phi', nu')  (i, j < n_s);  R[n_s][j] = u_h[j];  R[n_s][n_s] = 0;
//   padding rows/cols: identity.  phi'/nu' = the Philox proposal of MH parameter j_mh.
//   which | MK_CAND_NOBORDER: R[n_s][j] = 0 (the lookahead schedule factors the candidate before
//   u is known and solves for z' afterwards, k_border_step).
__device__ inline void candidate_theta(const Model& md, int s, int h, int which, int iter, double* phi, double* nu) {
  const Key key = subset_key(md, s);
  const double* th = md.theta + (long)s * md.n_theta;
  const int idx_phi = md.ntri + h, idx_nu = md.ntri + md.q + h;
  double tphi = th[idx_phi];
  double tnu = (md.cov_model == MK_COV_MATERN) ? th[idx_nu] : 0.0;
  if (which == 0 || which == 1) {   // which == 2: current values (initial factorisation)
    const int j_mh = (which == 0) ? md.o_phi + h : md.o_nu + h;
    const double z = proposal_normal(key, (uint32_t)j_mh, (uint32_t)iter);
    const double step = exp(md.tune[(long)s * md.n_mh_max + j_mh]) * z;
    if (which == 0) tphi += step; else tnu += step;
  }
  *phi = logit_inv(tphi, md.phi_a[h], md.phi_b[h]);
  *nu = (md.cov_model == MK_COV_MATERN) ? logit_inv(tnu, md.nu_a[h], md.nu_b[h]) : 0.0;
}

// Element (R, C) of the candidate matrix of one (subset, outcome).
struct CandGen {
  const double* cx;
  const double* cy;
  const double* uh;
  int ns;
  CorrFn rho;
  __device__ inline double operator()(int R, int C) const {
    if (R < ns && C < ns) return (R == C) ? 1.0 : rho(dist2d(cx[R], cy[R], cx[C], cy[C]));
    if (R == ns && C < ns) return uh ? uh[C] : 0.0;
    return (R == C && R != ns) ? 1.0 : 0.0;
  }
};

__device__ inline CandGen make_gen(const Model& md, int s, int h, int which, int iter) {
  CandGen g;
  double phi, nu;
  candidate_theta(md, s, h, which, iter, &phi, &nu);
  g.rho.init(phi, nu, md.cov_model);
  g.cx = md.coords + (long)s * 2 * md.n_pad;
  g.cy = g.cx + md.n_pad;
  g.uh = md.u + ((long)s * md.q + h) * md.n_pad;
  g.ns = md.n_s[s];
  return g;
}

// Lower tiles (i >= j) of every candidate of outcome h (tiles with j < jmin are skipped).
// Generating tiles inside k_chol_update at their first touch (gen = 1) was measured
// slower on cfg3 (+3.5 ms of exp work at 2 waves/SIMD vs 1.7 ms for this pass).
// Optional subset list (tiled kriging refactors only the subsets whose (phi, nu) changed):
// entry e -> subset slist[e] for e < *scount; slist == nullptr: every subset.
// Number of active (subset, outcome) entries of a launch over hc outcomes (list-aware).
__device__ inline int active_pairs(const int* slist, const int* scount, int S, int hc) {
  return (slist ? *scount : S) * hc;
}
__device__ inline bool pick_subset(const int* slist, const int* scount, int* s) {
  if (!slist) return true;
  if (*s >= *scount) return false;
  *s = slist[*s];
  return true;
}

// Entry e of a launch over hc outcomes h0 .. h0+hc-1 -> (subset, outcome).  The outcomes'
// factorisations are independent (LMC: u_h has its own GP), so one launch carries all q of
// them and the grid is q times fuller than an outcome-at-a-time schedule.
__device__ inline bool pick_pair(const int* slist, const int* scount, int e, int h0, int hc, int* s, int* h) {
  *s = e / hc;
  *h = h0 + e % hc;
  return pick_subset(slist, scount, s);
}

// MODEL = MK_COV_EXPONENTIAL: exp(-phi d) inline (the same expression CorrFn evaluates, so
// bit-identical), without the Matern/Bessel code and its registers in the kernel.
template <int MODEL>
__device__ inline double cand_value(const CandGen& g, int R, int C) {
  if (R < g.ns && C < g.ns) {
    if (R == C) return 1.0;
    const double d = dist2d(g.cx[R], g.cy[R], g.cx[C], g.cy[C]);
    return (MODEL == MK_COV_EXPONENTIAL) ? exp(-g.rho.phi * d) : g.rho(d);
  }
  if (R == g.ns && C < g.ns) return g.uh ? g.uh[C] : 0.0;
  return (R == C && R != g.ns) ? 1.0 : 0.0;
}

// Matern candidate tile, per 32-column chunk: every off-diagonal element inside the chunk is
// interpolated from the workgroup's Chebyshev table (cheb_eval); the few outside it (x = phi d
// < 0.5, or beyond the table) are compacted into a list by wave ballots and evaluated exactly
// afterwards, densely (an exact K_nu costs ~20x an interpolation: left in place, one such element
// would hold up its whole wave).  Results go through LDS and leave as the exponential path's
// 16-byte row-pair stores.
#define MK_MT_COLS 32
__device__ inline void matern_tile(const CandGen& g, const double* chtab, int ni, double* M, long ld, int ti, int tj,
                                   double* buf, unsigned short* idx, int* cnt) {
  const int tid = threadIdx.x, lane = tid & 63;
  constexpr int CH = MK_NB * MK_MT_COLS;   // elements per chunk
  constexpr int NJ = CH / 256;
  for (int c0 = 0; c0 < MK_NB; c0 += MK_MT_COLS) {
    if (tid == 0) cnt[0] = 0;
    __syncthreads();
#pragma unroll 2
    for (int j = 0; j < NJ; ++j) {
      const int e = tid + 256 * j;
      const int r = e & (MK_NB - 1), cc = e >> 7;
      const int R = ti * MK_NB + r, C = tj * MK_NB + c0 + cc;
      const bool skip = (ti == tj) && ((R & ~1) + 1 < C);      // pair never stored (upper half)
      bool exact = false;
      double v = 0.0;
      if (!skip) {
        if (R < g.ns && C < g.ns && R != C) {
          const double d = dist2d(g.cx[R], g.cy[R], g.cx[C], g.cy[C]);
          if (!cheb_eval(chtab, ni, d * g.rho.phi, &v)) {
            v = d;                                            // distance; rho applied below
            exact = true;
          }
        } else {
          v = cand_value<MK_COV_MATERN>(g, R, C);             // diagonal, border row, padding
        }
      }
      buf[e] = v;
      const unsigned long long m = __ballot(exact);
      if (m) {
        const int leader = __ffsll((long long)m) - 1;
        int base = 0;
        if (lane == leader) base = atomicAdd(cnt, __popcll(m));
        base = __shfl(base, leader, 64);
        if (exact) idx[base + __popcll(m & ((1ull << lane) - 1ull))] = (unsigned short)e;
      }
    }
    __syncthreads();
    const int n = cnt[0];
    for (int p = tid; p < n; p += 256) {
      const int e = idx[p];
      buf[e] = g.rho(buf[e]);
    }
    __syncthreads();
    const int r2 = 2 * lane;
    for (int cc = tid >> 6; cc < MK_MT_COLS; cc += 4) {
      const int R = ti * MK_NB + r2, C = tj * MK_NB + c0 + cc;
      if (ti == tj && R + 1 < C) continue;
      d2 v;
      v.x = buf[cc * MK_NB + r2];
      v.y = buf[cc * MK_NB + r2 + 1];
      *reinterpret_cast<d2*>(M + R + (long)C * ld) = v;
    }
    __syncthreads();
  }
}

// Matern tables in HBM: one workgroup per (subset, outcome) builds the Chebyshev table of its
// candidate (the same (phi', nu') k_cov_candidate draws) or of its current (phi, nu) (kriging), so
// the tile workgroups of a pair load it (11 KB, from L2) instead of each rebuilding it.
__device__ inline void cheb_build_store(CorrFn rho, double x_hi, double* out) {
  __shared__ double btab[5 * MK_BK_NTAB];
  __shared__ double chtab[MK_CH_NI_MAX * MK_CH_LD];
  __shared__ double vals[MK_CH_NI_MAX * MK_CH_N];
  __shared__ double cosm[MK_CH_N * MK_CH_N];
  rho.fill_tables(btab, threadIdx.x, 256);
  __syncthreads();
  rho.tab = btab;
  const int ni = cheb_count(x_hi);
  cheb_build(rho, ni, chtab, vals, cosm, threadIdx.x, 256);
  for (int i = threadIdx.x; i < ni * MK_CH_LD; i += 256) out[i] = chtab[i];
  if (threadIdx.x == 0) out[MK_CH_NI_MAX * MK_CH_LD] = (double)ni;
}
__global__ __launch_bounds__(256) void k_matern_table(Model md, int h0, int hc, int which, int iter, const int* slist,
                                                      const int* scount) {
  int s, h;
  if (!pick_pair(slist, scount, blockIdx.x, h0, hc, &s, &h)) return;
  double phi, nu;
  candidate_theta(md, s, h, which & 3, iter, &phi, &nu);
  CorrFn rho;
  rho.init(phi, nu, MK_COV_MATERN);
  cheb_build_store(rho, md.span ? phi * md.span[s] : INFINITY, md.chtab + ((long)s * md.q + h) * MK_CH_TAB);
}
// Load a stored table into LDS (returns the interval count; the caller synchronises).
__device__ inline int cheb_load(const double* src, double* chtab) {
  const int ni = (int)src[MK_CH_NI_MAX * MK_CH_LD];
  for (int i = threadIdx.x; i < ni * MK_CH_LD; i += 256) chtab[i] = src[i];
  return ni;
}

template <int MODEL>
__global__ __launch_bounds__(256) void k_cov_candidate(Model md, MatSet ms, int h0, int hc, int which, int iter,
                                                       const int* slist, const int* scount) {
  const int ntiles = ms.nt * (ms.nt + 1) / 2;
  int e, t, s, h;
  if (!xcd_map(active_pairs(slist, scount, md.S, hc), ntiles, &e, &t) || !pick_pair(slist, scount, e, h0, hc, &s, &h)) return;
  int ti = 0, tj = 0;
  while ((ti + 1) * (ti + 2) / 2 <= t) ++ti;
  tj = t - ti * (ti + 1) / 2;
  const int sh = s * md.q + h;
  CandGen g = make_gen(md, s, h, which & 3, iter);
  if (which & MK_CAND_NOBORDER) g.uh = nullptr;   // lookahead: u is not known yet (k_border_step)
  double* M = mat_slot(ms, sh, 1 - ms.cur[sh]);
  const long ld = ms.ld;
  if (MODEL == MK_COV_MATERN) {
    __shared__ double btab[5 * MK_BK_NTAB];
    __shared__ double buf[MK_NB * MK_MT_COLS];
    __shared__ unsigned short idx[MK_NB * MK_MT_COLS];
    __shared__ int cnt[1];
    __shared__ double chtab[MK_CH_NI_MAX * MK_CH_LD];
    __shared__ double cosm[MK_CH_N * MK_CH_N];
    g.rho.fill_tables(btab, threadIdx.x, 256);
    __syncthreads();
    g.rho.tab = btab;
    // table over [0.5, phi x the subset's extent] (every pair distance is within it): built by
    // k_matern_table for the session's launches, here for the standalone parity entry point
    int ni;
    if (md.chtab) {
      ni = cheb_load(md.chtab + (long)sh * MK_CH_TAB, chtab);
      __syncthreads();
    } else {
      ni = cheb_count(md.span ? g.rho.phi * md.span[s] : INFINITY);
      cheb_build(g.rho, ni, chtab, buf, cosm, threadIdx.x, 256);
    }
    matern_tile(g, chtab, ni, M, ld, ti, tj, buf, idx, cnt);
    return;
  }
  // two rows per lane, 16-byte stores; the upper half of a diagonal tile is never read (the
  // factor kernels read lower tiles only) and is left unwritten
  const int R = ti * MK_NB + (threadIdx.x & 63) * 2;
  if (ti != tj && (ti + 1) * MK_NB <= g.ns) {
    // interior tile (every element a distinct-site pair, no border row or padding): the lane's row
    // coordinates once, no per-element branches -- the same expression as cand_value, so the
    // same bits (measured store floor of this pattern: 0.92 ms at 250 subsets, tools/store_probe)
    const double x0 = g.cx[R], y0 = g.cy[R], x1 = g.cx[R + 1], y1 = g.cy[R + 1];
    const double phi = g.rho.phi;
    for (int cc = threadIdx.x >> 6; cc < MK_NB; cc += 4) {
      const int C = tj * MK_NB + cc;
      const double xc = g.cx[C], yc = g.cy[C];
      d2 v;
      v.x = exp(-phi * dist2d(x0, y0, xc, yc));
      v.y = exp(-phi * dist2d(x1, y1, xc, yc));
      *reinterpret_cast<d2*>(M + R + (long)C * ld) = v;
    }
    return;
  }
  for (int cc = threadIdx.x >> 6; cc < MK_NB; cc += 4) {
    const int C = tj * MK_NB + cc;
    if (ti == tj && R + 1 < C) continue;
    d2 v;
    v.x = cand_value<MODEL>(g, R, C);
    v.y = cand_value<MODEL>(g, R + 1, C);
    *reinterpret_cast<d2*>(M + R + (long)C * ld) = v;
  }
}
template __global__ void k_cov_candidate<MK_COV_EXPONENTIAL>(Model, MatSet, int, int, int, int, const int*, const int*);
template __global__ void k_cov_candidate<MK_COV_MATERN>(Model, MatSet, int, int, int, int, const int*, const int*);

// The bordered row of candidates assembled without it (MK_CAND_NOBORDER): R[n_s][C] = u_h[C], C < n_s,
// the values k_cov_candidate writes with u known -- the sequential schedule assembles the next
// iteration's candidates early, before the A step has produced u (run_iteration, cov_pre).
__global__ __launch_bounds__(256) void k_cand_border(Model md, MatSet ms, int h0, int hc) {
  const int per = (md.n_pad + 255) / 256;
  const int e = blockIdx.x / per, C = (blockIdx.x % per) * 256 + threadIdx.x;
  const int s = e / hc, h = h0 + e % hc;
  if (s >= md.S) return;
  const int ns = md.n_s[s];
  if (C >= ns) return;
  const int sh = s * md.q + h;
  mat_slot(ms, sh, 1 - ms.cur[sh])[ns + (long)C * ms.ld] = md.u[(long)sh * md.n_pad + C];
}

// Plain matrix (no border) loaded by the host for the standalone Cholesky test path.

// ---------------------------------------------------------------- Cholesky
// (Generating C(i,k) from coordinates at its first touch inside this kernel was measured
// slower on cfg3 and its code path made the kernel spill 80 VGPRs: candidates come from
// k_cov_candidate.)
// TM x TN = 128 x 128: one workgroup per 128-tile; 64 x 64 / 32 x 32: four / sixteen per tile
// (small shards: late panels have few tiles and long K), bit-identical (mk_gemm.hpp); sub-tiles
// of the diagonal tile entirely above the diagonal are skipped -- k_chol_diag reads the lower
// triangle only.  (64 x 128 row halves measured slower than 64 x 64 quarters at 32-63 subsets;
// two alternating bulk streams for consecutive columns, no faster than one.)
// Column k, tiles i in [ia, ib), panels j in [j0, j1) (j1 <= k): C(i,k) -= sum_j L(i,j) L(k,j)^T.
// The split schedule (launch_cholesky) runs panels [0, k-1) early on the bulk stream and panel
// k-1 on the critical stream; the accumulator round-trips through fp64 memory between the two,
// so every element sees the same MFMA sequence as one [0, k) launch (same bits).
template <int TM, int TN>
__global__ __launch_bounds__(256, 2) void k_chol_update(MatSet ms, int S, int h0, int hc, int k, int ia, int ib,
                                                       int j0, int j1, const int* slist, const int* scount) {
  extern __shared__ __attribute__((aligned(16))) double lds[];   // gb_lds_bytes(TM, TN) (two DMA stages)
  constexpr int SUBR = MK_NB / TM, SUB = SUBR * (MK_NB / TN);
  const int ntk = ib - ia;
  int e, t, s, h;
  if (!xcd_map(active_pairs(slist, scount, S, hc), ntk * SUB, &e, &t) || !pick_pair(slist, scount, e, h0, hc, &s, &h))
    return;
  const int st = t % SUB;
  t /= SUB;
  const int sr = st % SUBR, sc = st / SUBR;   // (0, 0) when TM = TN = 128
  const int i = ia + t;
  if (i == k && sc * TN >= (sr + 1) * TM) return;   // entirely above the diagonal
  const int sh = s * ms.q + h;
  double* M = mat_slot(ms, sh, 1 - ms.cur[sh]);
  const long ld = ms.ld;
  double* C = M + i * MK_NB + sr * TM + (long)(k * MK_NB + sc * TN) * ld;
  AccT<TM / 32, TN / 32> acc;
  acc_load(acc, C, ld);
  // (Skipping the diagonal tiles' unused upper quadrant -- per MFMA or per chunk -- measured slower.)
  const long jo = (long)j0 * MK_NB * ld;
  gemm_tile<TM, TN, true, true, true>(M + i * MK_NB + sr * TM + jo, ld, M + k * MK_NB + sc * TN + jo, ld,
                                      (j1 - j0) * MK_NB, (j1 - j0) * MK_NB, acc, lds);
  store_tile(C, ld, acc);
}
template __global__ void k_chol_update<128, 128>(MatSet, int, int, int, int, int, int, int, int, const int*, const int*);
template __global__ void k_chol_update<64, 64>(MatSet, int, int, int, int, int, int, int, int, const int*, const int*);
template __global__ void k_chol_update<32, 32>(MatSet, int, int, int, int, int, int, int, int, const int*, const int*);

// TM = 64: the tile's two row halves on two workgroups (in place: each reads and writes its own
// rows only), bit-identical.
// Tiles i in [ia, ib) of panel k (ia > k).
template <int TM>
__global__ __launch_bounds__(256, 2) void k_chol_trsm(MatSet ms, int S, int h0, int hc, int k, int ia, int ib,
                                                     const int* slist, const int* scount) {
  extern __shared__ __attribute__((aligned(16))) double lds[];   // gb_lds_bytes(TM, 128)
  constexpr int SUB = MK_NB / TM;
  const int ntk = ib - ia;
  int e, t, s, h;
  if (!xcd_map(active_pairs(slist, scount, S, hc), ntk * SUB, &e, &t) || !pick_pair(slist, scount, e, h0, hc, &s, &h))
    return;
  const int sr = t % SUB;
  t /= SUB;
  const int i = ia + t;
  const int sh = s * ms.q + h;
  const int slot = 1 - ms.cur[sh];
  double* M = mat_slot(ms, sh, slot);
  const double* W = winv_slot(ms, sh, slot, k);
  const long ld = ms.ld;
  double* C = M + i * MK_NB + sr * TM + (long)k * MK_NB * ld;
  AccT<TM / 32, 4> acc;
  acc_zero(acc);
  // Winv_k lower triangular: (C Winv^T)(m, n) = sum_{j <= n} C(m, j) Winv(n, j)
  gemm_tile<TM, 128, true, true, false, false, false, SKIP_TRI_B>(C, ld, W, MK_NB, MK_NB, MK_NB, acc, lds);
  store_tile(C, ld, acc);
}
template __global__ void k_chol_trsm<128>(MatSet, int, int, int, int, int, int, const int*, const int*);
template __global__ void k_chol_trsm<64>(MatSet, int, int, int, int, int, int, const int*, const int*);
template __global__ void k_chol_trsm<32>(MatSet, int, int, int, int, int, int, const int*, const int*);

// Column k's update with the panel solve in its epilogue (k_chol_update_trsm):
//   jobs t < ntk * 128/TM: rows of tile i = ia + t / (128/TM) (ia = k + 1, TM-row parts):
//     C(i,k) -= sum_{j0 <= j < k} L(i,j) L(k,j)^T (k_chol_update's MFMA sequence, in the row-wave
//     form: wave w holds TM/4 rows of all 128 columns; the accumulator starts from C in memory, so
//     panels [0, j0) may have come from an earlier launch -- the split schedule's bulk stream), then
//     L(i,k) = C(i,k) Winv_k^T straight from the accumulator (k_chol_trsm's sequence: chunks of 16
//     in order from zero, the same fragment values) -- C(i,k) never goes through HBM between the
//     two, and every wave solves its own rows: the same triangular work on all four SIMDs;
//   job t = ntk * 128/TM (extra = 1, sequential schedule): the next diagonal tile's update by
//     panels [0, k), stored partial; its correction by panel k (k_chol_update, accumulator from
//     memory) follows the launch, then its factor.
// Winv_k exists before the launch starts.  Same per-element sequences as U(k), T(k): same bits
// (tests/test_gpu_linalg.py).
// Epilogue: the accumulator's block (bm, c), k-step r is chunk c's A fragment, in registers; the
// output accumulates 32 columns at a time (the kernel stays within the 256 registers of two
// workgroups per CU).
template <int TM>
__global__ __launch_bounds__(256, 2) void k_chol_update_trsm(MatSet ms, int S, int h0, int hc, int k, int ia, int ib,
                                                            int j0, int extra, const int* slist, const int* scount) {
  extern __shared__ __attribute__((aligned(16))) double lds[];   // gb_lds_bytes(128, 128)
  constexpr int SUB = MK_NB / TM, BM = TM / 64;
  const int ntk = ib - ia;
  int e, t, s, h;
  if (!xcd_map(active_pairs(slist, scount, S, hc), ntk * SUB + extra, &e, &t) ||
      !pick_pair(slist, scount, e, h0, hc, &s, &h))
    return;
  const int sh = s * ms.q + h;
  const int slot = 1 - ms.cur[sh];
  double* M = mat_slot(ms, sh, slot);
  const long ld = ms.ld;
  if (t == ntk * SUB) {   // tile (ia, ia) of column ia, panels [0, k)
    double* C = M + ia * MK_NB + (long)ia * MK_NB * ld;
    Acc acc;
    acc_load(acc, C, ld);
    gemm_tile<128, 128, true, true, true>(M + ia * MK_NB, ld, M + ia * MK_NB, ld, k * MK_NB, k * MK_NB, acc, lds);
    store_tile(C, ld, acc);
    return;
  }
  const int i = ia + t / SUB, r0 = i * MK_NB + (t % SUB) * TM;
  double* C = M + r0 + (long)k * MK_NB * ld;
  AccRW<TM> c;
  acc_load_rw<TM>(c, C, ld);
  const long jo = (long)j0 * MK_NB * ld;
  gemm_tile_rw<TM, true>(M + r0 + jo, ld, M + k * MK_NB + jo, ld, (k - j0) * MK_NB, c, lds);   // ends with a barrier
  // opaque copies: the output addresses are computed here, not hoisted over the main loop beside
  // the accumulator (the compiler would otherwise keep acc_load's addresses live for the stores)
  double* Co = C;
  long ldo = ld;
  asm volatile("" : "+s"(Co), "+s"(ldo));
  const double* Wt = winv_slot(ms, sh, slot, k);   // op(B)(j, n) = Wt[j * 128 + n]
  asm volatile("" : "+s"(Wt));
  // four passes of 32 output columns, P = 3, 0, 2, 1 (pass P: n-blocks 2P, 2P+1, chunks 0 .. 2P+1);
  // each pass's 16 x 32 slices of Winv_k^T arrive by LDS-DMA while the previous pass multiplies
  // (buffers: passes 3, 2 at lds, passes 0, 1 behind pass 3's 48 KiB)
  constexpr int IMG = gb_img(32);
  auto issue = [&](int P, double* buf) {   // a rolled loop: one chunk's addresses live at a time
#pragma nounroll
    for (int ch = 0; ch < 2 * P + 2; ++ch) dma_chunk<true, 32>(Wt + 32 * P, MK_NB, GB_K * ch, buf + ch * IMG);
  };
  double* bufA = lds;
  double* bufB = lds + 8 * IMG;
  issue(3, bufA);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int idx = 0; idx < 4; ++idx) {
    const int P = idx == 0 ? 3 : (idx == 1 ? 0 : (idx == 2 ? 2 : 1));
    const double* buf = (idx & 1) ? bufB : bufA;
    if (idx < 3) {
      const int Pn = idx == 0 ? 0 : (idx == 1 ? 2 : 1);
      issue(Pn, (idx & 1) ? bufA : bufB);
    }
    AccT<BM, 2> o;
    acc_zero(o);
#pragma unroll
    for (int ch = 0; ch < 8; ++ch) {
      if (ch >= 2 * P + 2) break;
#pragma unroll
      for (int ks = 0; ks < GB_K / 4; ++ks) {
        const int kk = ks * 4 + lk;
        double xb[2];
#pragma unroll
        for (int b = 0; b < 2; ++b) xb[b] = frag<true, 32>(buf + ch * IMG, b * 16 + li, kk);
#pragma unroll
        for (int bm = 0; bm < BM; ++bm)
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            if (ch > 2 * P + b) continue;   // Winv(n, j) = 0 for j > n (k_chol_trsm's SKIP_TRI_B)
            o.v[bm][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(xb[b], c.v[bm][ch][ks], o.v[bm][b], 0, 0, 0);
          }
      }
    }
#pragma unroll
    for (int bm = 0; bm < BM; ++bm)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) Co[rw_row<TM>(bm) + (long)rw_col(2 * P + b, r) * ldo] = o.v[bm][b][r];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
}
template __global__ void k_chol_update_trsm<128>(MatSet, int, int, int, int, int, int, int, int, const int*, const int*);
template __global__ void k_chol_update_trsm<64>(MatSet, int, int, int, int, int, int, int, int, const int*, const int*);

// ---------------------------------------------------------------- diagonal tile: factor + invert in LDS
// 128x128 tile T (column-major, stride TLD) in LDS, 256 threads, blocked by 16 (see
// factor_invert_tile): F1 factor + invert of the 16x16 pivot in one wave's registers, F2 panel
// P = C Dinv^T, F3 trailing update T -= P P^T, inverse block rows X_pc = -Dinv_p sum L_pK X_Kc
// (MFMA 16x16x4 on LDS operands).
// Odd LDS column stride: lanes walking a row (the transposed inverse, column-index accesses)
// hit distinct banks instead of one (stride 128 doubles = 0 mod 64 banks).
#define TLD MK_TLD
#define SLD 17
#ifdef MK_DIAG_TIMING   // development probe only (tools/diag_probe.hip): shader-clock stamps per phase
__device__ long long* mk_diag_ts;
#define MK_TSTAMP(i) do { if (threadIdx.x == 0) mk_diag_ts[blockIdx.x * 128 + (i)] = clock64(); } while (0)
#define MK_TSTAMPW(i, t) do { if (threadIdx.x == (t)) mk_diag_ts[blockIdx.x * 128 + (i)] = clock64(); } while (0)
#else
#define MK_TSTAMP(i) do { } while (0)
#define MK_TSTAMPW(i, t) do { } while (0)
#endif     // wave-private 16 x 16 staging, padded likewise

__device__ inline double rlane(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// D(16x16) += sum_k A(i,k) B(k,j); lane l, reg r holds D[(l>>4) + 4r][l&15].  K is a
// multiple of 16: the operands of four MFMAs are loaded together (LDS latency paid once per 4).
template <class FA, class FB>
__device__ inline d4 mfma16(d4 acc, int K, FA fa, FB fb) {
  const int l = threadIdx.x & 63;
  for (int k0 = 0; k0 < K; k0 += 16) {
    double a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a[u] = fa(l & 15, k0 + 4 * u + (l >> 4));
      b[u] = fb(k0 + 4 * u + (l >> 4), l & 15);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u], b[u], acc, 0, 0, 0);
  }
  return acc;
}

// Value of lane n of this lane's 16-lane DPP row (row_newbcast:n, one v_mov_b64_dpp).
template <int N>
__device__ inline double bcast16_t(double v) { return __builtin_amdgcn_update_dpp(v, v, 0x150 + N, 0xf, 0xf, false); }
__device__ __forceinline__ double bcast16(double v, int n) {
  switch (n) {
    case 0: return bcast16_t<0>(v);   case 1: return bcast16_t<1>(v);   case 2: return bcast16_t<2>(v);
    case 3: return bcast16_t<3>(v);   case 4: return bcast16_t<4>(v);   case 5: return bcast16_t<5>(v);
    case 6: return bcast16_t<6>(v);   case 7: return bcast16_t<7>(v);   case 8: return bcast16_t<8>(v);
    case 9: return bcast16_t<9>(v);   case 10: return bcast16_t<10>(v); case 11: return bcast16_t<11>(v);
    case 12: return bcast16_t<12>(v); case 13: return bcast16_t<13>(v); case 14: return bcast16_t<14>(v);
    default: return bcast16_t<15>(v);
  }
}

// d = sqrt(a) and inv = 1/d from the hardware rsq estimate: two Newton steps on 1/sqrt(a), a
// residual-corrected square root and one Newton step on the reciprocal (both within 1 ulp).
__device__ inline void rsqrt_sqrt(double a, double* d, double* inv) {
  double y = __builtin_amdgcn_rsq(a);
  double e = fma(-a * y, y, 1.0);
  y = fma(0.5 * y, e, y);
  e = fma(-a * y, y, 1.0);
  y = fma(0.5 * y, e, y);
  const double d0 = a * y;
  const double r = fma(-d0, d0, a);
  const double dd = fma(r, 0.5 * y, d0);
  *d = dd;
  *inv = fma(y, fma(-dd, y, 1.0), y);
}

// X[r][c] of the inverse: stored transposed in the upper triangle, diagonal included
// (T[r + r*TLD] holds X[r][r] once its pivot block is done); zero above the diagonal.  The
// load is unconditional (always in bounds) and the mask a select: no per-element branch.
__device__ inline double xget(const double* T, int r, int c) {
  const double v = T[c + r * TLD];
  return (r >= c) ? v : 0.0;
}

// acc += (lane n's value of src within this lane's 16-lane DPP row) * mul: one v_fmac_f64 with a
// 64-bit row_newbcast DPP source (the compiler keeps v_mov_b64_dpp + v_fma_f64 apart, plus a copy
// for the old value: three instructions per element).  The asm is volatile, so the calls keep
// their program order; a DPP read needs two wait states after a VALU write of its source, which
// the callers give with NOP = true on the first call after such a write (the compiler does not
// see inside the asm).  SELF: the source is acc itself (one register, no copy the compiler could
// place right before the read).
#define MK_FMAC_BC(N)                                                                                   \
  do {                                                                                                  \
    if (SELF) {                                                                                         \
      if (NOP) asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %0, %1 row_newbcast:" #N " row_mask:0xf bank_mask:0xf" \
                            : "+v"(acc) : "v"(mul));                                                      \
      else asm volatile("v_fmac_f64_dpp %0, %0, %1 row_newbcast:" #N " row_mask:0xf bank_mask:0xf"        \
                        : "+v"(acc) : "v"(mul));                                                          \
    } else {                                                                                            \
      if (NOP) asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:" #N " row_mask:0xf bank_mask:0xf" \
                            : "+v"(acc) : "v"(src), "v"(mul));                                            \
      else asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:" #N " row_mask:0xf bank_mask:0xf"        \
                        : "+v"(acc) : "v"(src), "v"(mul));                                                \
    }                                                                                                   \
  } while (0)
template <bool NOP, bool SELF>
__device__ __forceinline__ void fmac_bc16(double& acc, double src, double mul, int n) {
  switch (n) {
    case 0: MK_FMAC_BC(0); break;   case 1: MK_FMAC_BC(1); break;   case 2: MK_FMAC_BC(2); break;
    case 3: MK_FMAC_BC(3); break;   case 4: MK_FMAC_BC(4); break;   case 5: MK_FMAC_BC(5); break;
    case 6: MK_FMAC_BC(6); break;   case 7: MK_FMAC_BC(7); break;   case 8: MK_FMAC_BC(8); break;
    case 9: MK_FMAC_BC(9); break;   case 10: MK_FMAC_BC(10); break; case 11: MK_FMAC_BC(11); break;
    case 12: MK_FMAC_BC(12); break; case 13: MK_FMAC_BC(13); break; case 14: MK_FMAC_BC(14); break;
    default: MK_FMAC_BC(15); break;
  }
}
#undef MK_FMAC_BC


// Pivot block p: factor the 16x16 block in registers of one wave and invert it (F1).  Lane l holds
// row (l & 15); in the factor lanes 16..63 mirror lanes 0..15 (same instructions, results unused),
// in the inverse each 16-lane row group owns a quarter of the columns.  Column values are broadcast
// by 64-bit DPP row_newbcast.  The pivot is issue-bound (~1,500 wave instructions, ~10k cycles per
// block before round 3's rework; 5.2k now, tools/lat_probe.hip), so every broadcast-multiply-add is
// one fused DPP instruction (fmac_bc16) -- the same fma, operands and order, so the same bits.
// Branch-free: the bordered row is a select and its pivot is stored after the loop; upper-triangle
// entries are updated unconditionally and never read.
__device__ inline void factor_pivot(double* T, double* dg, double* xd, int b, int rb, double* quad_out, bool& bad) {
  const int l = threadIdx.x & 63;
  // lr opaque to the compiler, so the ~50 lane masks (lr == j, lr > m, ...) are formed where they
  // are used instead of being hoisted out of the pivot-step loop and spilled to VGPR lanes
  int lr = l & 15;
  asm volatile("" : "+v"(lr));
  double row[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) row[c] = T[(b + lr) + (b + c) * TLD];
  double myinv = 0.0;   // 1 / L(lr, lr)
  double qv = 0.0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const double a = bcast16(row[j], j);
    const bool border = (b + j == rb);
    double d, inv;
    rsqrt_sqrt(a, &d, &inv);
    bad |= !border && !(a > 0.0);
    qv = border ? -a : qv;
    d = border ? 1.0 : d;
    inv = border ? 1.0 : inv;
    myinv = (lr == j) ? inv : myinv;
    row[j] = (lr == j) ? d : row[j] * inv;
    const double nrj = -row[j];
#pragma unroll
    for (int c = j + 1; c < 16; ++c) {
      // row[j] was written just above (first call waits); the later calls read it again
      if (c == j + 1) fmac_bc16<true, false>(row[c], row[j], nrj, c);
      else fmac_bc16<false, false>(row[c], row[j], nrj, c);
    }
  }
  if (l == 0 && rb >= b && rb < b + 16) *quad_out = qv;
  // inverse of the pivot block, row lr of Dinv in xr: with the row-scaled factor
  // Ls(l, m) = L(l, m) / L(l, l),  X(l, c) = [l == c] / L(l, l) - sum_{c <= m < l} Ls(l, m) X(m, c)
  // The four 16-lane row groups split the inverse's columns: group g = l >> 4 keeps X(lr, c) for
  // c = 4i + g in xr[i] (every broadcast it needs, X(m, c) at lane m, lives in its own row), so a
  // step issues ceil((m+1)/4) fused fmacs instead of m+1.  Columns past m in some groups take a zero
  // multiplier (adds an exact zero).  Each element sees the same fmas as one row per lane: same bits.
  const int g = l >> 4;
  double xr[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) xr[i] = (4 * i + g == lr) ? myinv : 0.0;
#pragma unroll
  for (int m = 0; m < 15; ++m) {
    const double ncf = (lr > m) ? -(row[m] * myinv) : -0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (4 * i <= m) {
        const double mi = (4 * i + g <= m) ? ncf : 0.0;
        fmac_bc16<true, true>(xr[i], xr[i], mi, m);   // xr[i] was written one or a few calls earlier
      }
    }
  }
  // X out, all 64 lanes (row lr, columns 4i + g): strictly lower transposed, the diagonal in place
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = 4 * i + g;
    if (c < lr) T[(b + c) + (b + lr) * TLD] = xr[i];
    if (c == lr) {
      xd[b + lr] = xr[i];
      T[(b + lr) + (b + lr) * TLD] = xr[i];   // X diagonal in place (the L diagonal lives in dg)
    }
  }
  if (l < 16) {
#pragma unroll
    for (int c = 0; c < 16; ++c)
      if (c < l) T[(b + l) + (b + c) * TLD] = row[c];
    dg[b + l] = row[l];
  }
}

// Trailing block index u (0 = (p, p)) of step p-1 -> (row, column) block offsets from p.
__device__ inline void trail_rc(int u, int* R, int* C) {
  int r = 0;
  while ((r + 1) * (r + 2) / 2 <= u) ++r;
  *R = r;
  *C = u - r * (r + 1) / 2;
}

// Phase-1 work of waves 1-3, software-pipelined: the three waves share the CU's LDS, and with their
// reads issued just before the MFMAs that consume them the tasks ran ~3x slower than one wave alone
// (LDS contention exposed on every group).  Each group's reads are now issued before the previous
// group's MFMAs (64 cycles each on the SIMD's matrix pipe), which hide them.  Same operands, same
// MFMA order per block: same bits.
// f64 MFMA modifier (the blgp operand of the f64 forms): negate the A operand, neg:[1,0,0] -- a
// negated fragment then needs no VALU pass between its LDS read and the MFMA.
#define MK_MFMA_NEG_A 1
struct TrailGrp {
  d4 a[4];
  double x[4][4], y[4][4];
  int R[4], C[4];
  int n;
};

// Group of up to four trailing blocks of step p-1 from this wave's tasks t, t+3, ... < ntask (task t
// = block u = t - p + 1); issues its LDS reads.
__device__ __forceinline__ void trail_load(const double* T, int p, int t, int ntask, TrailGrp& g) {
  const int l = threadIdx.x & 63, bc = 16 * (p - 1);
  g.n = t < ntask ? min(4, (ntask - t + 2) / 3) : 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (q < g.n) {
      int R, C;
      trail_rc(t + 3 * q - p + 1, &R, &C);
      R += p;
      C += p;
      g.R[q] = R;
      g.C[q] = C;
#pragma unroll
      for (int r = 0; r < 4; ++r) g.a[q][r] = T[(16 * R + (l >> 4) + 4 * r) + (16 * C + (l & 15)) * TLD];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = 4 * u + (l >> 4);
        g.x[q][u] = T[(16 * R + (l & 15)) + (bc + k) * TLD];   // negated by the MFMA (neg A)
        g.y[q][u] = T[(16 * C + (l & 15)) + (bc + k) * TLD];
      }
    }
  }
}

__device__ __forceinline__ void trail_mma_store(double* T, TrailGrp& g) {
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (q < g.n) g.a[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(g.x[q][u], g.y[q][u], g.a[q], 0, 0, MK_MFMA_NEG_A);
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (q < g.n) {
#pragma unroll
      for (int r = 0; r < 4; ++r) T[(16 * g.R[q] + (l >> 4) + 4 * r) + (16 * g.C[q] + (l & 15)) * TLD] = g.a[q][r];
    }
}

// This wave's trailing blocks (tasks t, t+3, ... < ntask), groups of four, double-buffered.
__device__ __forceinline__ void trail_tasks(double* T, int p, int t, int ntask) {
  TrailGrp g0, g1;
  trail_load(T, p, t, ntask, g0);
  t += 3 * g0.n;
  while (g0.n) {
    trail_load(T, p, t, ntask, g1);
    t += 3 * g1.n;
    trail_mma_store(T, g0);
    if (!g1.n) break;
    trail_load(T, p, t, ntask, g0);
    t += 3 * g0.n;
    trail_mma_store(T, g1);
  }
}

// S_pc = sum_{K=c}^{p-1} L_pK X_Kc into Sb, one 16-deep chunk per K, each chunk's reads issued before
// the previous chunk's MFMAs.  (mfma16's operands and order: same bits.)
__device__ __forceinline__ void s_task(const double* T, double* Sb, int p, int c) {
  const int l = threadIdx.x & 63;
  double a0[4], b0[4], a1[4], b1[4];
  // X_Kc: only the diagonal block (K = c) needs xget's mask; below it every entry is r > c
  auto ld = [&](int K, double* a, double* b) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int m = 4 * u + (l >> 4);
      a[u] = T[(16 * p + (l & 15)) + (16 * K + m) * TLD];
      b[u] = (K == c) ? xget(T, 16 * K + m, 16 * c + (l & 15)) : T[(16 * c + (l & 15)) + (16 * K + m) * TLD];
    }
  };
  d4 acc = {0.0, 0.0, 0.0, 0.0};
  ld(c, a0, b0);
  for (int K = c; K < p; K += 2) {
    if (K + 1 < p) ld(K + 1, a1, b1);
#pragma unroll
    for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a0[u], b0[u], acc, 0, 0, 0);
    if (K + 1 >= p) break;
    if (K + 2 < p) ld(K + 2, a0, b0);
#pragma unroll
    for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a1[u], b1[u], acc, 0, 0, 0);
  }
  double* S = Sb + c * 16 * SLD;
#pragma unroll
  for (int r = 0; r < 4; ++r) S[((l >> 4) + 4 * r) + (l & 15) * SLD] = acc[r];
}

// F3 block (RR, CC) of the trailing update after pivot column block pc: T_RC -= P_R P_C^T.
__device__ inline void trailing_block(double* T, int pc, int RR, int CC) {
  const int l = threadIdx.x & 63, bc = 16 * pc;
  d4 acc;
#pragma unroll
  for (int r = 0; r < 4; ++r) acc[r] = T[(16 * RR + (l >> 4) + 4 * r) + (16 * CC + (l & 15)) * TLD];
  acc = mfma16(acc, 16, [&](int i, int k) { return -T[(16 * RR + i) + (bc + k) * TLD]; },
               [&](int k, int j) { return T[(16 * CC + j) + (bc + k) * TLD]; });
#pragma unroll
  for (int r = 0; r < 4; ++r) T[(16 * RR + (l >> 4) + 4 * r) + (16 * CC + (l & 15)) * TLD] = acc[r];
}

// L (its diagonal from dg) into Mt and X = Winv_k into W, as 16-byte row pairs (rows r, r+1 of
// column c), all 256 threads, eight pairs per thread in flight (every LDS read of a batch issued
// before its stores: the loop was latency-bound at ~450 cycles per pair otherwise).  Pairs entirely
// above the diagonal are not stored -- the Winv slots are zeroed once when the session is created
// and never written there, and M's upper triangle is never read -- and the one upper element of a
// pair that straddles the diagonal gets a zero in both.
__device__ inline void store_tile_lw(const double* T, const double* dg, const double* xd, double* Mt, long ld,
                                     double* W) {
  constexpr int B = 8;
  const int tid = threadIdx.x;
#pragma unroll 1
  for (int e0 = 0; e0 < MK_NB * (MK_NB / 2); e0 += 256 * B) {
    // every read of the batch unconditional and issued before any use (the memory clobber keeps
    // the compiler from sinking them into per-select branches, one LDS round trip each)
    d2 lr2[B], wr2[B], dd[B], xx[B];
#pragma unroll
    for (int u = 0; u < B; ++u) {
      const int e = e0 + tid + 256 * u;
      const int c = e >> 6, r = 2 * (e & 63);
      lr2[u].x = T[r + c * TLD];
      lr2[u].y = T[r + 1 + c * TLD];
      wr2[u].x = T[c + r * TLD];
      wr2[u].y = T[c + (r + 1) * TLD];
      dd[u] = *reinterpret_cast<const d2*>(dg + r);
      xx[u] = *reinterpret_cast<const d2*>(xd + r);
    }
    asm volatile("" ::: "memory");
#pragma unroll
    for (int u = 0; u < B; ++u) {
      const int e = e0 + tid + 256 * u;
      const int c = e >> 6, r = 2 * (e & 63);
      d2 lv, wv;
      lv.x = (r > c) ? lr2[u].x : ((r == c) ? dd[u].x : 0.0);
      lv.y = (r + 1 > c) ? lr2[u].y : dd[u].y;
      wv.x = (r > c) ? wr2[u].x : ((r == c) ? xx[u].x : 0.0);
      wv.y = (r + 1 > c) ? wr2[u].y : xx[u].y;
      if (r + 1 >= c) {
        *reinterpret_cast<d2*>(Mt + r + (long)c * ld) = lv;
        *reinterpret_cast<d2*>(W + r + c * MK_NB) = wv;
      }
    }
  }
}

// Blocked by 16, two barriers per pivot step p, the inverse X = L^-1 computed by block rows
// alongside the factorisation (block row p of X needs L(p, <p) and X(<p, <p) only):
//   phase 1  wave 0: trailing block (p, p) of step p-1, then F1 (factor + invert the pivot);
//            waves 1-3: the other trailing blocks of step p-1, and S_pc = sum_{c<=K<p} L_pK X_Kc
//            for every c < p (staged in LDS);
//   phase 2  F2: panel P_R = C_R Dinv_p^T (R > p), and X_pc = -Dinv_p S_pc (c < p).
// Storage: L in the lower triangle; X strictly-lower transposed into the upper triangle
// (X[r][c] at T[c + r*TLD]); diag(L) in dg, diag(X) in xd; S stagings in Sb (7 x 16 x SLD).
__device__ void factor_invert_tile(double* T, double* dg, double* xd, double* Sb, int rb, double* quad_out,
                                   bool* bad_out) {
  // wv through readfirstlane: the task indices derived from it are wave-uniform scalars (in VGPRs the
  // compiler treated them as divergent: exec-masked MFMAs and full MFMA-drain waits around each one)
  const int tid = threadIdx.x, l = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  bool bad = false;
  for (int p = 0; p < 8; ++p) {
    // ---- phase 1
    const int nb = 8 - p;                       // trailing blocks of step p-1: rows/cols p..7
    const int ntrail = (p > 0) ? nb * (nb + 1) / 2 : 0;
    if (wv == 0) {
      // (block (p, p)'s update by step p-1 was done by this wave at the end of step p-1)
      MK_TSTAMPW(44 + 4 * p, 0);
      factor_pivot(T, dg, xd, 16 * p, rb, quad_out, bad);
      MK_TSTAMPW(45 + 4 * p, 0);
    } else {
      // tasks t (dealt round-robin over the three waves): S_pc for t < p (c = t, longest first),
      // then trailing blocks u = t - p + 1 = 1 .. ntrail-1
      const int ntask = p + ntrail - 1;
      MK_TSTAMPW(96 + p, 64);
      int t = wv - 1;
      for (; t < p; t += 3) s_task(T, Sb, p, t);
      MK_TSTAMPW(47 + 4 * p, 64);
      trail_tasks(T, p, t, ntask);
      MK_TSTAMPW(46 + 4 * p, 64);
      MK_TSTAMPW(80 + p, 128);
      MK_TSTAMPW(88 + p, 192);
    }
    __syncthreads();
    MK_TSTAMP(1 + 3 * p);
    // ---- phase 2: F2 panel blocks R = p+1..7, inverse blocks X_pc, c = 0..p-1 (tasks t < 7).
    // Wave 0 takes panel block p+1 and then the next pivot block's trailing update T_{p+1,p+1} -=
    // P_{p+1} P_{p+1}^T right away (the next pivot's only input from this step), so its phase 1
    // starts with the pivot; waves 1-3 take the other tasks.
    const int b = 16 * p;
    auto task = [&](int t) {
      if (t < 7 - p) {
        const int R = p + 1 + t;
        d4 acc = {0.0, 0.0, 0.0, 0.0};
        acc = mfma16(acc, 16, [&](int i, int k) { return T[(16 * R + i) + (b + k) * TLD]; },
                     [&](int k, int j) { return xget(T, b + j, b + k); });
#pragma unroll
        for (int r = 0; r < 4; ++r) T[(16 * R + (l >> 4) + 4 * r) + (b + (l & 15)) * TLD] = acc[r];
      } else {
        const int Cb = t - (7 - p);
        const double* S = Sb + Cb * 16 * SLD;
        d4 out = {0.0, 0.0, 0.0, 0.0};
        out = mfma16(out, 16, [&](int r, int m) { return -xget(T, b + r, b + m); },
                     [&](int m, int c) { return S[m + c * SLD]; });
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rr = b + (l >> 4) + 4 * r, cc = 16 * Cb + (l & 15);
          T[cc + rr * TLD] = out[r];
        }
      }
    };
    if (wv == 0) {
      task(0);
      if (p < 7) {
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        trailing_block(T, p, p + 1, p + 1);
      }
    } else {
      for (int t = wv; t < 7; t += 3) task(t);
    }
    __syncthreads();
    MK_TSTAMP(2 + 3 * p);
  }
  if (l == 0 && wv == 0) *bad_out = bad;
}

// Factor + invert the 128x128 diagonal tile k of each candidate.  Row rb = n_s - 128k
// (if inside the tile) is the bordered row: its pivot is -(u' R^-1 u) and it is not
// factored (pivot set to 1).
// cj0 < cj1 (the fused factorisation, launch_cholesky): the tile first takes its update by panels
// [cj0, cj1) -- k_chol_update's MFMA sequence from the tile in memory, the accumulator written
// straight into the LDS image instead of back to HBM (the launch it replaces would have stored
// exactly these values) -- then factors.
__global__ __launch_bounds__(256) void k_chol_diag(MatSet ms, const int* __restrict__ n_s, int h0, int hc, int k,
                                                   double* ld_part, double* quad_c, int* info, const int* slist,
                                                   const int* scount, int cj0, int cj1) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double* T = sm;                      // [128*128]
  double* dg = T + MK_NB * TLD;        // [128]
  double* xd = dg + MK_NB;             // [128]
  double* Sb = xd + MK_NB;             // [7][16 * SLD]
  int s, h;
  if (!pick_pair(slist, scount, blockIdx.x, h0, hc, &s, &h)) return;
  MK_TSTAMP(0);
  const int tid = threadIdx.x;
  const int sh = s * ms.q + h;
  const int slot = 1 - ms.cur[sh];
  double* M = mat_slot(ms, sh, slot);
  const long ld = ms.ld;
  const int base = k * MK_NB;
  const int ns = n_s[s];
  double* Mt = M + base + (long)base * ld;
  if (cj1 > cj0) {
    Acc acc;
    acc_load(acc, Mt, ld);
    const long jo = (long)cj0 * MK_NB * ld;
    gemm_tile<128, 128, true, true, true>(M + base + jo, ld, M + base + jo, ld, (cj1 - cj0) * MK_NB,
                                          (cj1 - cj0) * MK_NB, acc, sm);   // stages in T's space; ends with a barrier
#pragma unroll
    for (int bm = 0; bm < 4; ++bm)
#pragma unroll
      for (int bn = 0; bn < 4; ++bn)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rr = acc_row<128>(bm), cc = acc_col<128>(bn, r);
          T[rr + cc * TLD] = rr >= cc ? acc.v[bm][bn][r] : 0.0;
        }
  } else {
  // Unconditional 16-byte loads, all 32 per thread in flight at once (one memory round trip
  // instead of four), then the upper triangle is zeroed in LDS (a masked load per element
  // compiled to one dependent round trip each: 64 per thread).
    constexpr int NL = MK_NB * MK_NB / (256 * 2);
    d2 v[NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int e = 2 * (tid + 256 * j);
      v[j] = *reinterpret_cast<const d2*>(Mt + (e & 127) + (long)(e >> 7) * ld);
    }
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int e = 2 * (tid + 256 * j);
      const int r = e & 127, c = e >> 7;
      T[r + c * TLD] = (r >= c) ? v[j].x : 0.0;
      T[r + 1 + c * TLD] = (r + 1 >= c) ? v[j].y : 0.0;
    }
  }
  __syncthreads();
  MK_TSTAMP(40);
  bool bad = false;
  double* W = winv_slot(ms, sh, slot, k);
  factor_invert_tile(T, dg, xd, Sb, ns - base, quad_c + sh, &bad);   // ends with a barrier
  // wave 0: log-det partial and the factorisation flag (the pivot ran on wave 0; its test is on the
  // broadcast pivot, so every lane's flag is the same), then it joins the stores
  if (tid < 64) {
    double v = 0.0;
    for (int r = tid; r < MK_NB; r += 64) v += (base + r < ns) ? 2.0 * log(dg[r]) : 0.0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (tid == 0) {
      ld_part[(long)sh * ms.nt + k] = v;
      if (bad) info[sh] = 1;
    }
  }
  MK_TSTAMP(41);
  store_tile_lw(T, dg, xd, Mt, ld, W);
  MK_TSTAMP(42);
}

// ---------------------------------------------------------------- inverse (W = L^-1, persistent)
// MK_TRI_SKIP (compile time, default 1): the inverse levels skip the MFMA blocks of their diagonal W
// tiles' zero triangles (SKIP_TRI_A / SKIP_TRI_BL, mk_gemm.hpp: ~15 % of the top level's MFMAs);
// measured 0.570 -> 0.581 of peak over the inverse (profiles/r06/tri_skip).  0 builds the dense form
// (A/B builds only: the same results, the skipped products are exact zeros).
#ifndef MK_TRI_SKIP
#define MK_TRI_SKIP 1
#endif
__device__ inline double* wmat(const MatSet& ms, int sh) { return ms.W + (long)sh * mat_elems(ms); }

// Eight workgroups per 128-tile, each copying one eighth of it (16 rows' worth: 2,048
// doubles) with every load in flight at once: the copy is latency-bound (one tile per workgroup
// took 100-150 us per launch at small shards, on the main stream's critical path).
// MK_CD_SPLIT (mk_types.hpp): workgroups per tile, shared with the launch site's grid.
__global__ __launch_bounds__(256) void k_inv_copydiag(MatSet ms, const int* __restrict__ list, const int* __restrict__ count) {
  const int part = blockIdx.x % MK_CD_SPLIT, rest = blockIdx.x / MK_CD_SPLIT;
  const int e = rest / ms.nt, k = rest % ms.nt;
  if (e >= *count) return;
  const int sh = list[e];
  const double* Wd = winv_slot(ms, sh, ms.cur[sh], k);
  const long ld = ms.ld;
  double* Wt = wmat(ms, sh) + k * MK_NB + (long)k * MK_NB * ld;
  constexpr int PER = MK_NB * MK_NB / MK_CD_SPLIT;   // doubles per workgroup: 16 columns
  const int e0 = part * PER;
  d2 v[PER / 512];
#pragma unroll
  for (int j = 0; j < PER / 512; ++j) v[j] = *reinterpret_cast<const d2*>(Wd + e0 + 2 * (threadIdx.x + 256 * j));
#pragma unroll
  for (int j = 0; j < PER / 512; ++j) {
    const int e2 = e0 + 2 * (threadIdx.x + 256 * j);
    *reinterpret_cast<d2*>(Wt + (e2 & 127) + (long)(e2 >> 7) * ld) = v[j];
  }
}

// Recursive-doubling inverse.  At level sz (sz = 1, 2, 4, ... tiles) every pair of
// consecutive diagonal blocks T = [T0, T0+sz), B = [T0+sz, T0+2sz) of the factor gets
//   phase 0: Y_BT = L_BT W_TT        (Y kept in the free factor slot)
//   phase 1: W_BT = -W_BB Y_BT
// with W_TT, W_BB complete from the lower levels.  Triangularity bounds every K range.
// TM = 64: each 128-tile on four workgroups (small shards), bit-identical.
template <int TM>
__global__ __launch_bounds__(256, 2) void k_inv_level(MatSet ms, const int* __restrict__ list,
                                                      const int* __restrict__ count, int sz, int phase) {
  extern __shared__ __attribute__((aligned(16))) double lds[];   // gb_lds_bytes(TM, TM)
  constexpr int SUBR = MK_NB / TM, SUB = SUBR * SUBR;
  const int npairs = (ms.nt + 2 * sz - 1) / (2 * sz);
  const int per = npairs * sz * sz;
  int e, t;
  if (!xcd_map(*count, per * SUB, &e, &t)) return;
  const int st = t % SUB;
  t /= SUB;
  const int sr = st % SUBR, sc = st / SUBR;
  const int p = t / (sz * sz);
  t %= sz * sz;
  const int T0 = 2 * p * sz, B0 = T0 + sz;
  // consecutive work items share the operand whose K range is the same for all of them:
  // phase 0 a column j (W_TT(j:B0, j)), phase 1 a row i (W_BB(i, B0:i+1))
  const int i = B0 + (phase == 0 ? t % sz : t / sz), j = T0 + (phase == 0 ? t / sz : t % sz);
  if (i >= ms.nt) return;
  const int sh = list[e];
  const int cur = ms.cur[sh];
  const long ld = ms.ld;
  double* Wm = wmat(ms, sh);
  double* Y = ms.Y ? ms.Y + (long)sh * mat_elems(ms) : mat_slot(ms, sh, 1 - cur);
  const int ro = sr * TM;             // sub-tile row / column offsets in the 128-tile
  const long co = (long)sc * TM * ld;
  AccT<TM / 32, TM / 32> acc;
  acc_zero(acc);
  if (phase == 0) {
    const double* Lm = mat_slot(ms, sh, cur);
    const int K = (B0 - j) * MK_NB;
    // K ranges [j, B0) share their end: descending chunks keep the tiles of a subset in step (L2 reuse)
    // W_TT's first K tile is W_jj, lower-triangular in (k, n): its chunk c' feeds column blocks <= c'
    gemm_tile<TM, TM, true, false, false, true, false, MK_TRI_SKIP ? SKIP_TRI_BL : SKIP_NONE>(
        Lm + i * MK_NB + ro + (long)j * MK_NB * ld, ld, Wm + j * MK_NB + (long)j * MK_NB * ld + co, ld, K, K, acc, lds,
        0, ro / 16, sc * TM / 16);
    store_tile(Y + i * MK_NB + ro + (long)j * MK_NB * ld + co, ld, acc);
  } else {
    const int K = (i - B0 + 1) * MK_NB;
    // W_BB's last K tile is W_ii, lower-triangular in (m, k): its chunk c' feeds row blocks >= c'
    gemm_tile<TM, TM, true, false, true, false, false, MK_TRI_SKIP ? SKIP_TRI_A : SKIP_NONE>(
        Wm + i * MK_NB + ro + (long)B0 * MK_NB * ld, ld, Y + B0 * MK_NB + (long)j * MK_NB * ld + co, ld, K, K, acc, lds,
        K - MK_NB, ro / 16, sc * TM / 16);
    store_tile(Wm + i * MK_NB + ro + (long)j * MK_NB * ld + co, ld, acc);
  }
}
template __global__ void k_inv_level<128>(MatSet, const int*, const int*, int, int);
template __global__ void k_inv_level<64>(MatSet, const int*, const int*, int, int);
template __global__ void k_inv_level<32>(MatSet, const int*, const int*, int, int);

// Tiles (i,j), i >= j, of R^-1 = sum over rows l < n_s of W(l,i)^T W(l,j) (drops the bordered
// row and the padding).  diag_only: tiles (i,i) into QB; otherwise the full symmetric Q.
template <bool DIAG>
__device__ inline void wtw_tile(const MatSet& ms, int sh, int ns, int i, int j, Acc& acc, double* lds) {
  const double* X = wmat(ms, sh);
  const long ld = ms.ld;
  const int K = (ms.nt - i) * MK_NB;
  const int kvalid = ns - i * MK_NB;
  acc_zero(acc);
  // DIAG (i == j): both operands are the panel W(i:, i) -- loaded once
  if (kvalid > 0)
    gemm_128<false, false, false, false, DIAG, SKIP_NONE, true>(X + i * MK_NB + (long)i * MK_NB * ld, ld,
                                               X + i * MK_NB + (long)j * MK_NB * ld, ld, K, kvalid, acc, lds);
}

__global__ __launch_bounds__(256, 2) void k_lauum(MatSet ms, const int* __restrict__ n_s, const int* __restrict__ list,
                                               const int* __restrict__ count) {
  extern __shared__ __attribute__((aligned(16))) double lds[];   // MK_GD_LDS_BYTES
  const int ntiles = ms.nt * (ms.nt + 1) / 2;
  const int e = blockIdx.x / ntiles;
  if (e >= *count) return;
  int t = blockIdx.x % ntiles;
  int i = 0;
  while ((i + 1) * (i + 2) / 2 <= t) ++i;
  const int j = t - i * (i + 1) / 2;
  const int sh = list[e];
  Acc acc;
  wtw_tile<false>(ms, sh, n_s[sh / ms.q], i, j, acc, lds);
  const long ld = ms.ld;
  double* Q = ms.Q + (long)sh * mat_elems(ms);
  double* Ct = (i != j) ? Q + j * MK_NB + (long)i * MK_NB * ld : nullptr;
  store_tile(Q + i * MK_NB + (long)j * MK_NB * ld, ld, acc, Ct);
}

// Only the two diagonal 64-quadrants of each 128-tile of R^-1 are consumed (k_sweep reads the
// 64 x 64 block of its 64-site block), so each is one 64-sub-tile workgroup (the same bits as
// the 128-tile product) and the off-diagonal quadrants are never computed.
__global__ __launch_bounds__(256, 2) void k_qblocks(MatSet ms, const int* __restrict__ n_s, const int* __restrict__ list,
                                                 const int* __restrict__ count) {
  extern __shared__ __attribute__((aligned(16))) double lds[];   // gb_lds_bytes(64, 64)
  int e, t;
  if (!xcd_map(*count, ms.nt * 2, &e, &t)) return;
  const int i = t >> 1, sd = t & 1;
  const int sh = list[e];
  const int ns = n_s[sh / ms.q];
  const double* X = wmat(ms, sh);
  const long ld = ms.ld;
  const int K = (ms.nt - i) * MK_NB;
  const int kvalid = ns - i * MK_NB;
  AccT<2, 2> acc;
  acc_zero(acc);
  // both operands are the panel W(i:, 128 i + 64 sd : +64) -- loaded once
  if (kvalid > 0)
    gemm_tile<64, 64, false, false, false, false, true, SKIP_NONE, true>(
        X + i * MK_NB + (long)(i * MK_NB + 64 * sd) * ld, ld, X + i * MK_NB + (long)(i * MK_NB + 64 * sd) * ld, ld,
        K, kvalid, acc, lds);
  store_tile(ms.QB + ((long)sh * ms.nt + i) * MK_NB * MK_NB + 64 * sd + 64 * sd * MK_NB, MK_NB, acc);
}

// z_h = border row of the accepted factor = L^-1 u_h (exact for the u_h the candidate was built with),
// or (lookahead schedule, zc set) the candidate's solved z'_h.
__global__ __launch_bounds__(256) void k_take_border(Model md, MatSet ms, const int* __restrict__ list,
                                                     const int* __restrict__ count, const double* __restrict__ zc) {
  const int per = (md.n_pad + 255) / 256;
  const int e = blockIdx.x / per;
  if (e >= *count) return;
  const int sh = list[e];
  const int s = sh / md.q, h = sh % md.q;
  const int ns = md.n_s[s];
  const int j = (blockIdx.x % per) * 256 + threadIdx.x;
  if (j >= md.n_pad) return;
  const long zo = ((long)s * md.q + h) * md.n_pad + j;
  if (zc) {
    md.z[zo] = (j < ns) ? zc[zo] : 0.0;
    return;
  }
  const double* M = mat_slot(ms, sh, ms.cur[sh]);
  md.z[zo] = (j < ns) ? M[ns + (long)j * ms.ld] : 0.0;
}

// Lookahead schedule, Matern: the nu candidate is factored after the phi decision with its bordered
// row (u is known by then), so where the nu step accepted, z_h is that factor's border row; it
// replaces the phi candidate's solved z'_h in zc (which k_take_border then copies for every
// changed pair).
__global__ __launch_bounds__(256) void k_nu_border(Model md, MatSet ms) {
  const int per = (md.n_pad + 255) / 256;
  const int e = blockIdx.x / per;
  if (e >= md.S * md.q || !md.la_nu[e]) return;
  const int s = e / md.q;
  const int ns = md.n_s[s];
  const int j = (blockIdx.x % per) * 256 + threadIdx.x;
  if (j >= md.n_pad) return;
  const double* M = mat_slot(ms, e, ms.cur[e]);
  md.zc[(long)e * md.n_pad + j] = (j < ns) ? M[ns + (long)j * ms.ld] : 0.0;
}

// ---------------------------------------------------------------- lookahead border solve
// The lookahead schedule (mk_api.hip) factors iteration t+1's phi candidates while iteration t's
// inverse and sweep run, before u_{t+1} = A_{t+1}^-1 w_t exists, so the candidate has no bordered
// row and z'_h = L'_h^-1 u_h comes from a forward solve after the A step, one launch per tile
// column k, each behind the factorisation's panel k (right-looking: every (pair, row tile) reads
// its tile of L' once):
//   z'_k = Winv_k (u_k - acc_k)   (every workgroup of the pair, redundantly; Winv_k from L2)
//   acc_i += L'_ik z'_k           (workgroup t: row tile i = k+1+t; k = nt-1: z' only)
// Lane l holds rows 2l, 2l+1; wave v columns v, v+4, ...; the four waves' partials are added in
// wave order, acc's column sums in k order: deterministic.
__device__ inline d2 gemv_tile(const double* A, long lda, const double* x, double* red) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  d2 acc = {0.0, 0.0};
  const double* Ar = A + 2 * lane;
#pragma unroll 2
  for (int j0 = 0; j0 < 32; j0 += 8) {
    d2 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = *reinterpret_cast<const d2*>(Ar + (long)(wv + 4 * (j0 + j)) * lda);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const double xc = x[wv + 4 * (j0 + j)];
      acc.x = fma(v[j].x, xc, acc.x);
      acc.y = fma(v[j].y, xc, acc.y);
    }
  }
  red[wv * MK_NB + 2 * lane] = acc.x;
  red[wv * MK_NB + 2 * lane + 1] = acc.y;
  __syncthreads();
  d2 out;
  out.x = ((red[2 * lane] + red[MK_NB + 2 * lane]) + red[2 * MK_NB + 2 * lane]) + red[3 * MK_NB + 2 * lane];
  out.y = ((red[2 * lane + 1] + red[MK_NB + 2 * lane + 1]) + red[2 * MK_NB + 2 * lane + 1]) + red[3 * MK_NB + 2 * lane + 1];
  return out;   // meaningful in every wave (each reads the same sums)
}

__global__ __launch_bounds__(256) void k_border_step(Model md, MatSet ms, int k) {
  __shared__ double xs[MK_NB];
  __shared__ double red[4 * MK_NB];
  const int nt = ms.nt, T = max(1, nt - 1 - k);
  int e, t;
  if (!xcd_map(md.S * md.q, T, &e, &t)) return;
  const int s = e / md.q;
  const int ns = md.n_s[s];
  const int i = k + 1 + t;
  if (k * MK_NB >= ns) return;                          // z'_k = 0 (rows beyond the subset; never read)
  const bool acc_work = k < nt - 1 && i * MK_NB < ns;   // tile i holds sites: accumulate into it
  if (t > 0 && !acc_work) return;                       // (workgroup 0 always writes z'_k)
  const int slot = 1 - ms.cur[e];
  const long np = md.n_pad;
  const double* u = md.u + (long)e * np;                // [S][q][n_pad]: pair e = s*q + h
  double* zc = md.zc + (long)e * np;
  double* bacc = md.bacc + (long)e * np;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid < MK_NB) {
    const int row = k * MK_NB + tid;
    xs[tid] = (row < ns) ? u[row] - (k > 0 ? bacc[row] : 0.0) : 0.0;
  }
  __syncthreads();
  d2 y = gemv_tile(winv_slot(ms, e, slot, k), MK_NB, xs, red);
  const int row = k * MK_NB + 2 * lane;
  y.x = (row < ns) ? y.x : 0.0;
  y.y = (row + 1 < ns) ? y.y : 0.0;
  __syncthreads();                                      // every wave has read red and xs
  if (wv == 0) {
    xs[2 * lane] = y.x;
    xs[2 * lane + 1] = y.y;
    if (t == 0) *reinterpret_cast<d2*>(zc + row) = y;
  }
  __syncthreads();
  if (!acc_work) return;
  const d2 p = gemv_tile(mat_slot(ms, e, slot) + i * MK_NB + (long)k * MK_NB * ms.ld, ms.ld, xs, red);
  if (wv == 0) {
    d2* ap = reinterpret_cast<d2*>(bacc + i * MK_NB + 2 * lane);
    d2 v = p;
    if (k > 0) {
      const d2 o = *ap;
      v.x = o.x + v.x;
      v.y = o.y + v.y;
    }
    *ap = v;
  }
}

// quad_c = |z'_h|^2 (rows < n_s) for every pair: the candidate's u' R'^-1 u.
__global__ __launch_bounds__(256) void k_border_quad(Model md) {
  __shared__ double red[8];
  const int e = blockIdx.x, s = e / md.q;
  const int ns = md.n_s[s];
  const double* zc = md.zc + (long)e * md.n_pad;
  double loc = 0.0;
  for (int r = threadIdx.x; r < ns; r += 256) loc += zc[r] * zc[r];
  const double tot = block_sum<256>(loc, red);
  if (threadIdx.x == 0) md.quad_c[e] = tot;
}

// Z_{h,c} = W_h u_c for every subset, outcome h and c (q > 1, start of the A phase).
// Thread = row r of W_h (coalesced column walks); the q vectors u_c are staged in LDS per
// 512-column chunk (one broadcast read per column instead of q global loads), the column loop
// is unrolled by 8 with its loads issued together, and the q accumulators are indexed at
// compile time (loops over MK_QMAX, q-guarded: no scratch).
#define MK_ZCH 512
__global__ __launch_bounds__(256) void k_trmv_Z(Model md, MatSet ms) {
  __shared__ double us[MK_QMAX][MK_ZCH];
  const int per = (md.n_pad + 255) / 256;
  const int sh = blockIdx.x / per;
  const int s = sh / md.q, h = sh % md.q;
  const int ns = md.n_s[s];
  const int r0 = (blockIdx.x % per) * 256, r = r0 + threadIdx.x;
  const double* Wm = wmat(ms, sh) + r;
  const long ld = ms.ld;
  const int q = md.q;
  const double* u = md.u + (long)s * q * md.n_pad;
  double acc[MK_QMAX] = {0.0, 0.0, 0.0, 0.0};
  const int jmax = (r < md.n_pad) ? min(r + 1, ns) : 0;            // this row's columns
  const int jblk = min(min(r0 + 256, md.n_pad), ns);              // the block's widest row
  for (int j0 = 0; j0 < jblk; j0 += MK_ZCH) {
    __syncthreads();
    for (int t = threadIdx.x; t < q * MK_ZCH; t += 256) {
      const int c = t / MK_ZCH, jj = t % MK_ZCH;
      us[c][jj] = (j0 + jj < ns) ? u[(long)c * md.n_pad + j0 + jj] : 0.0;
    }
    __syncthreads();
    const int jend = min(MK_ZCH, jmax - j0);   // <= 0: nothing left for this row
    // 64 column loads in flight per row (one HBM round trip per 64 columns, not per 8; the bytes in
    // flight bound a single CU's bandwidth, and the bottom row block reads 2,000 columns); the
    // products are added in ascending column order as before (same bits)
    int jj = 0;
    for (; jj + 64 <= jend; jj += 64) {
      double wv[64];
#pragma unroll
      for (int v = 0; v < 64; ++v) wv[v] = Wm[(long)(j0 + jj + v) * ld];
#pragma unroll
      for (int v = 0; v < 64; ++v)
#pragma unroll
        for (int c = 0; c < MK_QMAX; ++c)
          if (c < q) acc[c] += wv[v] * us[c][jj + v];
    }
    for (; jj + 32 <= jend; jj += 32) {
      double wv[32];
#pragma unroll
      for (int v = 0; v < 32; ++v) wv[v] = Wm[(long)(j0 + jj + v) * ld];
#pragma unroll
      for (int v = 0; v < 32; ++v)
#pragma unroll
        for (int c = 0; c < MK_QMAX; ++c)
          if (c < q) acc[c] += wv[v] * us[c][jj + v];
    }
    for (; jj + 8 <= jend; jj += 8) {
      double wv[8];
#pragma unroll
      for (int v = 0; v < 8; ++v) wv[v] = Wm[(long)(j0 + jj + v) * ld];
#pragma unroll
      for (int v = 0; v < 8; ++v)
#pragma unroll
        for (int c = 0; c < MK_QMAX; ++c)
          if (c < q) acc[c] += wv[v] * us[c][jj + v];
    }
    for (; jj < jend; ++jj) {
      const double wv = Wm[(long)(j0 + jj) * ld];
#pragma unroll
      for (int c = 0; c < MK_QMAX; ++c)
        if (c < q) acc[c] += wv * us[c][jj];
    }
  }
  if (r >= md.n_pad) return;
#pragma unroll
  for (int c = 0; c < MK_QMAX; ++c)
    if (c < q) md.Z[(((long)s * q + h) * q + c) * md.n_pad + r] = (r < ns) ? acc[c] : 0.0;
}

// ---------------------------------------------------------------- kriging (kept iterations)
__device__ inline void current_phi_nu(const Model& md, int s, int h, double* phi, double* nu) {
  const double* th = md.theta + (long)s * md.n_theta;
  *phi = logit_inv(th[md.ntri + h], md.phi_a[h], md.phi_b[h]);
  *nu = (md.cov_model == MK_COV_MATERN) ? logit_inv(th[md.ntri + md.q + h], md.nu_a[h], md.nu_b[h]) : 0.0;
}

// P^T[k][t] = rho(|obs_k - test_t|) for the listed pairs (zero outside the valid block).
// MODEL = MK_COV_EXPONENTIAL: exp(-phi d) inline, as in cand_value (bit-identical to CorrFn).
template <int MODEL>
__global__ __launch_bounds__(256) void k_pred_PT(Model md, const int* __restrict__ list, const int* __restrict__ count) {
  const int per = md.n_pad;   // one block per observation row
  const int e = blockIdx.x / per;
  if (e >= *count) return;
  const int k = blockIdx.x % per;
  const int sh = list[e];
  const int s = sh / md.q, h = sh % md.q;
  const int ns = md.n_s[s];
  double phi, nu;
  current_phi_nu(md, s, h, &phi, &nu);
  CorrFn rho;
  rho.init(phi, nu, md.cov_model);
  __shared__ double btab[5 * MK_BK_NTAB];
  if (MODEL == MK_COV_MATERN) {
    rho.fill_tables(btab, threadIdx.x, 256);
    __syncthreads();
    rho.tab = btab;
  }
  const double* cx = md.coords + (long)s * 2 * md.n_pad;
  const double ox = cx[k], oy = cx[md.n_pad + k];
  double* row = md.PT + ((long)sh * md.n_pad + k) * md.n_test_pad;
  const int tlim = md.ntt * MK_NB;   // the column blocks k_pred_var reads (all of n_test_pad when fused)
  for (int t = threadIdx.x; t < tlim; t += 256) {
    double v = 0.0;
    if (k < ns && t < md.n_test) {
      const double d = dist2d(ox, oy, md.coords_test[t], md.coords_test[md.n_test_pad + t]);
      v = (MODEL == MK_COV_EXPONENTIAL) ? exp(-rho.phi * d) : rho(d);
    }
    row[t] = v;
  }
}
template __global__ void k_pred_PT<MK_COV_EXPONENTIAL>(Model, const int*, const int*);
template __global__ void k_pred_PT<MK_COV_MATERN>(Model, const int*, const int*);

// Kriging tables: the current (phi, nu) of every listed pair over [0.5, phi x span_pt].
__global__ __launch_bounds__(256) void k_matern_table_list(Model md, const int* __restrict__ list,
                                                           const int* __restrict__ count) {
  if ((int)blockIdx.x >= *count) return;
  const int sh = list[blockIdx.x];
  const int s = sh / md.q, h = sh % md.q;
  double phi, nu;
  current_phi_nu(md, s, h, &phi, &nu);
  CorrFn rho;
  rho.init(phi, nu, MK_COV_MATERN);
  cheb_build_store(rho, md.span_pt ? phi * md.span_pt[s] : INFINITY, md.chtab_p + (long)sh * MK_CH_TAB);
}

// Matern P^T: one workgroup per (pair, MK_PT_RB observation rows) builds the Chebyshev table of
// its pair's current (phi, nu) over [0.5, phi x the extent of subset + test sites] and
// interpolates; elements outside the table are compacted per 4,096-site chunk and evaluated
// exactly (as matern_tile).
__global__ __launch_bounds__(256) void k_pred_PT_matern(Model md, const int* __restrict__ list,
                                                        const int* __restrict__ count) {
  constexpr int CHUNK = 4096;
  __shared__ double btab[5 * MK_BK_NTAB];
  __shared__ double chtab[MK_CH_NI_MAX * MK_CH_LD];
  __shared__ double vals[MK_CH_NI_MAX * MK_CH_N];
  __shared__ double cosm[MK_CH_N * MK_CH_N];
  __shared__ unsigned short idx[CHUNK];
  __shared__ int cnt;
  const int per = md.n_pad / MK_PT_RB;
  const int e = blockIdx.x / per;
  if (e >= *count) return;
  const int k0 = (blockIdx.x % per) * MK_PT_RB;
  const int sh = list[e];
  const int s = sh / md.q, h = sh % md.q;
  const int ns = md.n_s[s];
  const int tid = threadIdx.x, lane = tid & 63;
  const int tlim = md.ntt * MK_NB;   // the column blocks k_pred_var reads
  double* PT = md.PT + ((long)sh * md.n_pad + k0) * md.n_test_pad;
  if (k0 >= ns) {                    // padding rows
    for (int rr = 0; rr < MK_PT_RB; ++rr)
      for (int t = tid; t < tlim; t += 256) PT[(long)rr * md.n_test_pad + t] = 0.0;
    return;
  }
  double phi, nu;
  current_phi_nu(md, s, h, &phi, &nu);
  CorrFn rho;
  rho.init(phi, nu, md.cov_model);
  rho.fill_tables(btab, tid, 256);
  __syncthreads();
  rho.tab = btab;
  int ni;
  if (md.chtab_p) {   // k_matern_table_list
    ni = cheb_load(md.chtab_p + (long)sh * MK_CH_TAB, chtab);
    __syncthreads();
  } else {
    ni = cheb_count(md.span_pt ? phi * md.span_pt[s] : INFINITY);
    cheb_build(rho, ni, chtab, vals, cosm, tid, 256);
  }
  const double* cx = md.coords + (long)s * 2 * md.n_pad;
  const double* tx = md.coords_test;
  const double* ty = md.coords_test + md.n_test_pad;
  for (int rr = 0; rr < MK_PT_RB; ++rr) {
    const int k = k0 + rr;
    double* row = PT + (long)rr * md.n_test_pad;
    const bool kv = k < ns;
    const double ox = cx[k], oy = cx[md.n_pad + k];
    for (int t0 = 0; t0 < tlim; t0 += CHUNK) {
      if (tid == 0) cnt = 0;
      __syncthreads();
      const int tend = min(tlim, t0 + CHUNK);
      for (int t = t0 + tid; t < tend; t += 256) {   // tend - t0 is a multiple of 128: whole waves
        double v = 0.0;
        bool exact = false;
        if (kv && t < md.n_test) {
          const double d = dist2d(ox, oy, tx[t], ty[t]);
          exact = !cheb_eval(chtab, ni, d * phi, &v);
        }
        if (!exact) row[t] = v;
        const unsigned long long m = __ballot(exact);
        if (m) {
          const int leader = __ffsll((long long)m) - 1;
          int base = 0;
          if (lane == leader) base = atomicAdd(&cnt, __popcll(m));
          base = __shfl(base, leader, 64);
          if (exact) idx[base + __popcll(m & ((1ull << lane) - 1ull))] = (unsigned short)(t - t0);
        }
      }
      __syncthreads();
      const int n = cnt;
      for (int p = tid; p < n; p += 256) {
        const int t = t0 + idx[p];
        row[t] = rho(dist2d(ox, oy, tx[t], ty[t]));
      }
      __syncthreads();
    }
  }
}

// X = W P^T (row tile i, test tile tb), stored column-major by test site (XK[t][row]);
// partial column sums of squares over valid rows -> s_part[sh][i][t].
// GEN (exponential model): the P^T tile is generated in LDS chunk by chunk -- exp(-phi d), the
// expression k_pred_PT stores -- so P^T never exists in HBM: the kernel reads W (kept in L2 across
// the test tiles of one row panel: consecutive workgroups of a pair share i) and writes X; a
// stored P^T was re-read from HBM once per row panel (~8.5 x its size at n_s = 2000).
// !GEN (Matern): P^T from k_pred_PT (its Bessel tables are too heavy to inline per element).
// Cost-balanced XCD maps: row panel i costs i + 1 K-chunks of 128 (W lower-triangular), and
// xcd_map's contiguous split of the (pair, panel, tile) items cut pairs at arbitrary panels whenever
// the count of listed pairs was not a multiple of 8 -- the XCD holding a pair's late panels then set
// the launch's length (configs[4]'s tiled replay refreshes ~12 pairs per launch: 1.16 x the mean
// XCD load).
//  * many test tiles (ntt >= 64, the tiled replay): XCD x takes test tiles [x q, x q + q), q =
//    ntt / 8 rounded up, of every panel of every pair -- exactly an eighth of every panel's cost
//    (each XCD reads every W panel into its own L2: 8 x W's bytes, small beside P^T's);
//  * few (the fused path, ntt = n_test / 128, ~100 pairs per launch at configs[2]): xcd_map's
//    contiguous split, which keeps a pair's panels on one XCD so its P^T is read into one L2 (1.6 %
//    above the mean XCD load at 107 pairs; rotating the panels over the XCDs measured 0.7 % slower).
int pv_grid(int max_entries, int nt, int ntt) {
  return ntt >= 64 ? 8 * max_entries * nt * ((ntt + 7) / 8) : xcd_grid(max_entries, nt * ntt);
}

template <bool GEN>
__global__ __launch_bounds__(256, 2) void k_pred_var(Model md, MatSet ms, const int* __restrict__ list,
                                                  const int* __restrict__ count) {
  extern __shared__ __attribute__((aligned(16))) double lds[];   // MK_GD_LDS_BYTES
  __shared__ double red[2][MK_NB];
  // block b runs on XCD b % 8 (xcd_map); within an XCD pair-major, then panels (largest first),
  // then test tiles: the workgroups an XCD holds at once share one W row panel (L2); grouped rasters
  // that share P^T blocks instead measured slower
  const int x = blockIdx.x & 7, jx = blockIdx.x >> 3;
  int e, i, tb;
  if (md.ntt >= 64) {
    const int qt = (md.ntt + 7) / 8, per_x = ms.nt * qt;
    e = jx / per_x;
    const int rr = jx % per_x;
    i = ms.nt - 1 - rr / qt;
    tb = x * qt + rr % qt;
    if (tb >= md.ntt) return;
  } else {
    int t_;
    if (!xcd_map(*count, ms.nt * md.ntt, &e, &t_)) return;
    i = t_ / md.ntt;
    tb = t_ % md.ntt;
  }
  if (e >= *count) return;
  const int sh = list[e];
  const int s = sh / md.q;
  const int ns = md.n_s[s];
  const long ld = ms.ld;
  const double* Wm = wmat(ms, sh);
  Acc acc;
  acc_zero(acc);
  const int K = (i + 1) * MK_NB;   // W lower-triangular
  if (GEN) {
    const int h = sh % md.q;
    double phi, nu;
    current_phi_nu(md, s, h, &phi, &nu);
    // thread: k-row r of every chunk, 8 consecutive test sites c0 .. c0+7 of the tile
    const int r = threadIdx.x >> 4, c0 = (threadIdx.x & 15) * 8;
    const double* cx = md.coords + (long)s * 2 * md.n_pad;
    double tx[8], ty[8];
    bool tv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int t = tb * MK_NB + c0 + j;
      tv[j] = t < md.n_test;
      tx[j] = tv[j] ? md.coords_test[t] : 0.0;
      ty[j] = tv[j] ? md.coords_test[md.n_test_pad + t] : 0.0;
    }
    gemm_tile_genb<128, 128, true>(Wm + i * MK_NB, ld, K, acc, lds, [&](int k0, double* img) {
      const int k = k0 + r;
      const bool kv = k < ns;
      const double ox = cx[k], oy = cx[md.n_pad + k];
      d2 v[4];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const double d = dist2d(ox, oy, tx[j], ty[j]);
        const double x = (kv && tv[j]) ? exp(-phi * d) : 0.0;
        if (j & 1) v[j >> 1].y = x;
        else v[j >> 1].x = x;
      }
      d2* dst = reinterpret_cast<d2*>(img + r * gb_stride(128) + c0);
#pragma unroll
      for (int j = 0; j < 4; ++j) dst[j] = v[j];
    });
  } else {
    const double* PT = md.PT + (long)sh * md.n_pad * md.n_test_pad + tb * MK_NB;
    // dense: skipping W_ii's zero triangle (SKIP_TRI_A, 5 % of the MFMAs) measured slower here, 0.736 vs
    // 0.758 of peak (profiles/r06/tri_skip), unlike in the inverse levels
    gemm_128<true, true>(Wm + i * MK_NB, ld, PT, md.n_test_pad, K, K, acc, lds);
  }
  double* XK = md.XK + (long)sh * md.n_test_pad * md.n_pad + (long)tb * MK_NB * md.n_pad + i * MK_NB;
  store_tile(XK, md.n_pad, acc);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w & 1;
  double colsum[4][4];
#pragma unroll
  for (int bn = 0; bn < 4; ++bn)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      double v = 0.0;
#pragma unroll
      for (int bm = 0; bm < 4; ++bm) {
        const int m = i * MK_NB + acc_row(bm);
        const double x = acc.v[bm][bn][r];
        v += (m < ns) ? x * x : 0.0;
      }
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      colsum[bn][r] = v;
    }
  __syncthreads();
  if ((lane & 15) == 0) {
#pragma unroll
    for (int bn = 0; bn < 4; ++bn)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wm][acc_col(bn, r)] = colsum[bn][r];
  }
  __syncthreads();
  if (threadIdx.x < MK_NB) {
    const int n = threadIdx.x;
    md.s_part[((long)sh * ms.nt + i) * md.n_test_pad + tb * MK_NB + n] = red[0][n] + red[1][n];
  }
}
template __global__ void k_pred_var<true>(Model, MatSet, const int*, const int*);
template __global__ void k_pred_var<false>(Model, MatSet, const int*, const int*);

__global__ __launch_bounds__(256) void k_pred_var_reduce(Model md, int nt, const int* __restrict__ list,
                                                         const int* __restrict__ count) {
  const int per = md.n_test_pad / 256;
  const int e = blockIdx.x / per;
  if (e >= *count) return;
  const int sh = list[e];
  const int t = (blockIdx.x % per) * 256 + threadIdx.x;
  double v = 0.0;
  for (int i = 0; i < nt; ++i) v += md.s_part[((long)sh * nt + i) * md.n_test_pad + t];
  md.s_pred[(long)sh * md.n_test_pad + t] = v;
}

}  // namespace mk
