// Adaptive Metropolis-within-Gibbs for spMvGLM (binomial logit, LMC), batched
// over every subset of the shard, plus the fused kriging draw, type-7
// quantile summaries and the quantile-average combine.
//
// Reference: MetaKriging_BinaryResponse.R:80-84 (spMvGLM amcmc, n.batch x
// batch.length, accept.rate 0.43), MK.R:87 (spPredict), MK.R:88-89 (200
// type-7 quantiles), MK.R:123-133 (mean of subset grids).  The parameter
// order, transforms, priors and adaptation rule are spBayes'; the ratios are
// computed incrementally (DESIGN.md "Sampler specification") and are
// identical to oracle/spmvglm.py, which tests/ replays on the same Philox draws.
#include "mk_types.hpp"
#include "mk_corr.hpp"

namespace mk {

// ---------------------------------------------------------------- small q x q helpers (thread-local)
__device__ inline void tri_to_A(const double* tri, int q, double* A) {
  for (int i = 0; i < q * q; ++i) A[i] = 0.0;
  int k = 0;
  for (int j = 0; j < q; ++j)
    for (int i = j; i < q; ++i, ++k) A[i + j * q] = (i == j) ? exp(tri[k]) : tri[k];
}

__device__ inline void lower_inverse(const double* A, int q, double* Ai) {
  // forward substitution, column by column (A lower, col-major)
  for (int c = 0; c < q; ++c) {
    for (int r = 0; r < q; ++r) {
      if (r < c) { Ai[r + c * q] = 0.0; continue; }
      double s = (r == c) ? 1.0 : 0.0;
      for (int m = c; m < r; ++m) s -= A[r + m * q] * Ai[m + c * q];
      Ai[r + c * q] = s / A[r + r * q];
    }
  }
}

// IW(df,S) log prior of K = A A' + Jacobian of (lower A, log diag) -> K (spBayes spMvGLM).
__device__ inline double iw_logprior(const double* A, const double* Ai, int q, double df, const double* S,
                                     double* logdetK) {
  double ld = 0.0;
  for (int k = 0; k < q; ++k) ld += log(A[k + k * q]);
  ld *= 2.0;
  double tr = 0.0;  // sum_ij S_ij Kinv_ji, Kinv = Ai' Ai
  for (int i = 0; i < q; ++i)
    for (int j = 0; j < q; ++j) {
      double kinv = 0.0;
      for (int m = 0; m < q; ++m) kinv += Ai[m + j * q] * Ai[m + i * q];
      tr += S[i + j * q] * kinv;
    }
  double out = -0.5 * (df + q + 1.0) * ld - 0.5 * tr;
  for (int k = 0; k < q; ++k) out += (q - k) * log(A[k + k * q]) + log(A[k + k * q]);
  *logdetK = ld;
  return out;
}

// ---------------------------------------------------------------- 1. beta_j (flat prior)
// One workgroup per subset walks its n_s q sites once per beta_j: the loads of MK_BATCH strided
// iterations are issued together before their terms are added (in the same order as a plain
// strided loop: the same bits), so the loop pays the HBM latency once per batch, not per site.
#define MK_BATCH 8
__global__ __launch_bounds__(256) void k_beta(Model md, int iter) {
  __shared__ double red[8];
  const int s = blockIdx.x, tid = threadIdx.x;
  const Key key = subset_key(md, s);
  const int Ns = md.n_s[s] * md.q;
  const double* y = md.y + (long)s * md.Np;
  const double* wt = md.wt + (long)s * md.Np;
  double* eta = md.eta + (long)s * md.Np;
  for (int j = 0; j < md.p; ++j) {
    const double z = proposal_normal(key, j, iter);
    const double lu = accept_log_uniform(key, j, iter);
    const double delta = exp(md.tune[(long)s * md.n_mh_max + j]) * z;
    const double* xj = md.X + ((long)s * md.p + j) * md.Np;
    double loc = 0.0;
    for (int k0 = tid; k0 < Ns; k0 += 256 * MK_BATCH) {
      double yv[MK_BATCH], wv[MK_BATCH], ev[MK_BATCH], xv[MK_BATCH];
#pragma unroll
      for (int u = 0; u < MK_BATCH; ++u) {
        const int k = min(k0 + 256 * u, Ns - 1);   // clamped: in bounds, unused past Ns
        yv[u] = y[k];
        wv[u] = wt[k];
        ev[u] = eta[k];
        xv[u] = xj[k];
      }
      // the batch's terms are independent (no branch between them: their exp / log1p chains
      // interleave); past-the-end entries add an exact +0.0 (loc is never -0.0), same bits
      double tv[MK_BATCH];
#pragma unroll
      for (int u = 0; u < MK_BATCH; ++u) {
        const double t =
            loglik_term(yv[u], wv[u], ev[u] + delta * xv[u], md.link) - loglik_term(yv[u], wv[u], ev[u], md.link);
        tv[u] = (k0 + 256 * u < Ns) ? t : 0.0;
      }
#pragma unroll
      for (int u = 0; u < MK_BATCH; ++u) loc += tv[u];
    }
    const double tot = block_sum<256>(loc, red);
    if (lu <= tot) {
      for (int k = tid; k < Ns; k += 256) eta[k] = eta[k] + delta * xj[k];
      if (tid == 0) {
        md.beta[(long)s * md.p + j] += delta;
        md.acc[(long)s * md.n_mh_max + j] += 1.0;
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- 2. A entries
// T[h][c][d] = u_c' R_h^-1 u_d = Z_{h,c} . Z_{h,d} (q = 1: |z|^2); every candidate's
// quadratic form is sum_h sum_cd M_hc M_hd T_hcd with M = A'^-1 A_base (O(q^3) per proposal).
__global__ __launch_bounds__(256) void k_Aphase(Model md, int iter) {
  __shared__ double red[8];
  __shared__ double T[MK_QMAX * MK_QMAX * MK_QMAX];
  __shared__ double Msh[MK_QMAX * MK_QMAX], Aish[MK_QMAX * MK_QMAX];
  const int s = blockIdx.x, tid = threadIdx.x;
  const int q = md.q, ns = md.n_s[s];
  const Key key = subset_key(md, s);
  double* z = md.z + (long)s * q * md.n_pad;
  const double* Z = md.Z + (long)s * q * q * md.n_pad;
  // ---- T (symmetric in c,d); batched loads as in k_beta (same order, same bits)
  for (int h = 0; h < q; ++h)
    for (int c = 0; c < q; ++c)
      for (int d = c; d < q; ++d) {
        const double* zc = (q == 1) ? z : Z + ((long)h * q + c) * md.n_pad;
        const double* zd = (q == 1) ? z : Z + ((long)h * q + d) * md.n_pad;
        double loc = 0.0;
        for (int i0 = tid; i0 < ns; i0 += 256 * MK_BATCH) {
          double a[MK_BATCH], b[MK_BATCH];
#pragma unroll
          for (int u = 0; u < MK_BATCH; ++u) {
            const int i = min(i0 + 256 * u, ns - 1);
            a[u] = zc[i];
            b[u] = zd[i];
          }
#pragma unroll
          for (int u = 0; u < MK_BATCH; ++u)
            if (i0 + 256 * u < ns) loc += a[u] * b[u];
        }
        const double tot = block_sum<256>(loc, red);
        if (tid == 0) { T[(h * q + c) * q + d] = tot; T[(h * q + d) * q + c] = tot; }
      }
  __syncthreads();
  if (tid == 0) {
    double* th = md.theta + (long)s * md.n_theta;
    double Ab[16], Ac[16], Ai[16], M[16], tri[10], trc[10];
    for (int k = 0; k < md.ntri; ++k) tri[k] = th[k];
    tri_to_A(tri, q, Ab);
    auto objective = [&](const double* Acand, double* Aiout) -> double {
      lower_inverse(Acand, q, Aiout);
      for (int r = 0; r < q; ++r)
        for (int c = 0; c < q; ++c) {
          double v = 0.0;
          for (int m = 0; m < q; ++m) v += Aiout[r + m * q] * Ab[m + c * q];
          M[r + c * q] = v;
        }
      double quad = 0.0;
      for (int h = 0; h < q; ++h)
        for (int c = 0; c < q; ++c)
          for (int d = 0; d < q; ++d) quad += M[h + c * q] * M[h + d * q] * T[(h * q + c) * q + d];
      double ldK;
      const double lp = iw_logprior(Acand, Aiout, q, md.iw_df, md.iw_S, &ldK);
      return -0.5 * ns * ldK - 0.5 * quad + lp;
    };
    double f_cur = objective(Ab, Ai);
    for (int k = 0; k < md.ntri; ++k) {
      const int j = md.o_A + k;
      const double zz = proposal_normal(key, j, iter);
      const double lu = accept_log_uniform(key, j, iter);
      for (int m = 0; m < md.ntri; ++m) trc[m] = tri[m];
      trc[k] += exp(md.tune[(long)s * md.n_mh_max + j]) * zz;
      tri_to_A(trc, q, Ac);
      double Aic[16];
      const double f_c = objective(Ac, Aic);
      if (lu <= f_c - f_cur) {
        for (int m = 0; m < md.ntri; ++m) tri[m] = trc[m];
        f_cur = f_c;
        md.acc[(long)s * md.n_mh_max + j] += 1.0;
      }
    }
    for (int k = 0; k < md.ntri; ++k) th[k] = tri[k];
    double Af[16];
    tri_to_A(tri, q, Af);
    lower_inverse(Af, q, Ai);
    for (int r = 0; r < q; ++r)
      for (int c = 0; c < q; ++c) {
        double v = 0.0;
        for (int m = 0; m < q; ++m) v += Ai[r + m * q] * Ab[m + c * q];
        Msh[r + c * q] = v;
      }
    for (int i = 0; i < q * q; ++i) {
      Aish[i] = Ai[i];
      md.A_full[(long)s * q * q + i] = Af[i];
      md.Ainv[(long)s * q * q + i] = Ai[i];
    }
  }
  __syncthreads();
  // ---- u = A^-1 w,  z_h = W_h u_h = sum_c M_hc Z_{h,c}
  const double* w = md.w + (long)s * md.Np;
  double* uw = md.u + (long)s * q * md.n_pad;
  for (int i = tid; i < ns; i += 256) {
    for (int h = 0; h < q; ++h) {
      double uv = 0.0;
      for (int a = 0; a < q; ++a) uv += Aish[h + a * q] * w[i * q + a];
      uw[(long)h * md.n_pad + i] = uv;
      if (q == 1) {
        z[i] = Msh[0] * z[i];
      } else {
        double zv = 0.0;
        for (int c = 0; c < q; ++c) zv += Msh[h + c * q] * Z[((long)h * q + c) * md.n_pad + i];
        z[(long)h * md.n_pad + i] = zv;
      }
    }
  }
  __syncthreads();
  // ---- current quadratic forms |z_h|^2 = u_h' R_h^-1 u_h for the phi / nu proposals
  for (int h = 0; h < q; ++h) {
    double loc = 0.0;
    const double* zh = z + (long)h * md.n_pad;
    for (int i0 = tid; i0 < ns; i0 += 256 * MK_BATCH) {
      double a[MK_BATCH];
#pragma unroll
      for (int u = 0; u < MK_BATCH; ++u) a[u] = zh[min(i0 + 256 * u, ns - 1)];
#pragma unroll
      for (int u = 0; u < MK_BATCH; ++u)
        if (i0 + 256 * u < ns) loc += a[u] * a[u];
    }
    const double tot = block_sum<256>(loc, red);
    if (tid == 0) md.quad[(long)s * q + h] = tot;
  }
}

// ---------------------------------------------------------------- 3. phi_h / nu_h decision
__global__ __launch_bounds__(64) void k_theta_mh(Model md, MatSet ms, int h0, int hc, int which, int iter) {
  const int e = blockIdx.x * 64 + threadIdx.x;
  if (e >= md.S * hc) return;
  const int s = e / hc, h = h0 + e % hc;
  const Key key = subset_key(md, s);
  const int sh = s * md.q + h;
  double* th = md.theta + (long)s * md.n_theta;
  const int idx = (which == 0) ? md.ntri + h : md.ntri + md.q + h;
  const int j_mh = (which == 0) ? md.o_phi + h : md.o_nu + h;
  const double a = (which == 0) ? md.phi_a[h] : md.nu_a[h];
  const double b = (which == 0) ? md.phi_b[h] : md.nu_b[h];
  const double z = proposal_normal(key, j_mh, iter);
  const double lu = accept_log_uniform(key, j_mh, iter);
  const double th_c = th[idx] + exp(md.tune[(long)s * md.n_mh_max + j_mh]) * z;
  const double v_c = logit_inv(th_c, a, b), v_cur = logit_inv(th[idx], a, b);
  double ldc = 0.0;
  for (int k = 0; k < md.nt; ++k) ldc += md.ld_part[(long)sh * md.nt + k];
  const double qc = md.quad_c[sh];
  const double ratio = -0.5 * (ldc - md.logdetR[sh]) - 0.5 * (qc - md.quad[sh]) + unif_jacobian(v_c, a, b) -
                       unif_jacobian(v_cur, a, b);
  const bool accept = md.info[sh] == 0 && lu <= ratio;
  if (accept) {
    th[idx] = th_c;
    ms.cur[sh] ^= 1;
    md.logdetR[sh] = ldc;
    md.quad[sh] = qc;
    md.dirty[sh] = 1;
    md.acc[(long)s * md.n_mh_max + j_mh] += 1.0;
  }
  if (which == 1 && md.la_nu) md.la_nu[sh] = accept ? 1 : 0;   // lookahead schedule: k_nu_border
  md.info[sh] = 0;
}

// Compact lists (deterministic order) of (subset, outcome) pairs: list_inv = pairs whose
// factor changed this iteration; list_pred = those, or every pair when `force` (first
// kept iteration: kriging needs X for the current factors).
__global__ __launch_bounds__(256) void k_dirty_list(Model md, int force, int* list_inv, int* count_inv,
                                                    int* list_pred, int* count_pred) {
  __shared__ int base[2];
  __shared__ int wc[2][4];
  if (threadIdx.x < 2) base[threadIdx.x] = 0;
  __syncthreads();
  const int n = md.S * md.q;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int c0 = 0; c0 < n; c0 += 256) {
    const int e = c0 + threadIdx.x;
    const int d = (e < n) ? md.dirty[e] : 0;
    const int flag[2] = {d, (e < n) ? (force || d) : 0};
    int before[2];
    for (int l = 0; l < 2; ++l) {
      const unsigned long long bal = __ballot(flag[l]);
      before[l] = __popcll(bal & ((1ull << lane) - 1ull));
      if (lane == 0) wc[l][wv] = __popcll(bal);
    }
    __syncthreads();
    for (int l = 0; l < 2; ++l) {
      int off = base[l];
      for (int k = 0; k < wv; ++k) off += wc[l][k];
      if (flag[l]) (l == 0 ? list_inv : list_pred)[off + before[l]] = e;
    }
    if (e < n) md.dirty[e] = 0;
    __syncthreads();
    if (threadIdx.x < 2) base[threadIdx.x] += wc[threadIdx.x][0] + wc[threadIdx.x][1] + wc[threadIdx.x][2] + wc[threadIdx.x][3];
    __syncthreads();
  }
  if (threadIdx.x == 0) { *count_inv = base[0]; *count_pred = base[1]; }
}

// ---------------------------------------------------------------- 5. single-site w sweep
// Sites in blocks of 64.  For block B: g_B = W[:,B]' z (dots over rows >= b0), then the
// sequential MH steps inside the block use the 64x64 tile Q_BB of R^-1 (from QB) to carry
// accepted moves forward (g_i += delta'_k Q_ik), then z += W[:,B] delta'_B (rows >= b0).
//
// Two kernels, bit-identical by construction (the chains do not depend on which one runs):
//   k_sweep     one 1024-thread workgroup per subset, W panels streamed twice (dots, update):
//               large shards (every CU already has a subset);
//   k_sweep_mg  one 256-thread workgroup per (subset, 128-row tile), behind an admission consensus: the
//               workgroup keeps its tile's 128 x 64 panel of W in registers from the dots to
//               the update (one pass over W), the tiles' partial dots meet through a per-subset
//               counter barrier and every workgroup runs the block's MH steps itself: small
//               shards (32 subsets on 256 CUs).
// The shared summation order: dot g_i = sum over 128-row tiles t = b0/128, ... in tile order of
// p_t = wave-xor-reduce(a0 + a1), lane l holding rows 128t + 2l, +1 (a0, a1 masked to
// b0 <= row < n_s); update z_r += ((s0 + s1) + s2) + s3, s_w = fma chain over the block's columns
// i = w, w + 4, ... (ascending).
#define SW_B 64
#define SW_T MK_SW_T
// Lane i's value (i wave-uniform) as a scalar: two v_readlane_b32.
__device__ inline double rlane_u(double v, int i) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), i);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), i);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// 64-bit DPP move as two 32-bit halves (gfx950's 64-bit DPP takes row_newbcast only).
template <int CTRL>
__device__ inline double dpp_f64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffll), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// Sum of the 64 lanes' values, the same in every lane: within each 16-lane row by DPP (quad
// xor 1, quad xor 2, half-row mirror, row mirror -- VALU only, no LDS crossbar), then the four
// row sums as ((r0 + r1) + (r2 + r3)) from lanes 0, 16, 32, 48.  The sweep's dot products use
// this tree in both kernels.
__device__ inline double wave_sum_dpp(double x) {
  x += dpp_f64<0xB1>(x);    // quad_perm [1,0,3,2]
  x += dpp_f64<0x4E>(x);    // quad_perm [2,3,0,1]
  x += dpp_f64<0x141>(x);   // row_half_mirror
  x += dpp_f64<0x140>(x);   // row_mirror
  return (rlane_u(x, 0) + rlane_u(x, 16)) + (rlane_u(x, 32) + rlane_u(x, 48));
}

// Data the multi-workgroup sweep exchanges between the workgroups of one subset -- which all
// run on one XCD (k_sweep_mg's block map; checked at run time) -- moves through that XCD's L2:
// plain stores (the vector L1 writes through), s_waitcnt for their completion before the
// barrier counter's atomic increment, and L1-bypassing loads (buffer loads with sc0) on the
// reader's side.  No cache-wide release / acquire fence (an L2 write-back / invalidate per
// workgroup) is needed.  COH = false: ordinary loads (the one-workgroup kernel).
typedef unsigned int u2v __attribute__((ext_vector_type(2)));
template <bool COH>
__device__ inline double ld_l2(const double* base, long idx) {
  if (!COH) return base[idx];
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 0x7fffffff, 0x00020000);
  const u2v v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)(idx * 8), 0, 1);   // aux 1: sc0 (bypass L1)
  return __builtin_bit_cast(double, v);
}

// Proposals, likelihood differences and accept draws of sites [k0, k1) (location-major entries):
// independent of the sweep order.
__device__ inline void sweep_precompute(const Model& md, int s, int iter, int k0, int k1, int t0, int nthr) {
  const Key key = subset_key(md, s);
  const double* y = md.y + (long)s * md.Np;
  const double* wt = md.wt + (long)s * md.Np;
  const double* eta = md.eta + (long)s * md.Np;
  const double* tune = md.tune + (long)s * md.n_mh_max + md.o_w;
  double* dl = md.sw_delta + (long)s * md.Np;
  double* dll = md.sw_dll + (long)s * md.Np;
  double* lgu = md.sw_logu + (long)s * md.Np;
  int* sacc = md.sw_acc + (long)s * md.Np;
  for (int k = k0 + t0; k < k1; k += nthr) {
    const int j = md.o_w + k;
    const double zz = proposal_normal(key, j, iter);
    const double d = exp(tune[k]) * zz;
    dl[k] = d;
    dll[k] = loglik_term(y[k], wt[k], eta[k] + d, md.link) - loglik_term(y[k], wt[k], eta[k], md.link);
    lgu[k] = accept_log_uniform(key, j, iter);
    sacc[k] = 0;
  }
}

// The sequential Metropolis steps of one block (wave 0 only).  Lane i preloads site b0+i's
// proposal d, likelihood difference, accept draw and the step's g-independent term
// 0.5 d^2 sum_h A^-1_ha^2 Q_ii; each step reads them (and the carried g) by readlane with the
// uniform step index, the LDS column of Q_BB it may need was requested one step earlier, and an
// accepted move updates g by a select rather than a branch -- the step's dependent chain is
// readlane, three multiply-adds, a compare and a select.  Lane i collects site b0+i's
// coefficients and accept flags; they leave after the loop.
// gb [q][64] dots, Qb [q][64*64], Ai [q*q]; out: dacc [q][64] coefficients, accept flags
// (write_acc) into sw_acc.  Returns whether any site moved (the same in every lane).
// Accept iff log U <= dll - (d c + 0.5 d^2 dd), c = sum_h A^-1_ha g_h, dd = sum_h (A^-1_ha)^2 Q_ii.
template <int Q, bool COH>
__device__ inline int sweep_block_mh_q(const Model& md, int s, int b0, int nb, const double* gb, const double* Qb,
                                       const double* Ai, double* dacc, bool write_acc) {
  constexpr int q = Q;   // outcomes, at compile time: every loop below unrolls without branches
  const int lane = threadIdx.x & 63;
  const double* dl = md.sw_delta + (long)s * md.Np;
  const double* dll = md.sw_dll + (long)s * md.Np;
  const double* lgu = md.sw_logu + (long)s * md.Np;
  int* sacc = md.sw_acc + (long)s * md.Np;
  double gl[Q], dlr[Q], dllr[Q], lgr[Q], hdd[Q], dsum[Q], qn[Q], ai[Q * Q];
  const int ls = (lane < nb) ? lane : 0;
#pragma unroll
  for (int e = 0; e < Q * Q; ++e) ai[e] = Ai[e];
#pragma unroll
  for (int h = 0; h < Q; ++h) {
    gl[h] = (lane < nb) ? gb[h * SW_B + lane] : 0.0;
    const int k = (b0 + ls) * q + h;
    dlr[h] = ld_l2<COH>(dl, k);
    dllr[h] = ld_l2<COH>(dll, k);
    lgr[h] = ld_l2<COH>(lgu, k);
    dsum[h] = 0.0;
    qn[h] = Qb[h * SW_B * SW_B + lane];
  }
#pragma unroll
  for (int a = 0; a < Q; ++a) {
    double dd = 0.0;
#pragma unroll
    for (int h = 0; h < Q; ++h) {
      const double aih = ai[h + a * q];
      dd += (aih * aih) * Qb[h * SW_B * SW_B + ls * SW_B + ls];
    }
    const double d = dlr[a];
    hdd[a] = 0.5 * d * d * dd;
  }
  int flags = 0, anyl = 0;
  for (int i = 0; i < nb; ++i) {
    const int iu = __builtin_amdgcn_readfirstlane(i);
    const int inext = __builtin_amdgcn_readfirstlane(min(i + 1, nb - 1));   // next step's column (clamped)
    double qc[Q];
#pragma unroll
    for (int h = 0; h < Q; ++h) {
      qc[h] = qn[h];
      qn[h] = Qb[h * SW_B * SW_B + inext * SW_B + lane];
    }
#pragma unroll
    for (int a = 0; a < Q; ++a) {
      const double d = rlane_u(dlr[a], iu);
      double c = ai[a * q] * rlane_u(gl[0], iu);
#pragma unroll
      for (int h = 1; h < Q; ++h) c += ai[h + a * q] * rlane_u(gl[h], iu);
      const double ratio = rlane_u(dllr[a], iu) - (d * c + rlane_u(hdd[a], iu));
      const bool acc = rlane_u(lgr[a], iu) <= ratio;     // uniform
#pragma unroll
      for (int h = 0; h < Q; ++h) {
        const double coef = d * ai[h + a * q];
        const double gn = gl[h] + coef * qc[h];
        gl[h] = acc ? gn : gl[h];
        const double ds = dsum[h] + coef;
        dsum[h] = (acc && lane == iu) ? ds : dsum[h];
      }
      flags |= (acc && lane == iu) ? (1 << a) : 0;
      anyl |= acc ? 1 : 0;
    }
  }
#pragma unroll
  for (int h = 0; h < Q; ++h) dacc[h * SW_B + lane] = dsum[h];
  if (write_acc && lane < nb)
    for (int a = 0; a < q; ++a)
      if ((flags >> a) & 1) sacc[(b0 + lane) * q + a] = 1;
  return anyl;
}

// Accepted moves of sites [i0, i1) into w, eta, u and the batch accept counts.
__device__ inline void sweep_apply(const Model& md, int s, int i0, int i1, const double* Ai, int t0, int nthr) {
  const int q = md.q;
  double* w = md.w + (long)s * md.Np;
  double* eta = md.eta + (long)s * md.Np;
  double* u = md.u + (long)s * q * md.n_pad;
  double* acc = md.acc + (long)s * md.n_mh_max + md.o_w;
  const double* dl = md.sw_delta + (long)s * md.Np;
  const int* sacc = md.sw_acc + (long)s * md.Np;
  for (int i = i0 + t0; i < i1; i += nthr) {
    for (int a = 0; a < q; ++a) {
      const int k = i * q + a;
      if (sacc[k]) {
        w[k] += dl[k];
        eta[k] += dl[k];
        acc[k] += 1.0;
        for (int h = 0; h < q; ++h) u[(long)h * md.n_pad + i] += dl[k] * Ai[h + a * q];
      }
    }
  }
}

// adm (optional): the multi-workgroup sweep's admission words; subsets it swept (MK_ADM_DONE) are
// skipped, so this launch is the fallback for the subsets it did not admit (same bits, §4.3); fb counts them.
template <int Q>
__global__ __launch_bounds__(SW_T) void k_sweep(Model md, MatSet ms, int iter, const int* __restrict__ adm,
                                                int* __restrict__ fb) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  constexpr int q = Q;
  if (adm) {
    if (adm[blockIdx.x] & MK_ADM_DONE) return;
    if (threadIdx.x == 0) atomicAdd(fb, 1);   // KS_SWEEP_FALLBACK
  }
  double* Qb = smem;                              // [q][SW_B*SW_B] column-major
  double* gb = smem + q * SW_B * SW_B;            // [q][SW_B]
  double* dacc = gb + q * SW_B;                   // [q][SW_B]
  __shared__ int any_acc;
  __shared__ double Ai[MK_QMAX * MK_QMAX];
  const int s = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int ns = md.n_s[s];
  const long ld = ms.ld;
  double* z = md.z + (long)s * q * md.n_pad;
  if (tid < q * q) Ai[tid] = md.Ainv[(long)s * q * q + tid];
  sweep_precompute(md, s, iter, 0, ns * q, tid, SW_T);
  if (tid == 0) any_acc = 0;
  __syncthreads();
  const int tl = (ns - 1) / MK_NB;                // last tile holding sites
  int p0 = 0, pnb = 0;
  for (int b0 = 0; b0 < ns + SW_B; b0 += SW_B) {
    const int nb = min(SW_B, ns - b0);
    // ---- (a) z += W[:, prev block] delta'_prev   (rows >= p0)
    // Thread t owns the row pair p0 + 2t, p0 + 2t + 1 (16-byte loads; p0 is even, ld even) and
    // issues the 16 column loads of a group before using them: unconditional loads (clamped
    // column; W is finite everywhere), the short-block tail masked by a zero coefficient.  Four
    // accumulators by column residue mod 4 (the shared order).
    if (pnb > 0 && any_acc) {
      for (int h = 0; h < q; ++h) {
        for (int r = p0 + 2 * tid; r < ns; r += 2 * SW_T) {
          const double* Wp = ms.W + ((long)s * q + h) * (ld * ld) + (long)p0 * ld + r;
          const double* da = dacc + h * SW_B;
          double* zh = z + (long)h * md.n_pad;
          d2 v4[4] = {{0.0, 0.0}, {0.0, 0.0}, {0.0, 0.0}, {0.0, 0.0}};
          for (int k0 = 0; k0 < pnb; k0 += 16) {
            d2 wv2[16];
#pragma unroll
            for (int u = 0; u < 16; ++u)
              wv2[u] = *reinterpret_cast<const d2*>(Wp + (long)min(k0 + u, pnb - 1) * ld);
#pragma unroll
            for (int u = 0; u < 16; ++u) {
              const double c = (k0 + u < pnb) ? da[k0 + u] : 0.0;
              v4[u & 3].x = fma(wv2[u].x, c, v4[u & 3].x);
              v4[u & 3].y = fma(wv2[u].y, c, v4[u & 3].y);
            }
          }
          const double vx = ((v4[0].x + v4[1].x) + v4[2].x) + v4[3].x;
          const double vy = ((v4[0].y + v4[1].y) + v4[2].y) + v4[3].y;
          zh[r] += vx;
          if (r + 1 < ns) zh[r + 1] += vy;
        }
      }
    }
    __syncthreads();
    if (nb <= 0) break;
    if (tid == 0) any_acc = 0;
    // ---- (b) Q_BB tile into LDS, dots g_B = W[:,B]' z over rows >= b0
    const int tile = b0 / MK_NB, off = b0 % MK_NB;
    for (int h = 0; h < q; ++h) {
      const double* QBt = ms.QB + (((long)s * q + h) * ms.nt + tile) * MK_NB * MK_NB;
      for (int e = tid; e < SW_B * SW_B; e += SW_T) {
        const int r = e & (SW_B - 1), c = e / SW_B;
        const double v = QBt[(off + r) + (off + c) * MK_NB];   // in the tile: off + 63 < 128
        Qb[h * SW_B * SW_B + e] = (r < nb && c < nb) ? v : 0.0;  // (a masked load would serialise)
      }
      const double* Wb = ms.W + ((long)s * q + h) * (ld * ld) + (long)b0 * ld;
      const double* zh = z + (long)h * md.n_pad;
      // one wave per column; lane l reads rows 128t + 2l, +1 of tiles t = tile .. tl (16-byte loads,
      // 8 tiles in flight, clamped to the last tile and masked by selects), one reduction per tile
      for (int i = wv; i < nb; i += SW_T / 64) {
        const double* col = Wb + (long)i * ld;
        double g = 0.0;
        for (int t0 = tile; t0 <= tl; t0 += 8) {
          d2 wv2[8], zv2[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int rc = MK_NB * min(t0 + u, tl) + 2 * lane;
            wv2[u] = *reinterpret_cast<const d2*>(col + rc);
            zv2[u] = *reinterpret_cast<const d2*>(zh + rc);
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            if (t0 + u > tl) break;
            const int r0 = MK_NB * (t0 + u) + 2 * lane;
            const double a0 = (r0 >= b0 && r0 < ns) ? wv2[u].x * zv2[u].x : 0.0;
            const double a1 = (r0 + 1 >= b0 && r0 + 1 < ns) ? wv2[u].y * zv2[u].y : 0.0;
            const double p = wave_sum_dpp(a0 + a1);
            g = (t0 + u == tile) ? p : g + p;
          }
        }
        if (lane == 0) gb[h * SW_B + i] = g;
      }
    }
    __syncthreads();
    // ---- (c) sequential Metropolis steps of the block (wave 0)
    if (wv == 0) {
      const int anyl = sweep_block_mh_q<Q, false>(md, s, b0, nb, gb, Qb, Ai, dacc, true);
      if (lane == 0) any_acc = anyl;
    }
    __syncthreads();
    p0 = b0;
    pnb = nb;
  }
  // ---- apply accepted moves to w, eta, u and the batch accept counts
  sweep_apply(md, s, 0, ns, Ai, tid, SW_T);
}

// Multi-workgroup sweep (small shards).  Grid: xcd_grid(S, nt) workgroups of 256 threads, a plain
// launch.  ADMISSION (before any chain state is touched): every workgroup of subset s arrives on
// the subset's admission word adm[s] (release) and waits -- bounded -- until all tl + 1 of them have
// arrived; a workgroup that times out marks the subset aborted (compare-and-swap, only while the
// count is short), and a late arrival that finds the mark leaves.  The decision is a consensus: every
// workgroup of s reads the same word.  Admitted, the subset's workgroups are co-resident -- a resident
// workgroup is never descheduled -- so every later wait among them completes; they also check that
// they share one XCD (the L2 exchange below needs it) and tile 0 marks the subset MK_ADM_DONE.  A
// subset not admitted leaves its state untouched and the next launch on the stream, k_sweep with
// adm, sweeps it (the same bits: the shared summation order below).  So no wait here depends on
// co-residency the hardware does not give, under any schedule (round 4 had relied on it).
// Workgroup (s, t) owns rows [128t, 128t + 128) of subset s
// (its z rows in registers, replicated in the four waves; its sites' proposals and final
// moves) and takes part in blocks b0 < min(n_s, 128t + 128).  Per block: partial dots of its
// tile for every column (wave w: columns w + 4j, lane l: rows 2l, 2l+1) into part[s][B & 1][t],
// arrive on cnt[s][B], prefetch Q_BB, wait for the block's tiles tf..tl, sum the partials in
// tile order, run the MH steps, update z from the same registers.  REG (q == 1): the panel
// stays in registers across the wait; else it is reloaded for the update.  The partial dots and
// the sites' proposals move through the subset's XCD L2 (ld_l2); the counters are atomics.  A
// barrier wait gives up after ~2^22 sleeps (err |= 1: the net under the admission argument; the host
// poisons the session) and every wave always exits; a subset split over XCDs is refused at admission.
// Q_BB of the block at b0 (q 64 x 64 column-major tiles of R_h^-1) straight into LDS by
// LDS-DMA: one wave instruction moves two columns (lanes 0-31 column 2j, 32-63 column 2j+1),
// no registers; completion is covered by the s_waitcnt before the next barrier arrival.  Entries
// beyond the block's last site are copied as they are (finite, and never read by the MH steps).
__device__ inline void qbb_dma(const Model& md, const MatSet& ms, int s, int b0, double* Qb) {
  const int q = md.q, tile = b0 / MK_NB, off = b0 % MK_NB;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int col = lane >> 5, row = 2 * (lane & 31);
  for (int h = 0; h < q; ++h) {
    const double* QBt = ms.QB + (((long)s * q + h) * ms.nt + tile) * MK_NB * MK_NB;
    for (int j = w; j < SW_B / 2; j += 4)
      __builtin_amdgcn_global_load_lds((const void*)(QBt + (off + row) + (long)(off + 2 * j + col) * MK_NB),
                                       (void*)(Qb + h * SW_B * SW_B + 2 * j * SW_B), 16, 0, 0);
  }
}

#define MK_NT_MAX_MG 32   // tiles per subset the multi-workgroup sweep supports (n_s <= 4095)
#ifdef MK_SWEEP_PROBE     // development probe only (tools/sweep_probe.py): per-phase clock of subset 0, tile 0
__device__ long long mk_sweep_ts[64 * 8];
#define SW_STAMP(B, i) do { if (s == 0 && t == tl && threadIdx.x == 0 && (B) < 64) mk_sweep_ts[(B) * 8 + (i)] = wall_clock64(); } while (0)
}  // namespace mk
extern "C" int mk_debug_sweep_probe(long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(mk::mk_sweep_ts), sizeof(long long) * 64 * 8) == hipSuccess ? 0 : -2;
}
namespace mk {
#else
#define SW_STAMP(B, i) do { } while (0)
#endif
template <int Q>
__global__ __launch_bounds__(256) void k_sweep_mg(Model md, MatSet ms, int iter, double* __restrict__ part,
                                                  int* __restrict__ cnt, int* __restrict__ xcc, int* __restrict__ err,
                                                  int* __restrict__ adm, int spins_max) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  constexpr int q = Q;
  constexpr bool REG = (Q == 1);
  const int nt = ms.nt;
  double* Qb = smem;                              // [q][SW_B*SW_B]
  double* gb = Qb + q * SW_B * SW_B;              // [q][SW_B]
  double* dacc = gb + q * SW_B;                   // [q][SW_B]
  double* red = dacc + q * SW_B;                  // [4][MK_NB] per-wave update sums
  __shared__ double Ai[MK_QMAX * MK_QMAX];
  __shared__ int any_acc, admitted;
  // block map: block b runs on XCD b % 8 (the dispatch order every kernel here relies on); subset
  // s takes slots (s / 8) * nt ... of XCD s % 8, so all of its tiles share one L2
  const int j = blockIdx.x >> 3;
  const int s = (blockIdx.x & 7) + 8 * (j / nt), t = j % nt;
  if (s >= md.S) return;
  const int ns = md.n_s[s];
  const int tl = (ns - 1) / MK_NB;
  if (t > tl) return;                             // rows >= n_s only: no sites, no dots
  // the exchange through L2 is sound only if the subset's workgroups share an XCD: each publishes
  // its XCC id before it arrives, and the admitted ones compare them
  const unsigned my_xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);   // hwreg(HW_REG_XCC_ID, 0, 4)
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) {
    __hip_atomic_store(xcc + (long)s * nt + t, (int)my_xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int target = tl + 1;
    int* a = adm + s;
    int v = __hip_atomic_fetch_add(a, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1;
    int ok = 0;
    for (int spins = 0; spins_max >= 0; ++spins) {   // spins_max < 0 (tests): refuse every subset
      if (v & MK_ADM_ABORT) break;
      if ((v & MK_ADM_COUNT) == target) {
        ok = 1;
        break;
      }
      if (spins >= spins_max) {   // give up on this subset unless the count completed meanwhile
        int expected = v;
        if (__hip_atomic_compare_exchange_strong(a, &expected, v | MK_ADM_ABORT, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE,
                                                 __HIP_MEMORY_SCOPE_AGENT))
          break;
        v = expected;
        continue;
      }
      __builtin_amdgcn_s_sleep(2);
      v = __hip_atomic_load(a, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (ok)   // every id was published before its arrival (release), this read follows all of them
      for (int u = 0; u <= tl; ++u)
        if (__hip_atomic_load(xcc + (long)s * nt + u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != (int)my_xcc) ok = 0;
    if (ok && t == 0) __hip_atomic_fetch_or(a, MK_ADM_DONE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    admitted = ok;
  }
  __syncthreads();
  if (!admitted) return;   // nothing written yet: k_sweep (adm) sweeps this subset
  const long ld = ms.ld;
  const int r0 = MK_NB * t + 2 * lane;            // this lane's rows r0, r0 + 1
  if (tid < q * q) Ai[tid] = md.Ainv[(long)s * q * q + tid];
  // own sites' proposals (read by the MH of blocks 2t, 2t+1 after barrier 2t)
  sweep_precompute(md, s, iter, MK_NB * t * q, min(MK_NB * (t + 1), ns) * q, tid, 256);
  d2 zr[Q];
#pragma unroll
  for (int h = 0; h < Q; ++h) zr[h] = *reinterpret_cast<const d2*>(md.z + ((long)s * q + h) * md.n_pad + r0);
  const long pstride = (long)nt * q * SW_B;       // one parity buffer of a subset
  double* ps = part + (long)s * 2 * pstride;
  int* cs = cnt + (long)s * (md.n_pad / SW_B);
  const int last_b = min(ns - 1, MK_NB * t + MK_NB - 1) / SW_B;
  qbb_dma(md, ms, s, 0, Qb);                      // block 0's Q_BB lands while the dots run
  for (int B = 0; B <= last_b; ++B) {
    const int b0 = B * SW_B, nb = min(SW_B, ns - b0), tf = b0 / MK_NB;
    double* pb = ps + (B & 1) * pstride;
    SW_STAMP(B, 0);
    // ---- partial dots of tile t for every column of the block
    d2 wreg[16];
    for (int h = 0; h < q; ++h) {
      const double* Wt = ms.W + ((long)s * q + h) * (ld * ld) + (long)b0 * ld + r0;
#pragma unroll
      for (int j = 0; j < 16; ++j) wreg[j] = *reinterpret_cast<const d2*>(Wt + (long)(wv + 4 * j) * ld);
      d2 zz = zr[0];
#pragma unroll
      for (int hh = 1; hh < Q; ++hh)
        if (hh == h) zz = zr[hh];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const double a0 = (r0 >= b0 && r0 < ns) ? wreg[j].x * zz.x : 0.0;
        const double a1 = (r0 + 1 >= b0 && r0 + 1 < ns) ? wreg[j].y * zz.y : 0.0;
        const double p = wave_sum_dpp(a0 + a1);
        if (lane == 0) pb[((long)t * q + h) * SW_B + wv + 4 * j] = p;
      }
    }
    __builtin_amdgcn_s_waitcnt(0);                // this wave's stores have reached L2
    __syncthreads();
    SW_STAMP(B, 1);
    if (tid == 0) __hip_atomic_fetch_add(cs + B, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    SW_STAMP(B, 2);
    if (tid == 0) {
      // tiles tf .. tl arrive at every barrier; at an even B > 0 also tile tf - 1, which left after
      // block B - 1 (its last) -- it arrives once it has read block B - 1's partials, so block B + 1
      // cannot overwrite that parity buffer under its reads
      const int target = tl - tf + 1 + ((B & 1) == 0 && B > 0 ? 1 : 0);
      int spins = 0;
      while (__hip_atomic_load(cs + B, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1 << 22)) {
          __hip_atomic_fetch_or(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    __syncthreads();
    SW_STAMP(B, 3);
    // ---- dots: partials of tiles tf .. tl summed in tile order (every workgroup, same bits);
    // L1-bypassing loads, all issued before the adds
    for (int e = tid; e < q * SW_B; e += 256) {
      const int h = e / SW_B, i = e % SW_B;
      double pv[MK_NT_MAX_MG];
#pragma unroll
      for (int u = 0; u < MK_NT_MAX_MG; ++u) pv[u] = ld_l2<true>(pb, ((long)min(tf + u, tl) * q + h) * SW_B + i);
      double g = pv[0];
#pragma unroll
      for (int u = 1; u < MK_NT_MAX_MG; ++u)
        if (tf + u <= tl) g = g + pv[u];
      gb[e] = g;
    }
    __syncthreads();
    if (B == last_b && t < tl && tid == 0)          // last read of this parity buffer by tile t
      __hip_atomic_fetch_add(cs + B + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    SW_STAMP(B, 4);
    // ---- the block's MH steps (wave 0 of every workgroup; the sites' owner records them)
    if (wv == 0) {
      const int anyl = sweep_block_mh_q<Q, true>(md, s, b0, nb, gb, Qb, Ai, dacc, t == tf);
      if (lane == 0) any_acc = anyl;
    }
    __syncthreads();
    SW_STAMP(B, 5);
    if (B < last_b) qbb_dma(md, ms, s, b0 + SW_B, Qb);   // next block's Q_BB behind the update and dots
    // ---- z rows of tile t (rows >= b0) += W[:, B] delta'_B
    if (any_acc) {
      for (int h = 0; h < q; ++h) {
        if (!REG) {
          const double* Wt = ms.W + ((long)s * q + h) * (ld * ld) + (long)b0 * ld + r0;
#pragma unroll
          for (int j = 0; j < 16; ++j) wreg[j] = *reinterpret_cast<const d2*>(Wt + (long)(wv + 4 * j) * ld);
        }
        d2 sw = {0.0, 0.0};
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int i = wv + 4 * j;
          const double c = (i < nb) ? dacc[h * SW_B + i] : 0.0;
          sw.x = fma(wreg[j].x, c, sw.x);
          sw.y = fma(wreg[j].y, c, sw.y);
        }
        red[wv * MK_NB + 2 * lane] = sw.x;
        red[wv * MK_NB + 2 * lane + 1] = sw.y;
        __syncthreads();
        const double vx = ((red[2 * lane] + red[MK_NB + 2 * lane]) + red[2 * MK_NB + 2 * lane]) + red[3 * MK_NB + 2 * lane];
        const double vy = ((red[2 * lane + 1] + red[MK_NB + 2 * lane + 1]) + red[2 * MK_NB + 2 * lane + 1]) +
                          red[3 * MK_NB + 2 * lane + 1];
        __syncthreads();
#pragma unroll
        for (int hh = 0; hh < Q; ++hh) {
          if (hh != h) continue;
          if (r0 >= b0 && r0 < ns) zr[hh].x += vx;
          if (r0 + 1 >= b0 && r0 + 1 < ns) zr[hh].y += vy;
        }
      }
    }
  }
  // ---- write back z rows; apply this tile's accepted moves
  if (wv == 0) {
#pragma unroll
    for (int h = 0; h < Q; ++h) *reinterpret_cast<d2*>(md.z + ((long)s * q + h) * md.n_pad + r0) = zr[h];
  }
  __syncthreads();
  sweep_apply(md, s, MK_NB * t, min(MK_NB * (t + 1), ns), Ai, tid, 256);
}
// Split-launch sweep (small shards, no inter-workgroup waiting).  The sweep's only sequential
// dependency -- block B's dots need z after block B-1's accepted moves -- is carried by stream
// order instead of by barriers between co-resident workgroups: one launch per 64-site block, one
// 256-thread workgroup per (subset, 128-row tile).  Launch B (i) runs block B-1's MH steps from the
// partial dots of the previous launch, redundantly in every tile workgroup of the subset -- the
// same partials summed in the same tile order, the same Q_BB and draws, so every copy makes the same
// decisions and computes the same delta' (the owner tile, tf, records the accept flags); (ii) adds
// W[:, B-1] delta'_{B-1} to its z rows; (iii) writes its partial dots of block B's columns.  B = 0
// also computes the tile's proposals; the launch after a subset's last block applies its moves.  The
// partials are double-buffered by block parity (launch B reads block B-1's while it writes block
// B's).  part: [S][2][nt][q][64].  A workgroup never waits on another, so nothing depends on
// co-residency, queue priority or CU masks.  The arithmetic and its order are k_sweep's /
// k_sweep_mg's (per-tile DPP dot reductions summed in tile order; per-wave column-residue FMA chains
// summed over the four waves): same bits.
template <int Q>
__global__ __launch_bounds__(256) void k_sweep_step(Model md, MatSet ms, int iter, int B, double* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  constexpr int q = Q;
  double* Qb = smem;                              // [q][SW_B*SW_B]
  double* gb = Qb + q * SW_B * SW_B;              // [q][SW_B]
  double* dacc = gb + q * SW_B;                   // [q][SW_B]
  double* red = dacc + q * SW_B;                  // [4][MK_NB]
  __shared__ double Ai[MK_QMAX * MK_QMAX];
  __shared__ int any_acc;
  const int nt = ms.nt;
  const int s = blockIdx.x / nt, t = blockIdx.x % nt;
  const int ns = md.n_s[s];
  const int tl = (ns - 1) / MK_NB;
  if (t > tl) return;
  const int n_blk = (ns + SW_B - 1) / SW_B;
  if (B > n_blk) return;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const long ld = ms.ld;
  const int r0 = MK_NB * t + 2 * lane;
  const long pstride = (long)nt * q * SW_B;       // one parity buffer of a subset
  double* ps = part + (long)s * 2 * pstride;
  if (tid < q * q) Ai[tid] = md.Ainv[(long)s * q * q + tid];
  if (B == 0) sweep_precompute(md, s, iter, MK_NB * t * q, min(MK_NB * (t + 1), ns) * q, tid, 256);
  d2 zr[Q];
#pragma unroll
  for (int h = 0; h < Q; ++h) zr[h] = *reinterpret_cast<const d2*>(md.z + ((long)s * q + h) * md.n_pad + r0);
  bool zdirty = false;
  if (B > 0) {
    const int bp = (B - 1) * SW_B, nbp = min(SW_B, ns - bp), tfp = bp / MK_NB;
    if (t >= tfp) {
      // ---- prologue: block B-1's MH steps (k_sweep_block), redundantly in every tile workgroup.
      // Q_BB by LDS-DMA (in flight while the partials load), the partials of tiles tfp .. tl all
      // loaded before they are summed in tile order (same values, same order: same bits)
      qbb_dma(md, ms, s, bp, Qb);
      const double* pb = ps + ((B - 1) & 1) * pstride;
      for (int e = tid; e < q * SW_B; e += 256) {
        const int h = e / SW_B, i = e % SW_B;
        const double* pp = pb + (long)h * SW_B + i;
        double pv[MK_NT_MAX_MG];
#pragma unroll
        for (int u = 0; u < MK_NT_MAX_MG; ++u) pv[u] = pp[(long)min(tfp + u, tl) * q * SW_B];
        double g = pv[0];
#pragma unroll
        for (int u = 1; u < MK_NT_MAX_MG; ++u)
          if (tfp + u <= tl) g = g + pv[u];
        gb[e] = g;
      }
      __builtin_amdgcn_s_waitcnt(0);   // this wave's Q_BB DMA has landed
      __syncthreads();
      // the update's first W panel streams in under the MH steps; each later panel under the
      // previous one's arithmetic (same values, same arithmetic: same bits)
      const double* Wu = ms.W + (long)s * q * (ld * ld) + (long)bp * ld + r0;
      d2 wa[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) wa[j] = *reinterpret_cast<const d2*>(Wu + (long)(wv + 4 * j) * ld);
      if (wv == 0) {
        const int anyl = sweep_block_mh_q<Q, false>(md, s, bp, nbp, gb, Qb, Ai, dacc, t == tfp);
        if (lane == 0) any_acc = anyl;
      }
      __syncthreads();
      // ---- z rows of tile t (rows >= bp) += W[:, B-1] delta'_{B-1}
      if (any_acc) {
        zdirty = true;
#pragma unroll
        for (int h = 0; h < Q; ++h) {
          d2 wb[16];
          if (h + 1 < Q) {
#pragma unroll
            for (int j = 0; j < 16; ++j)
              wb[j] = *reinterpret_cast<const d2*>(Wu + (long)(h + 1) * (ld * ld) + (long)(wv + 4 * j) * ld);
          }
          d2 sw = {0.0, 0.0};
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            const int i = wv + 4 * j;
            const double c = (i < nbp) ? dacc[h * SW_B + i] : 0.0;
            sw.x = fma(wa[j].x, c, sw.x);
            sw.y = fma(wa[j].y, c, sw.y);
          }
          if (h + 1 < Q) {
#pragma unroll
            for (int j = 0; j < 16; ++j) wa[j] = wb[j];
          }
          red[wv * MK_NB + 2 * lane] = sw.x;
          red[wv * MK_NB + 2 * lane + 1] = sw.y;
          __syncthreads();
          const double vx =
              ((red[2 * lane] + red[MK_NB + 2 * lane]) + red[2 * MK_NB + 2 * lane]) + red[3 * MK_NB + 2 * lane];
          const double vy = ((red[2 * lane + 1] + red[MK_NB + 2 * lane + 1]) + red[2 * MK_NB + 2 * lane + 1]) +
                            red[3 * MK_NB + 2 * lane + 1];
          __syncthreads();
#pragma unroll
          for (int hh = 0; hh < Q; ++hh) {
            if (hh != h) continue;
            if (r0 >= bp && r0 < ns) zr[hh].x += vx;
            if (r0 + 1 >= bp && r0 + 1 < ns) zr[hh].y += vy;
          }
        }
      }
    }
  }
  if (B < n_blk) {
    // ---- partial dots of tile t for block B's columns (tiles >= the block's first tile)
    const int b0 = B * SW_B;
    if (t >= b0 / MK_NB) {
      double* pb = ps + (B & 1) * pstride + (long)t * q * SW_B;
      const double* Wd = ms.W + (long)s * q * (ld * ld) + (long)b0 * ld + r0;
      d2 wa[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) wa[j] = *reinterpret_cast<const d2*>(Wd + (long)(wv + 4 * j) * ld);
#pragma unroll
      for (int h = 0; h < Q; ++h) {
        d2 wb[16];
        if (h + 1 < Q) {
#pragma unroll
          for (int j = 0; j < 16; ++j)
            wb[j] = *reinterpret_cast<const d2*>(Wd + (long)(h + 1) * (ld * ld) + (long)(wv + 4 * j) * ld);
        }
        const d2 zz = zr[h];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const double a0 = (r0 >= b0 && r0 < ns) ? wa[j].x * zz.x : 0.0;
          const double a1 = (r0 + 1 >= b0 && r0 + 1 < ns) ? wa[j].y * zz.y : 0.0;
          const double p = wave_sum_dpp(a0 + a1);
          if (lane == 0) pb[h * SW_B + wv + 4 * j] = p;
        }
        if (h + 1 < Q) {
#pragma unroll
          for (int j = 0; j < 16; ++j) wa[j] = wb[j];
        }
      }
    }
  }
  if (zdirty && wv == 0) {
#pragma unroll
    for (int h = 0; h < Q; ++h) *reinterpret_cast<d2*>(md.z + ((long)s * q + h) * md.n_pad + r0) = zr[h];
  }
  if (B == n_blk) {   // the subset's last block is done: apply this tile's accepted moves
    __syncthreads();
    sweep_apply(md, s, MK_NB * t, min(MK_NB * (t + 1), ns), Ai, tid, 256);
  }
}

template __global__ void k_sweep<1>(Model, MatSet, int, const int*, int*);
template __global__ void k_sweep<2>(Model, MatSet, int, const int*, int*);
template __global__ void k_sweep<3>(Model, MatSet, int, const int*, int*);
template __global__ void k_sweep<4>(Model, MatSet, int, const int*, int*);
template __global__ void k_sweep_mg<1>(Model, MatSet, int, double*, int*, int*, int*, int*, int);
template __global__ void k_sweep_mg<2>(Model, MatSet, int, double*, int*, int*, int*, int*, int);
template __global__ void k_sweep_mg<3>(Model, MatSet, int, double*, int*, int*, int*, int*, int);
template __global__ void k_sweep_mg<4>(Model, MatSet, int, double*, int*, int*, int*, int*, int);
#define MK_INST_STEP(Q) template __global__ void k_sweep_step<Q>(Model, MatSet, int, int, double*);
MK_INST_STEP(1)
MK_INST_STEP(2)
MK_INST_STEP(3)
MK_INST_STEP(4)

// ---------------------------------------------------------------- 5b. one-pass site sweep (default)
// The single-site w updates of spMvGLM (MK.R:80-84) with every column of W_h = L_h^-1 read from HBM
// exactly once per sweep.  One 256-thread workgroup per subset (a wave per SIMD: the per-site work every
// wave repeats is issued once per SIMD -- with 16 waves the site took ~3,000 cycles, issue-bound);
// thread t owns the row pairs 2t + 512k (k < KR = 4, or 8 beyond 2,048 rows) of every z_h and keeps
// them in registers for the whole sweep; the W columns
// stream through a register ring D sites ahead of use.  Site i, outcomes a = 0 .. q-1 in order:
//   every wave: p_h = sum over its rows of W_h[r,i] z_h[r] and s_h = sum of W_h[r,i]^2 (rows
//     i <= r < n_s), one 16-lane DPP row tree each, the four row sums into LDS slots
//     [i & 1][value][4 wave + row], then one s_barrier -- LDS writes drained (lgkmcnt) but no wait on
//     the W loads in flight;
//   every wave: g_h = the 16 row sums summed by a 16-lane DPP row tree (the same order in every
//     wave, so the same bits) and Q_ii,h = (R_h^-1)_ii the same way from s_h; the site's q MH
//     steps, computed redundantly by every wave with identical decisions (accept iff
//     log U <= dll - (d c + 0.5 d^2 dd), c = sum_h A^-1_ha g_h, dd = sum_h (A^-1_ha)^2 Q_ii,h), the
//     carry to the site's next outcome g_h += coef_h Q_ii,h, and on acceptance
//     z_h += coef_h W_h[:,i] from the registers that held the column (coef_h = d A^-1_ha).
// Against the 64-site-block kernels (k_sweep and its multi-workgroup forms): one W pass instead of
// two, no Q_BB tiles (k_qblocks is not launched for sessions on this kernel), one barrier per site.
// The arithmetic is the same chain; the dot products' summation order differs (rounding only).
// The loop body holds no memory-dependent control flow, so the W ring's loads stay in flight
// across steps (the compiler's wait counts are exact): the column loads are buffer loads whose
// skipped row pairs (the zero upper triangle, the border and padding rows) take an out-of-range
// offset and return zero without touching memory; the sites' proposals, likelihood differences
// and accept draws (sweep_precompute) and the accept flags live in LDS.
#define SS_T MK_SS_T
#define SS_W (SS_T / 64)   // four waves: one per SIMD, so the per-site work each wave repeats is issued once per SIMD
#define SS_OOB 0x7ffffff0u   // buffer offset beyond every W matrix: the load returns zero
// Sums of the 16-lane rows of a wave, in every lane of the row (quad xor 1, quad xor 2, half-row
// mirror, row mirror: the first four steps of wave_sum_dpp).
// (mov_dpp: every lane reads a lane of its own row, so no `old` value has to be materialised first)
template <int CTRL>
__device__ inline double dpp_f64_mov(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffffll), CTRL, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xf, 0xf, true);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ inline double row_sum_dpp(double x) {
  x += dpp_f64_mov<0xB1>(x);
  x += dpp_f64_mov<0x4E>(x);
  x += dpp_f64_mov<0x141>(x);
  x += dpp_f64_mov<0x140>(x);
  return x;
}
__device__ inline double rfl_f64(double v) {   // a wave-uniform VGPR value as a scalar
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readfirstlane((int)(b & 0xffffffffll));
  const int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
typedef unsigned int u4v __attribute__((ext_vector_type(4)));
// A compiler-only fence: keeps LDS accesses on their side of s_barrier without the hardware
// waits of a release fence (which would drain the W loads in flight).
#define SS_CFENCE() asm volatile("" ::: "memory")

// Dynamic LDS (sweep_site_lds_bytes): site data [3][n_s q] (proposal, likelihood difference, log
// accept draw; LN > 0: [4], the proposal as its coefficient d A^-1 plus half its square) + accept
// flags [n_s] (bit a: outcome a).

// The loop is issue-bound, not HBM- or latency-bound (profiles/r04/lean: a ring of 2, 6 or 8 columns
// per half instead of 4 changes nothing or loses; fewer instructions per site is what pays), so
// LN > 0 (q = 1 pairs, the default) is the lean form: fused-multiply-add dots, no row masks at use
// (W's upper triangle is zero in memory), the load offsets from per-thread row parts, and per site
// the move's coefficient d A^-1 and half its square precomputed -- 253 instead of 336 VALU
// instructions per pair; 1.12 -> 0.97 ms per sweep at 250 subsets, 0.92-0.94 ms with the sites' data
// read from registers (pair_step).
// P = 2 (q = 1, always with LN > 0): two sites per barrier.  The pair (i, i+1) exchanges five values --
// both dots, both squared norms and c = W[:,i] . W[:,i+1] = (R^-1)_{i+1,i} -- so site i+1's dot
// after a move at site i is g_{i+1} + coef_i c (the same carry the 64-site blocks make through Q_BB);
// half the barriers, one more reduction per pair.
template <int Q, int KR, int P = 1, int HH = 0, int LN = 0>
__global__ __launch_bounds__(SS_T) void k_sweep_site(Model md, MatSet ms, int iter) {
  constexpr bool FM = LN > 0;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  // ring: 2H columns (VGPRs: 8 H Q KR); NV values exchanged per site, four per row-sum round
  constexpr int q = Q, H = HH > 0 ? HH : ((16 / (Q * KR)) > 0 ? 16 / (Q * KR) : 1), NV = P == 2 ? 5 : 2 * Q;
  constexpr int NR = (NV + 3) / 4;
  static_assert(H >= 1 && NV <= 8, "q <= 4");   // instantiated for q <= 2 and (q = 3, KR = 1): no spills
  static_assert(P == 1 || (Q == 1 && H % 2 == 0), "site pairs: q = 1");
  __shared__ double part[2][NV][16];   // per value: the 16-lane row sums of the four waves
  __shared__ double Ai_s[MK_QMAX * MK_QMAX];
  const int s = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int ns = md.n_s[s];
  const int nq = ns * q;
  const long ld = ms.ld;
  double* sd_dl = smem;
  double* sd_dll = smem + nq;
  double* sd_lgu = smem + 2 * nq;
  double* sd_d2 = smem + 3 * nq;   // LN: 0.5 (d A^-1)^2 (sd_dl then holds d A^-1)
  int* sflag = reinterpret_cast<int*>(smem + (FM ? 4 : 3) * nq);
  double* z = md.z + (long)s * q * md.n_pad;
  if (tid < q * q) Ai_s[tid] = md.Ainv[(long)s * q * q + tid];
  {   // the sites' data into LDS (sweep_precompute's values; the proposals also to sw_delta for sweep_apply)
    const Key key = subset_key(md, s);
    const double* y = md.y + (long)s * md.Np;
    const double* wt = md.wt + (long)s * md.Np;
    const double* eta = md.eta + (long)s * md.Np;
    const double* tune = md.tune + (long)s * md.n_mh_max + md.o_w;
    double* gdl = md.sw_delta + (long)s * md.Np;
    for (int k = tid; k < nq; k += SS_T) {
      const int j = md.o_w + k;
      const double d = exp(tune[k]) * proposal_normal(key, j, iter);
      if constexpr (FM) {   // q = 1: the site's move on z (coefficient of its W column) and half its square
        const double cf = d * md.Ainv[(long)s];
        sd_dl[k] = cf;
        sd_d2[k] = 0.5 * cf * cf;
      } else {
        sd_dl[k] = d;
      }
      gdl[k] = d;
      sd_dll[k] = loglik_term(y[k], wt[k], eta[k] + d, md.link) - loglik_term(y[k], wt[k], eta[k], md.link);
      sd_lgu[k] = accept_log_uniform(key, j, iter);
    }
    for (int k = tid; k < ns; k += SS_T) sflag[k] = 0;
  }
  __syncthreads();
  double ai[Q * Q];
#pragma unroll
  for (int e = 0; e < Q * Q; ++e) ai[e] = Ai_s[e];
  d2 zr[KR][Q];
#pragma unroll
  for (int k = 0; k < KR; ++k) {
    const int r0 = 2 * tid + 2 * SS_T * k;
#pragma unroll
    for (int h = 0; h < Q; ++h)
      zr[k][h] = (r0 < md.n_pad) ? *reinterpret_cast<const d2*>(z + (long)h * md.n_pad + r0) : d2{0.0, 0.0};
  }
  __amdgpu_buffer_rsrc_t rs[Q];
#pragma unroll
  for (int h = 0; h < Q; ++h)
    rs[h] = __builtin_amdgcn_make_buffer_rsrc((void*)(ms.W + ((long)s * q + h) * (ld * ld)), (short)0,
                                              (int)(ld * ld * 8), 0x00020000);
  // column c of every W_h for this thread's rows; pairs wholly outside rows c <= r < n_s (the upper
  // triangle, the border and padding rows) are not fetched and read as zero.  The rest of the mask
  // is applied where the column is used (a select right after the load would wait for it).
  // FM (lean form, q = 1 pairs): the row part of the offset and the border-row factor once per thread
  unsigned rb[KR];
  double ym[KR];
#pragma unroll
  for (int k = 0; k < KR; ++k) {
    const int r0 = 2 * tid + 2 * SS_T * k;
    rb[k] = r0 < ns ? (unsigned)(r0 * 8) : 0x40000000u;   // rows past n_s: beyond every W (no wrap)
    ym[k] = (r0 + 1 < ns) ? 1.0 : 0.0;
  }
  auto load_col = [&](int c, d2 (&w)[KR][Q]) {
    const unsigned cb = c < ns ? (unsigned)((long)c * ld * 8) : 0x40000000u;
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      const int r0 = 2 * tid + 2 * SS_T * k;
      const bool any = c < ns && r0 + 1 >= c && r0 < ns;
      const unsigned off = FM ? ((r0 + 1 >= c) ? cb + rb[k] : SS_OOB) : (any ? (unsigned)(((long)c * ld + r0) * 8) : SS_OOB);
#pragma unroll
      for (int h = 0; h < Q; ++h)
        w[k][h] = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(rs[h], (int)off, 0, 0));
    }
  };
  // The ring in two halves of H columns, used and refilled in turn: while the sites of one half
  // run, the other half's columns are in flight (issued H sites earlier).  A loop iteration holds
  // both halves, so at its back edge only the half issued H sites ago is outstanding -- the wait
  // the compiler places at the loop head (it does not track loads across the back edge) finds
  // them arrived instead of stalling on a column issued one site earlier.
  auto step = [&](const int i, d2 (&w)[KR][Q]) {
    // Straight-line body (no early exit): every path issues the same loads, so the compiler's
    // wait counts stay exact across the steps and the loop's back edge.  Steps past the last site
    // (i >= n_s, in the last round) see an all-zero column and reject.
    const bool live = i < ns;
    const int ic = live ? i : ns - 1;
    // the site's data (uniform LDS reads, issued ahead of the reductions)
    double dl_[Q], dll_[Q], lg_[Q];
#pragma unroll
    for (int a = 0; a < Q; ++a) {
      dl_[a] = sd_dl[ic * q + a];
      dll_[a] = sd_dll[ic * q + a];
      lg_[a] = live ? sd_lgu[ic * q + a] : __builtin_huge_val();
    }
    // ---- column i masked to rows i <= r < n_s; the wave's partial dots and squared norms
    d2 wc[KR][Q];
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      const int r0 = 2 * tid + 2 * SS_T * k;
#pragma unroll
      for (int h = 0; h < Q; ++h) {
        wc[k][h].x = (r0 >= i) ? w[k][h].x : 0.0;
        wc[k][h].y = (r0 + 1 >= i && r0 + 1 < ns) ? w[k][h].y : 0.0;
      }
    }
    double v[NV];
#pragma unroll
    for (int h = 0; h < Q; ++h) {
      double pd = 0.0, sq = 0.0;
#pragma unroll
      for (int k = 0; k < KR; ++k) {
        if constexpr (FM) {
          pd = fma(wc[k][h].y, zr[k][h].y, fma(wc[k][h].x, zr[k][h].x, pd));
          sq = fma(wc[k][h].y, wc[k][h].y, fma(wc[k][h].x, wc[k][h].x, sq));
        } else {
          pd += wc[k][h].x * zr[k][h].x + wc[k][h].y * zr[k][h].y;
          sq += wc[k][h].x * wc[k][h].x + wc[k][h].y * wc[k][h].y;
        }
      }
      v[h] = pd;
      v[Q + h] = sq;
    }
#pragma unroll
    for (int e = 0; e < NV; ++e) v[e] = row_sum_dpp(v[e]);
    SS_CFENCE();
    if ((lane & 15) == 0) {
#pragma unroll
      for (int e = 0; e < NV; ++e) part[i & 1][e][4 * wv + (lane >> 4)] = v[e];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    SS_CFENCE();
    // ---- every wave: the workgroup sums (row e of 16 lanes: value e over the 16 waves)
    double tot[4 * NR];
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) {
      const int e_l = 4 * rr + (lane >> 4);
      const double pv = part[i & 1][e_l < NV ? e_l : 0][lane & 15];
      const double rsum = row_sum_dpp(e_l < NV ? pv : 0.0);
#pragma unroll
      for (int e = 0; e < 4; ++e) tot[4 * rr + e] = rlane_u(rsum, 16 * e);
    }
    double g[Q], qd[Q];
#pragma unroll
    for (int h = 0; h < Q; ++h) {
      g[h] = tot[h];
      qd[h] = tot[Q + h];
    }
    // ---- the site's MH steps (outcomes in order) and the z update
    int fl = 0;
#pragma unroll
    for (int a = 0; a < Q; ++a) {
      const double d = rfl_f64(dl_[a]);
      double c = ai[a * q] * g[0];
#pragma unroll
      for (int h = 1; h < Q; ++h) c += ai[h + a * q] * g[h];
      double dd = 0.0;
#pragma unroll
      for (int h = 0; h < Q; ++h) dd += (ai[h + a * q] * ai[h + a * q]) * qd[h];
      const double ratio = rfl_f64(dll_[a]) - (d * c + 0.5 * d * d * dd);
      if (rfl_f64(lg_[a]) <= ratio) {   // uniform
#pragma unroll
        for (int h = 0; h < Q; ++h) {
          const double coef = d * ai[h + a * q];
          g[h] += coef * qd[h];
#pragma unroll
          for (int k = 0; k < KR; ++k) {
            zr[k][h].x = fma(coef, wc[k][h].x, zr[k][h].x);
            zr[k][h].y = fma(coef, wc[k][h].y, zr[k][h].y);
          }
        }
        fl |= 1 << a;
      }
    }
    if (tid == 0 && live) sflag[i] = fl;
  };
  // sites i, i + 1 (q = 1): one exchange, the carry of site i's move into site i + 1's dot
  // LN: the sites' data in registers, lane l holding site 64 b + l of the current block of 64 (refilled
  // from LDS at each block's first pair); a pair reads its two sites with v_readlane at a uniform lane
  // index instead of LDS reads, address arithmetic and readfirstlanes.  Sites past n_s: accept draw +inf.
  double vcf = 0.0, vdll = 0.0, vh = 0.0, vlg = __builtin_huge_val();
  auto pair_step = [&](const int i, d2 (&w0)[KR][Q], d2 (&w1)[KR][Q]) {
    static_assert(P == 1 || FM, "site pairs: the lean form");
    {
      if ((i & 63) == 0) {   // uniform
        const int kk = i + lane;
        const bool lv = kk < ns;
        const int kc = lv ? kk : ns - 1;
        vcf = sd_dl[kc];
        vdll = sd_dll[kc];
        vh = sd_d2[kc];
        vlg = lv ? sd_lgu[kc] : __builtin_huge_val();
      }
    }
    const bool live0 = i < ns, live1 = i + 1 < ns;
    d2 c0[KR], c1[KR];
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      {
        // No row masks but one: i is even, so the loads already return zero for every row pair wholly
        // above column i's diagonal; the one upper element left, W[i, i+1] (column i+1 in the pair
        // starting at row i), is zero in memory (W's upper triangle is zeroed at session creation and
        // store_tile_lw, k_inv_copydiag, k_inv_level write lower tiles and zero-upper diagonal tiles)
        // and is masked here anyway -- one select per pair, so no future writer of W's upper triangle
        // can reach z.  Row n_s (the border row, nonzero in W) sits in a loaded pair only
        // for odd n_s: LN = 1 drops it with a factor 0; LN = 2 is launched only when every subset's n_s
        // is even.
        c0[k].x = w0[k][0].x;
        c0[k].y = LN == 1 ? w0[k][0].y * ym[k] : w0[k][0].y;
        c1[k].x = (2 * tid + 2 * SS_T * k == i) ? 0.0 : w1[k][0].x;
        c1[k].y = LN == 1 ? w1[k][0].y * ym[k] : w1[k][0].y;
      }
    }
    double v[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      v[0] = fma(c0[k].y, zr[k][0].y, fma(c0[k].x, zr[k][0].x, v[0]));
      v[1] = fma(c1[k].y, zr[k][0].y, fma(c1[k].x, zr[k][0].x, v[1]));
      v[2] = fma(c0[k].y, c0[k].y, fma(c0[k].x, c0[k].x, v[2]));
      v[3] = fma(c1[k].y, c1[k].y, fma(c1[k].x, c1[k].x, v[3]));
      v[4] = fma(c0[k].y, c1[k].y, fma(c0[k].x, c1[k].x, v[4]));
    }
#pragma unroll
    for (int e = 0; e < 5; ++e) v[e] = row_sum_dpp(v[e]);
    const int par = (i >> 1) & 1;
    SS_CFENCE();
    if ((lane & 15) == 0) {
#pragma unroll
      for (int e = 0; e < 5; ++e) part[par][e][4 * wv + (lane >> 4)] = v[e];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    SS_CFENCE();
    double tot[8];
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
      const int e_l = 4 * rr + (lane >> 4);
      const double pv = part[par][e_l < 5 ? e_l : 0][lane & 15];
      const double rsum = row_sum_dpp(e_l < 5 ? pv : 0.0);
#pragma unroll
      for (int e = 0; e < 4; ++e) tot[4 * rr + e] = rlane_u(rsum, 16 * e);
    }
    int f0 = 0, f1 = 0;
    double coef0 = 0.0, coef1 = 0.0;
    {   // ratio = dll - (cf g + 0.5 cf^2 Q_ii), cf = d A^-1 (precomputed per site)
      const int l0 = i & 63, l1 = l0 + 1;
      const double cf0 = rlane_u(vcf, l0), cf1 = rlane_u(vcf, l1);
      const double h0 = rlane_u(vh, l0), h1 = rlane_u(vh, l1);
      if (rlane_u(vlg, l0) <= rlane_u(vdll, l0) - fma(cf0, tot[0], h0 * tot[2])) {
        coef0 = cf0;
        f0 = 1;
      }
      const double g1 = fma(coef0, tot[4], tot[1]);
      if (rlane_u(vlg, l1) <= rlane_u(vdll, l1) - fma(cf1, g1, h1 * tot[3])) {
        coef1 = cf1;
        f1 = 1;
      }
    }
    if (f0 | f1) {
#pragma unroll
      for (int k = 0; k < KR; ++k) {
        zr[k][0].x = fma(coef1, c1[k].x, fma(coef0, c0[k].x, zr[k][0].x));
        zr[k][0].y = fma(coef1, c1[k].y, fma(coef0, c0[k].y, zr[k][0].y));
      }
    }
    if (tid == 0 && live0) sflag[i] = f0;
    if (tid == 0 && live1) sflag[i + 1] = f1;
  };
  d2 wa[H][KR][Q], wb[H][KR][Q];
#pragma unroll
  for (int u = 0; u < H; ++u) load_col(u, wa[u]);
  for (int i0 = 0; i0 < ns; i0 += 2 * H) {
#pragma unroll
    for (int u = 0; u < H; ++u) load_col(i0 + H + u, wb[u]);
    if constexpr (P == 2) {
#pragma unroll
      for (int u = 0; u < H; u += 2) pair_step(i0 + u, wa[u], wa[u + 1]);
    } else {
#pragma unroll
      for (int u = 0; u < H; ++u) step(i0 + u, wa[u]);
    }
#pragma unroll
    for (int u = 0; u < H; ++u) load_col(i0 + 2 * H + u, wa[u]);
    if constexpr (P == 2) {
#pragma unroll
      for (int u = 0; u < H; u += 2) pair_step(i0 + H + u, wb[u], wb[u + 1]);
    } else {
#pragma unroll
      for (int u = 0; u < H; ++u) step(i0 + H + u, wb[u]);
    }
  }
  // ---- write back own z rows; the accept flags to sw_acc; apply accepted moves
#pragma unroll
  for (int k = 0; k < KR; ++k) {
    const int r0 = 2 * tid + 2 * SS_T * k;
    if (r0 < md.n_pad) {
#pragma unroll
      for (int h = 0; h < Q; ++h) *reinterpret_cast<d2*>(z + (long)h * md.n_pad + r0) = zr[k][h];
    }
  }
  __syncthreads();
  int* sacc = md.sw_acc + (long)s * md.Np;
  for (int k = tid; k < nq; k += SS_T) sacc[k] = (sflag[k / q] >> (k % q)) & 1;
  __syncthreads();
  sweep_apply(md, s, 0, ns, Ai_s, tid, SS_T);
}
template __global__ void k_sweep_site<2, 4, 1>(Model, MatSet, int);
template __global__ void k_sweep_site<2, 8, 1>(Model, MatSet, int);
template __global__ void k_sweep_site<3, 4, 1>(Model, MatSet, int);
template __global__ void k_sweep_site<1, 4, 2, 0, 1>(Model, MatSet, int);
template __global__ void k_sweep_site<1, 4, 2, 0, 2>(Model, MatSet, int);
template __global__ void k_sweep_site<1, 8, 2, 0, 1>(Model, MatSet, int);
template __global__ void k_sweep_site<1, 8, 2, 0, 2>(Model, MatSet, int);

// ---------------------------------------------------------------- 6. record / adapt
__global__ __launch_bounds__(64) void k_record(Model md, int iter) {
  const int s = blockIdx.x * 64 + threadIdx.x;
  if (s >= md.S) return;
  const int q = md.q;
  double* out = md.samples + ((long)s * md.n_samples + iter) * md.P;
  for (int j = 0; j < md.p; ++j) out[j] = md.beta[(long)s * md.p + j];
  const double* th = md.theta + (long)s * md.n_theta;
  double A[16];
  tri_to_A(th, q, A);
  int k = md.p;
  for (int c = 0; c < q; ++c)
    for (int r = c; r < q; ++r) {
      double v = 0.0;
      for (int m = 0; m < q; ++m) v += A[r + m * q] * A[c + m * q];
      out[k++] = v;
    }
  for (int h = 0; h < q; ++h) out[k++] = logit_inv(th[md.ntri + h], md.phi_a[h], md.phi_b[h]);
  if (md.cov_model == MK_COV_MATERN)
    for (int h = 0; h < q; ++h) out[k++] = logit_inv(th[md.ntri + q + h], md.nu_a[h], md.nu_b[h]);
}

__global__ __launch_bounds__(256) void k_record_w(Model md, int iter) {
  const int s = blockIdx.y;
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= md.Np) return;
  md.w_samples[((long)s * md.n_samples + iter) * md.Np + k] = md.w[(long)s * md.Np + k];
}

__global__ __launch_bounds__(256) void k_adapt(Model md, int b) {
  __shared__ double red[8];
  const int s = blockIdx.x, tid = threadIdx.x;
  const int n_mh = md.o_w + md.n_s[s] * md.q;
  const double step = (b > 0) ? fmin(0.01, 1.0 / sqrt((double)b)) : 0.01;
  double* tune = md.tune + (long)s * md.n_mh_max;
  double* acc = md.acc + (long)s * md.n_mh_max;
  const int nrep = md.o_w + 1;
  double* hist = md.acc_hist + ((long)s * md.n_batch + b) * nrep;
  double wsum = 0.0;
  for (int j = tid; j < n_mh; j += 256) {
    const double rate = acc[j] / md.batch_length;
    if (j < md.o_w) hist[j] = rate; else wsum += rate;
    tune[j] = (rate > md.accept_rate) ? tune[j] + step : tune[j] - step;
    acc[j] = 0.0;
  }
  const double tot = block_sum<256>(wsum, red);
  if (tid == 0) hist[md.o_w] = tot / (md.n_s[s] * md.q);
}

// ---------------------------------------------------------------- 7. kriging draw (kept iterations)
// w*_t = A (m_t + diag(sqrt(1 - s_h(t))) z*_t),  m_{t,h} = rho_h(t)' R_h^-1 u_h = X_{h,t} . z_h
// (spPredict per-site marginal; X_h = W_h P_h^T from the last (phi, nu) change).
__global__ __launch_bounds__(256) void k_pred_draw(Model md, int iter, int kidx) {
  const int per = (md.n_test + 3) / 4;
  const int s = blockIdx.x / per;
  const int t = (blockIdx.x % per) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= md.n_test) return;
  const int q = md.q, ns = md.n_s[s];
  double mean[MK_QMAX], sd[MK_QMAX];
  for (int h = 0; h < q; ++h) {
    const long sh = (long)s * q + h;
    const double* xk = md.XK + (sh * md.n_test_pad + t) * md.n_pad;
    const double* zh = md.z + sh * md.n_pad;
    // 16-byte row pairs, 4 pairs per lane in flight (unconditional loads clamped inside the
    // n_pad rows, rows >= n_s masked by selects); fixed summation order
    const int np2 = md.n_pad >> 1;
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    for (int base = 0; base < ns; base += 512) {
      d2 xv[4], zv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int pr = min((base >> 1) + u * 64 + lane, np2 - 1);
        xv[u] = *reinterpret_cast<const d2*>(xk + 2 * pr);
        zv[u] = *reinterpret_cast<const d2*>(zh + 2 * pr);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int r = base + 2 * (u * 64 + lane);
        a[u] += (r < ns) ? xv[u].x * zv[u].x : 0.0;
        a[u] += (r + 1 < ns) ? xv[u].y * zv[u].y : 0.0;
      }
    }
    double acc = (a[0] + a[1]) + (a[2] + a[3]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    mean[h] = acc;
    sd[h] = sqrt(fmax(1.0 - md.s_pred[sh * md.n_test_pad + t], 0.0));
  }
  if (lane == 0) {
    const Key key = subset_key(md, s);
    double v[MK_QMAX];
    for (int h = 0; h < q; ++h) v[h] = mean[h] + sd[h] * predict_normal(key, (md.t_off + t) * q + h, iter);
    const double* A = md.A_full + (long)s * q * q;
    double* out = md.w_pred + ((long)s * md.n_kept + kidx) * q * md.n_test + (long)t * q;
    for (int a = 0; a < q; ++a) {
      double o = 0.0;
      for (int h = 0; h < q; ++h) o += v[h] * A[a + h * q];
      out[a] = o;
    }
  }
}

// Tiled replay, q = 1: the draws of kept states [run_start[s], j_end) of the listed subsets (plist;
// nullptr: every subset) from X as it stands -- the states of one phi run share X, so it is read once
// per 4 states instead of once per state.  State j is window state j (iteration kept0 + k_lo + j);
// its z and A are the recorded ones (kz, kA).  The per-state arithmetic is k_pred_draw's -- the same
// loads, the same order of the two products per row pair, the same reduction -- so the same bits.
__global__ __launch_bounds__(256) void k_pred_draw_runs(Model md, const double* __restrict__ kz,
                                                        const double* __restrict__ kA, int k_lo,
                                                        const int* __restrict__ plist, const int* __restrict__ pcount,
                                                        const int* __restrict__ run_start, int j_end) {
  const int per = (md.n_test + 3) / 4;
  const int e = blockIdx.x / per;
  if (e >= (plist ? *pcount : md.S)) return;
  const int s = plist ? plist[e] : e;   // q = 1: the pair is the subset
  const int t = (blockIdx.x % per) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int j0 = run_start[s];
  if (t >= md.n_test || j0 >= j_end) return;
  const int ns = md.n_s[s];
  const double* xk = md.XK + ((long)s * md.n_test_pad + t) * md.n_pad;
  const double sd = sqrt(fmax(1.0 - md.s_pred[(long)s * md.n_test_pad + t], 0.0));
  const int np2 = md.n_pad >> 1;
  const Key key = subset_key(md, s);
  for (int jg = j0; jg < j_end; jg += 4) {
    const int nr = min(4, j_end - jg);
    double a[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int u = 0; u < 4; ++u) a[r][u] = 0.0;
    for (int base = 0; base < ns; base += 512) {
      d2 xv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int pr = min((base >> 1) + u * 64 + lane, np2 - 1);
        xv[u] = *reinterpret_cast<const d2*>(xk + 2 * pr);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (r >= nr) break;
        const double* zh = kz + ((long)(k_lo + jg + r) * md.S + s) * md.n_pad;
        d2 zv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int pr = min((base >> 1) + u * 64 + lane, np2 - 1);
          zv[u] = *reinterpret_cast<const d2*>(zh + 2 * pr);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int row = base + 2 * (u * 64 + lane);
          a[r][u] += (row < ns) ? xv[u].x * zv[u].x : 0.0;
          a[r][u] += (row + 1 < ns) ? xv[u].y * zv[u].y : 0.0;
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (r >= nr) break;
      double acc = (a[r][0] + a[r][1]) + (a[r][2] + a[r][3]);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
      if (lane == 0) {
        const int j = jg + r, k = k_lo + j;
        const double v = acc + sd * predict_normal(key, md.t_off + t, md.kept0 + k);
        double o = 0.0;
        o += v * kA[(long)k * md.S + s];
        md.w_pred[((long)s * md.n_kept + j) * md.n_test + t] = o;
      }
    }
  }
}

// run_start[s] = j for the listed subsets (their X is refreshed at window state j).
__global__ __launch_bounds__(256) void k_run_start(const int* __restrict__ plist, const int* __restrict__ pcount,
                                                   int* run_start, int j) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e < *pcount) run_start[plist[e]] = j;
}

// ---------------------------------------------------------------- 8. type-7 quantiles (MK.R:88-89)
// One workgroup per (subset, column): bitonic sort of the kept values in LDS (dynamic: the next
// power of two >= n_rows doubles, at most MK_QUANT_MAX = 128 KB), then R's quantile.default type 7:
// (1-h) x[lo] + h x[hi] (no FMA contraction).
__global__ __launch_bounds__(256) void k_quantiles(const double* __restrict__ data, long subset_stride, long row_stride,
                                                   int n_rows, int n_cols, const double* __restrict__ probs, int n_probs,
                                                   double* __restrict__ out /* [S][n_cols][n_probs] */) {
  extern __shared__ double v[];
  const int s = blockIdx.x / n_cols, c = blockIdx.x % n_cols;
  const double* src = data + (long)s * subset_stride + c;
  int n2 = 1;
  while (n2 < n_rows) n2 <<= 1;
  for (int r = threadIdx.x; r < n2; r += 256) v[r] = (r < n_rows) ? src[(long)r * row_stride] : INFINITY;
  __syncthreads();
  for (int size = 2; size <= n2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < n2 / 2; t += 256) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool up = ((lo & size) == 0);
        const double a = v[lo], b = v[hi];
        if ((a > b) == up) { v[lo] = b; v[hi] = a; }
      }
      __syncthreads();
    }
  }
  double* o = out + ((long)s * n_cols + c) * n_probs;
  for (int l = threadIdx.x; l < n_probs; l += 256) {
    const double index = 1.0 + (double)(n_rows - 1) * probs[l];
    const double flo = floor(index), fhi = ceil(index);
    const int lo = (int)flo, hi = (int)fhi;
    const double qlo = v[lo - 1], qhi = v[hi - 1];
    const double hh = index - flo;
    o[l] = (index > flo && qhi != qlo) ? (1.0 - hh) * qlo + hh * qhi : qlo;
  }
}

// ---------------------------------------------------------------- 9. combine (MK.R:123-133)
// out = (((g_0 + g_1) + g_2) + ...) / K : the reference's sequential order (mean = 0: the sum only,
// one shard's term of the combine).
__global__ __launch_bounds__(256) void k_combine(const double* __restrict__ grids, int K, long G, double* __restrict__ out,
                                                 int mean) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= G) return;
  double acc = grids[e];
  for (int k = 1; k < K; ++k) acc = acc + grids[(long)k * G + e];
  out[e] = mean ? acc / K : acc;
}

// ---------------------------------------------------------------- 10. tiled kriging support
// Kept iteration kidx: record z, theta and A of every subset ([n_kept][S_all][...] records).
__global__ __launch_bounds__(256) void k_record_kept(Model md, int kidx) {
  const int s = blockIdx.x, q = md.q;
  const long row = (long)kidx * md.S_all + s;
  for (int i = threadIdx.x; i < q * md.n_pad; i += 256) md.kz[row * q * md.n_pad + i] = md.z[(long)s * q * md.n_pad + i];
  if (threadIdx.x < md.n_theta) md.kth[row * md.n_theta + threadIdx.x] = md.theta[(long)s * md.n_theta + threadIdx.x];
  if (threadIdx.x < q * q) md.kA[row * q * q + threadIdx.x] = md.A_full[(long)s * q * q + threadIdx.x];
}

// Replaying kept sample k (md.theta = its record): the (subset, outcome) pairs whose (phi_h, nu_h)
// differ from sample k-1 (all of them when th_prev == nullptr).  Outputs, in subset order:
// per outcome h the subset list slist[h*S .. ] / scount[h] (candidate + Cholesky launches), and
// the pair list (s*q + h) plist / pcount (inverse + kriging refresh).  One 256-thread block.
__global__ __launch_bounds__(256) void k_kept_dirty(Model md, const double* __restrict__ th_prev, int* slist,
                                                    int* scount, int* plist, int* pcount) {
  __shared__ int wc[4];
  __shared__ int base, pbase;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int q = md.q, S = md.S;
  if (threadIdx.x == 0) pbase = 0;
  for (int h = 0; h < q; ++h) {
    if (threadIdx.x == 0) base = 0;
    __syncthreads();
    for (int c0 = 0; c0 < S; c0 += 256) {
      const int s = c0 + threadIdx.x;
      int d = 0;
      if (s < S) {
        const double* th = md.theta + (long)s * md.n_theta;
        if (!th_prev) {
          d = 1;
        } else {
          const double* tp = th_prev + (long)s * md.n_theta;
          d = th[md.ntri + h] != tp[md.ntri + h];
          if (md.cov_model == MK_COV_MATERN) d |= th[md.ntri + q + h] != tp[md.ntri + q + h];
        }
      }
      const unsigned long long bal = __ballot(d);
      const int before = __popcll(bal & ((1ull << lane) - 1ull));
      if (lane == 0) wc[wv] = __popcll(bal);
      __syncthreads();
      int off = 0;
      for (int k = 0; k < wv; ++k) off += wc[k];
      if (d) {
        slist[h * S + base + off + before] = s;
        plist[pbase + base + off + before] = s * q + h;
      }
      __syncthreads();
      if (threadIdx.x == 0) base += wc[0] + wc[1] + wc[2] + wc[3];
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      scount[h] = base;
      pbase += base;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) *pcount = pbase;
}

// The freshly factored candidates of the listed pairs become the current factors.
__global__ __launch_bounds__(256) void k_flip_pairs(MatSet ms, const int* __restrict__ plist, const int* __restrict__ pcount) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e < *pcount) ms.cur[plist[e]] ^= 1;
}

// ---------------------------------------------------------------- 11. phi-interpolated tiled kriging
// (exponential, q = 1; mk_api.hip predict_tile_cheb).  spPredict's draw for kept state k at test site t
// is w*_k(t) = A_k (m_k(t) + sqrt(1 - s(t; phi_k)) e), with m_k(t) = rho_t(phi_k)' R(phi_k)^-1 u_k and
// s(t; phi) = rho_t(phi)' R(phi)^-1 rho_t(phi).  The exact replay recomputes X = W P^T, i.e. s at every
// phi the chain visited (0.39 refreshes per kept state at configs[4]).  s is an analytic function of
// phi on the kept range: it is interpolated instead from exact values at Chebyshev nodes of that range
// (barycentric form, nodes of the first kind), and every tile checks the interpolant against exact
// values at the range's two ends and its middle before any draw uses it.  The mean needs no X:
// m_k(t) = rho_t(phi_k)' g_k with g_k = W_k' z_k (z_k recorded, W_k the state's inverse factor).

// |s_i - t| for the interpolated draws' means: a square root from the hardware reciprocal square-root
// estimate and one Newton-Raphson step (x r, then the residual correction, as the library's rounding
// sequence does without its denormal scaling -- squared distances here are >= 1e-24 or 0); within an ulp
// or two of the correctly rounded root, which only enters rho = exp(-phi d).
__device__ inline double dist_fast(double x0, double y0, double x1, double y1) {
  const double dx = x0 - x1, dy = y0 - y1;
  const double x = fma(dx, dx, dy * dy);
  const double r = __builtin_amdgcn_rsq(x);
  double g = x * r, h = 0.5 * r;
  const double e = fma(-g, h, 0.5);
  g = fma(g, e, g);
  h = fma(h, e, h);
  g = fma(fma(-g, g, x), h, g);
  return x > 0.0 ? g : 0.0;
}

// phis[j][s] = phi of record j (th: [n][S][n_theta] records): the candidate assembly's formula
// (candidate_theta, which = 2), so a record's phi here is bit for bit the one its factor used.
__global__ __launch_bounds__(256) void k_kept_phi(Model md, const double* __restrict__ th, int n,
                                                  double* __restrict__ phis) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long)n * md.S) return;
  phis[e] = logit_inv(th[e * md.n_theta + md.ntri], md.phi_a[0], md.phi_b[0]);
}

// g = W' z for every subset (q = 1): g_i = sum_{i <= r < n_s} W[r, i] z_r, one wave per column i
// (W column-major: the wave's loads are contiguous); g_i = 0 for i >= n_s.  Stored state-minor,
// Gt[s][i][j] (j: the window state, nkp per row), so a pass over 8 states reads 64 contiguous bytes.
__global__ __launch_bounds__(256) void k_krig_g(Model md, MatSet ms, const double* __restrict__ z,
                                                double* __restrict__ Gt, int j, int nkp) {
  const int per = md.n_pad / 4;
  const int s = blockIdx.x / per;
  const int i = (blockIdx.x % per) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int ns = md.n_s[s];
  const long ld = ms.ld;
  const double* Wc = ms.W + (long)s * ld * ld + (long)i * ld;
  const double* zs = z + (long)s * md.n_pad;
  double a0 = 0.0, a1 = 0.0;
  if (i < ns) {
    for (int r = i + lane; r < ns; r += 128) {
      a0 += Wc[r] * zs[r];
      if (r + 64 < ns) a1 += Wc[r + 64] * zs[r + 64];
    }
  }
  double acc = a0 + a1;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (lane == 0) Gt[((long)s * md.n_pad + i) * nkp + j] = (i < ns) ? acc : 0.0;
}

// s(t; phi) of subset s from its nodes (slots 0 .. nc-1): barycentric interpolation of the second
// kind with the Chebyshev weights (-1)^i sin((2i + 1) pi / (2 nc)) (wts[s][i]); a node's own value
// at its phi.
__device__ inline double cheb_s(const ChebK& c, int S, int s, long t, double phi) {
  const int nc = c.nc[s];
  const double* w = c.wts + (long)s * MK_CHEB_MAX;
  double num = 0.0, den = 0.0;
  for (int i = 0; i < nc; ++i) {
    const double f = c.Sn[((long)i * S + s) * c.T_pad + t];
    const double d = phi - c.nphi[(long)i * S + s];
    if (d == 0.0) return f;
    const double ci = w[i] / d;
    num += ci * f;
    den += ci;
  }
  return num / den;
}

// The interpolant against the exact values at the check slots nc .. nc+nchk-1 (the range's ends, its
// middle, its quarters): the largest |difference| over the tile's sites and subsets into *err (bit pattern of a
// non-negative double; a NaN counts as +inf).
__global__ __launch_bounds__(256) void k_cheb_check(Model md, ChebK c, unsigned long long* err) {
  __shared__ double red[4];
  const int nb = (md.n_test + 255) / 256;
  const int s = blockIdx.x / nb;
  const int t = (blockIdx.x % nb) * 256 + threadIdx.x;
  double e = 0.0;
  if (t < md.n_test) {
    const int nc = c.nc[s];
    for (int k = 0; k < c.nchk; ++k) {
      const int slot = nc + k;
      const double phi = c.nphi[(long)slot * md.S + s];
      const double ex = c.Sn[((long)slot * md.S + s) * c.T_pad + t];
      const double d = fabs(cheb_s(c, md.S, s, t, phi) - ex);
      if (!(d <= e)) e = (d != d) ? INFINITY : d;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) e = fmax(e, __shfl_xor(e, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = e;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double m = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
    atomicMax(err, (unsigned long long)__double_as_longlong(m));
  }
}

// The draws of the window's kept states j = 0 .. md.n_kept-1 (state k = k_lo + j) at the tile's sites,
// one thread per (subset, site), 8 states per pass over the subset's sites: the distance once per
// site and pass (dist_fast), rho_t(phi) = exp(-phi d) once per distinct phi among the 8 (consecutive
// states share phi while the chain stays), m_k(t) = sum_i rho_i g_k,i in site order (fma).  Gt [S][n_pad][nkp] and phit
// [S][nkp] are zero / last-phi padded to nkp (a multiple of 8), and with the coordinates they are read
// through scalar loads (uniform addresses).  The normal, the A factor and the output layout are
// k_pred_draw_runs' (q = 1).
__global__ __launch_bounds__(256) void k_pred_cheb_draw(Model md, ChebK c, const double* __restrict__ Gt,
                                                        const double* __restrict__ phit,
                                                        const double* __restrict__ coords,
                                                        const double* __restrict__ kA, int k_lo, int nkp) {
  const int nb = (md.n_test + 255) / 256;
  const int s = blockIdx.x / nb;
  const int t0 = (blockIdx.x % nb) * 256 + threadIdx.x;
  const bool act = t0 < md.n_test;
  const int t = act ? t0 : md.n_test - 1;
  const int S = md.S, n = md.n_kept, ns = md.n_s[s], np = md.n_pad;
  const double xt = md.coords_test[t], yt = md.coords_test[md.n_test_pad + t];
  const double* cx = coords + (long)s * 2 * np;
  const double* cy = cx + np;
  const double* ph = phit + (long)s * nkp;
  const double* gs = Gt + (long)s * np * nkp;
  const Key key = subset_key(md, s);
  for (int j0 = 0; j0 < n; j0 += 8) {
    double p[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) p[b] = ph[j0 + b];
    double a[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) a[b] = 0.0;
#pragma unroll 2
    for (int i = 0; i < ns; ++i) {
      const double d = dist_fast(cx[i], cy[i], xt, yt);
      const double* gi = gs + (long)i * nkp + j0;
      double e = exp(-p[0] * d);
      a[0] = fma(e, gi[0], a[0]);
#pragma unroll
      for (int b = 1; b < 8; ++b) {
        if (p[b] != p[b - 1]) e = exp(-p[b] * d);
        a[b] = fma(e, gi[b], a[b]);
      }
    }
    double sd = 0.0;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      if (j0 + b >= n) break;
      if (b == 0 || p[b] != p[b - 1]) sd = sqrt(fmax(1.0 - cheb_s(c, S, s, t, p[b]), 0.0));
      const int k = k_lo + j0 + b;
      const double v = a[b] + sd * predict_normal(key, md.t_off + t, md.kept0 + k);
      double o = 0.0;
      o += v * kA[(long)k * S + s];
      if (act) md.w_pred[((long)s * n + j0 + b) * md.n_test + t] = o;
    }
  }
}

// Fused kriging from the session's phi tables (mk_api.hip krig_tables; q = 1): what a kept iteration's
// draws read, captured after its sweep (z, phi, A), so they can run on a side stream while the next
// iteration's A step, decision and inverse move on.
__global__ __launch_bounds__(256) void k_kt_snap(Model md, double* __restrict__ zs, double* __restrict__ phis,
                                                 double* __restrict__ As) {
  const int s = blockIdx.x;
  for (int i = threadIdx.x; i < md.n_pad; i += 256) zs[(long)s * md.n_pad + i] = md.z[(long)s * md.n_pad + i];
  if (threadIdx.x == 0) {
    phis[s] = logit_inv(md.theta[(long)s * md.n_theta + md.ntri], md.phi_a[0], md.phi_b[0]);
    As[s] = md.A_full[s];
  }
}

// k_pred_draw's draw (kept iteration `iter`, record kidx) with s(t; phi) interpolated from the tables and
// the mean m(t) = rho_t(phi)' g, g = W' z (k_krig_g over the snapshot), instead of X = W P^T refreshed
// wherever phi changed.  One thread per (subset, site).
__global__ __launch_bounds__(256) void k_pred_tab_draw(Model md, ChebK c, const double* __restrict__ g,
                                                       const double* __restrict__ coords,
                                                       const double* __restrict__ phis,
                                                       const double* __restrict__ As, int iter, int kidx) {
  const int nb = (md.n_test + 255) / 256;
  const int s = blockIdx.x / nb;
  const int t0 = (blockIdx.x % nb) * 256 + threadIdx.x;
  const bool act = t0 < md.n_test;
  const int t = act ? t0 : md.n_test - 1;
  const int ns = md.n_s[s], np = md.n_pad;
  const double phi = phis[s];
  const double xt = md.coords_test[t], yt = md.coords_test[md.n_test_pad + t];
  const double* cx = coords + (long)s * 2 * np;
  const double* cy = cx + np;
  const double* gs = g + (long)s * np;
  double a0 = 0.0, a1 = 0.0;
  int i = 0;
  for (; i + 1 < ns; i += 2) {
    a0 = fma(exp(-phi * dist_fast(cx[i], cy[i], xt, yt)), gs[i], a0);
    a1 = fma(exp(-phi * dist_fast(cx[i + 1], cy[i + 1], xt, yt)), gs[i + 1], a1);
  }
  if (i < ns) a0 = fma(exp(-phi * dist_fast(cx[i], cy[i], xt, yt)), gs[i], a0);
  const double sd = sqrt(fmax(1.0 - cheb_s(c, md.S, s, t, phi), 0.0));
  const Key key = subset_key(md, s);
  const double v = (a0 + a1) + sd * predict_normal(key, md.t_off + t, iter);   // q = 1: index (t_off + t) q + h
  double o = 0.0;
  o += v * As[s];
  if (act) md.w_pred[((long)s * md.n_kept + kidx) * md.n_test + t] = o;
}

}  // namespace mk
