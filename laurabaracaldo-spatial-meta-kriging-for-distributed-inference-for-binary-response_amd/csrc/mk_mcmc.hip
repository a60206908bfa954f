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
    for (int k = tid; k < Ns; k += 256) {
      const double e0 = eta[k];
      loc += loglik_term(y[k], wt[k], e0 + delta * xj[k], md.link) - loglik_term(y[k], wt[k], e0, md.link);
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
  // ---- T (symmetric in c,d)
  for (int h = 0; h < q; ++h)
    for (int c = 0; c < q; ++c)
      for (int d = c; d < q; ++d) {
        const double* zc = (q == 1) ? z : Z + ((long)h * q + c) * md.n_pad;
        const double* zd = (q == 1) ? z : Z + ((long)h * q + d) * md.n_pad;
        double loc = 0.0;
        for (int i = tid; i < ns; i += 256) loc += zc[i] * zd[i];
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
    for (int i = tid; i < ns; i += 256) loc += z[(long)h * md.n_pad + i] * z[(long)h * md.n_pad + i];
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
  if (md.info[sh] == 0 && lu <= ratio) {
    th[idx] = th_c;
    ms.cur[sh] ^= 1;
    md.logdetR[sh] = ldc;
    md.quad[sh] = qc;
    md.dirty[sh] = 1;
    md.acc[(long)s * md.n_mh_max + j_mh] += 1.0;
  }
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
// W panels are streamed twice per sweep (dots, update) -> n^2 doubles per subset per sweep.
#define SW_B 64
#define SW_T MK_SW_T
// Lane i's value (i wave-uniform) as a scalar: two v_readlane_b32.
__device__ inline double rlane_u(double v, int i) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), i);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), i);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__global__ __launch_bounds__(SW_T) void k_sweep(Model md, MatSet ms, int iter) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int q = md.q;
  double* Qb = smem;                              // [q][SW_B*SW_B] column-major
  double* gb = smem + q * SW_B * SW_B;            // [q][SW_B]
  double* dacc = gb + q * SW_B;                   // [q][SW_B]
  __shared__ int any_acc;
  __shared__ double Ai[MK_QMAX * MK_QMAX];
  const int s = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int ns = md.n_s[s], Ns = ns * q;
  const Key key = subset_key(md, s);
  const long ld = ms.ld;
  const double* y = md.y + (long)s * md.Np;
  const double* wt = md.wt + (long)s * md.Np;
  double* eta = md.eta + (long)s * md.Np;
  double* w = md.w + (long)s * md.Np;
  double* dl = md.sw_delta + (long)s * md.Np;
  double* dll = md.sw_dll + (long)s * md.Np;
  double* lgu = md.sw_logu + (long)s * md.Np;
  int* sacc = md.sw_acc + (long)s * md.Np;
  double* z = md.z + (long)s * q * md.n_pad;
  const double* tune = md.tune + (long)s * md.n_mh_max + md.o_w;
  if (tid < q * q) Ai[tid] = md.Ainv[(long)s * q * q + tid];
  // ---- proposals, likelihood differences and accept draws: independent of the sweep order
  for (int k = tid; k < Ns; k += SW_T) {
    const int j = md.o_w + k;
    const double zz = proposal_normal(key, j, iter);
    const double d = exp(tune[k]) * zz;
    dl[k] = d;
    dll[k] = loglik_term(y[k], wt[k], eta[k] + d, md.link) - loglik_term(y[k], wt[k], eta[k], md.link);
    lgu[k] = accept_log_uniform(key, j, iter);
    sacc[k] = 0;
  }
  if (tid == 0) any_acc = 0;
  __syncthreads();
  int p0 = 0, pnb = 0;
  for (int b0 = 0; b0 < ns + SW_B; b0 += SW_B) {
    const int nb = min(SW_B, ns - b0);
    // ---- (a) z += W[:, prev block] delta'_prev   (rows >= p0)
    // Thread t owns the row pair p0 + 2t, p0 + 2t + 1 (16-byte loads; p0 is even, ld even) and
    // issues the 16 column loads of a group before using them: unconditional loads (clamped
    // column; W is finite everywhere), the short-block tail masked by a zero coefficient.
    if (pnb > 0 && any_acc) {
      for (int h = 0; h < q; ++h) {
        for (int r = p0 + 2 * tid; r < ns; r += 2 * SW_T) {
          const double* Wp = ms.W + ((long)s * q + h) * (ld * ld) + (long)p0 * ld + r;
          const double* da = dacc + h * SW_B;
          double* zh = z + (long)h * md.n_pad;
          d2 v = {0.0, 0.0};
          for (int k0 = 0; k0 < pnb; k0 += 16) {
            d2 wv2[16];
#pragma unroll
            for (int u = 0; u < 16; ++u)
              wv2[u] = *reinterpret_cast<const d2*>(Wp + (long)min(k0 + u, pnb - 1) * ld);
#pragma unroll
            for (int u = 0; u < 16; ++u) {
              const double c = (k0 + u < pnb) ? da[k0 + u] : 0.0;
              v.x = fma(wv2[u].x, c, v.x);
              v.y = fma(wv2[u].y, c, v.y);
            }
          }
          zh[r] += v.x;
          if (r + 1 < ns) zh[r + 1] += v.y;
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
      if (tid < SW_B) dacc[h * SW_B + tid] = 0.0;
      const double* Wb = ms.W + ((long)s * q + h) * (ld * ld) + (long)b0 * ld;
      const double* zh = z + (long)h * md.n_pad;
      // one wave per column; lane l reads rows b0 + 2l + 128j (16-byte loads, 8 in flight,
      // clamped inside the padded column and masked by a select)
      const int nj = (ns - b0 + 127) / 128;
      for (int i = wv; i < nb; i += SW_T / 64) {
        const double* col = Wb + (long)i * ld;
        double a0 = 0.0, a1 = 0.0;
        for (int j0 = 0; j0 < nj; j0 += 8) {
          d2 wv2[8], zv2[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int rc = min(b0 + 2 * lane + 128 * (j0 + u), md.n_pad - 2);
            wv2[u] = *reinterpret_cast<const d2*>(col + rc);
            zv2[u] = *reinterpret_cast<const d2*>(zh + rc);
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int rr = b0 + 2 * lane + 128 * (j0 + u);
            a0 = (rr < ns) ? fma(wv2[u].x, zv2[u].x, a0) : a0;
            a1 = (rr + 1 < ns) ? fma(wv2[u].y, zv2[u].y, a1) : a1;
          }
        }
        double acc = a0 + a1;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
        if (lane == 0) gb[h * SW_B + i] = acc;
      }
    }
    __syncthreads();
    // ---- (c) sequential Metropolis steps of the block (wave 0).  Lane i preloads site b0+i's
    // proposal, likelihood difference, accept draw and Q diagonal; each step reads them (and
    // the carried g) by readlane with the uniform step index: no memory round trip per step.
    if (wv == 0) {
      // (register arrays indexed by compile-time constants only: loops over MK_QMAX, q-guarded)
      double gl[MK_QMAX], qd[MK_QMAX], dlr[MK_QMAX], dllr[MK_QMAX], lgr[MK_QMAX];
      const int ls = (lane < nb) ? lane : 0;
#pragma unroll
      for (int h = 0; h < MK_QMAX; ++h) {
        gl[h] = (h < q && lane < nb) ? gb[h * SW_B + lane] : 0.0;
        qd[h] = (h < q) ? Qb[h * SW_B * SW_B + ls * SW_B + ls] : 0.0;
        const int k = (b0 + ls) * q + h;
        dlr[h] = (h < q) ? dl[k] : 0.0;
        dllr[h] = (h < q) ? dll[k] : 0.0;
        lgr[h] = (h < q) ? lgu[k] : 0.0;
      }
      int anyl = 0;
      for (int i = 0; i < nb; ++i) {
#pragma unroll
        for (int a = 0; a < MK_QMAX; ++a) {
          if (a >= q) break;
          const int k = (b0 + i) * q + a;
          const double d = rlane_u(dlr[a], i);
          double c = 0.0, dd = 0.0;
#pragma unroll
          for (int h = 0; h < MK_QMAX; ++h) {
            if (h >= q) break;
            const double aih = Ai[h + a * q];
            c += aih * rlane_u(gl[h], i);
            dd += (aih * aih) * rlane_u(qd[h], i);
          }
          const double ratio = rlane_u(dllr[a], i) - (d * c + 0.5 * d * d * dd);
          if (rlane_u(lgr[a], i) <= ratio) {
#pragma unroll
            for (int h = 0; h < MK_QMAX; ++h) {
              if (h >= q) break;
              const double coef = d * Ai[h + a * q];
              gl[h] = gl[h] + coef * Qb[h * SW_B * SW_B + i * SW_B + lane];
              if (lane == 0) dacc[h * SW_B + i] += coef;
            }
            if (lane == 0) sacc[k] = 1;
            anyl = 1;
          }
        }
      }
      if (lane == 0) any_acc = anyl;
    }
    __syncthreads();
    p0 = b0;
    pnb = nb;
  }
  // ---- apply accepted moves to w, eta, u and the batch accept counts
  double* u = md.u + (long)s * q * md.n_pad;
  double* acc = md.acc + (long)s * md.n_mh_max + md.o_w;
  for (int i = tid; i < ns; i += SW_T) {
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

// ---------------------------------------------------------------- 8. type-7 quantiles (MK.R:88-89)
// One workgroup per (subset, column): bitonic sort of the kept values in LDS,
// then R's quantile.default type 7: (1-h) x[lo] + h x[hi] (no FMA contraction).
__global__ __launch_bounds__(256) void k_quantiles(const double* __restrict__ data, long subset_stride, long row_stride,
                                                   int n_rows, int n_cols, const double* __restrict__ probs, int n_probs,
                                                   double* __restrict__ out /* [S][n_cols][n_probs] */) {
  __shared__ double v[2048];
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

}  // namespace mk
