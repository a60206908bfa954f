// Steps either side of the per-subset fits, on device:
//   k_weiszfeld    geometric median of the K subset quantile functions, column by column, in the
//                  W2 (L2-over-levels) metric -- the north-star combine extension (SURVEY.md 8f
//                  row 2); spec and CPU oracle: oracle/post.py weiszfeld_median.
//   k_post_*       MetaKriging_BinaryResponse.R:136-165: approx() of the combined grids at the
//                  resampled Xout levels (MK.R:140-146), one shared index vector (MK.R:141) and
//                  p(y=1) = 1/(1+exp(-(x.test %*% B.s + Samplew[j,]))) (MK.R:156-161); the
//                  (0.5, 0.025, 0.975) summaries reuse k_quantiles (MK.R:163-165).
//   k_glm_pass     one data pass of glm.fit's binomial-logit IRLS on the full data (MK.R:53-55,
//                  SURVEY.md 8f row 3): deviance of the current fit and the weighted normal
//                  equations of the next step, as per-block partials summed by the host in block
//                  order (deterministic).
#include "mk_types.hpp"

namespace mk {

__device__ inline double wave_sum64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

#define WZ_R 4   // levels per lane: L <= 256

// One wave per column c.  Grid k is L x C column-major at grids + k*L*C, so column c of every
// grid is L contiguous doubles.  Iterates live in registers; the K columns stream from L2.
__global__ __launch_bounds__(256) void k_weiszfeld(const double* __restrict__ grids, int K, int L, long C,
                                                   int max_iter, double tol, double* __restrict__ out,
                                                   int* __restrict__ iters) {
  const int lane = threadIdx.x & 63;
  const long c = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= C) return;
  const long LC = (long)L * C;
  const double* g0 = grids + c * L;
  const double Ld = (double)L;
  double y[WZ_R];
  bool on[WZ_R];
#pragma unroll
  for (int r = 0; r < WZ_R; ++r) {
    const int l = lane + 64 * r;
    on[r] = l < L;
    y[r] = on[r] ? g0[l] : 0.0;
  }
  // barycenter = the reference's combine: ((g_0 + g_1) + ...) / K  (MK.R:123-127)
  for (int k = 1; k < K; ++k) {
    const double* gk = g0 + k * LC;
#pragma unroll
    for (int r = 0; r < WZ_R; ++r)
      if (on[r]) y[r] = y[r] + gk[lane + 64 * r];
  }
#pragma unroll
  for (int r = 0; r < WZ_R; ++r) y[r] = y[r] / K;
  int it = 0;
  while (it < max_iter) {
    double yy = 0.0;
#pragma unroll
    for (int r = 0; r < WZ_R; ++r) yy += y[r] * y[r];
    const double floor_d = 1e-14 * (1.0 + sqrt(wave_sum64(yy) / Ld));
    double num[WZ_R] = {0.0, 0.0, 0.0, 0.0};
    double den = 0.0;
    for (int k = 0; k < K; ++k) {
      const double* gk = g0 + k * LC;
      double qv[WZ_R];
      double ss = 0.0;
#pragma unroll
      for (int r = 0; r < WZ_R; ++r) {
        qv[r] = on[r] ? gk[lane + 64 * r] : 0.0;
        const double dl = qv[r] - y[r];
        ss += dl * dl;
      }
      const double d = fmax(sqrt(wave_sum64(ss) / Ld), floor_d);
      const double wk = 1.0 / d;
#pragma unroll
      for (int r = 0; r < WZ_R; ++r) num[r] = num[r] + qv[r] * wk;
      den = den + wk;
    }
    double st = 0.0, yn2 = 0.0;
#pragma unroll
    for (int r = 0; r < WZ_R; ++r) {
      const double yn = on[r] ? num[r] / den : 0.0;
      const double dl = yn - y[r];
      st += dl * dl;
      yn2 += yn * yn;
      y[r] = yn;
    }
    ++it;
    if (sqrt(wave_sum64(st) / Ld) <= tol * (1.0 + sqrt(wave_sum64(yn2) / Ld))) break;
  }
#pragma unroll
  for (int r = 0; r < WZ_R; ++r)
    if (on[r]) out[c * L + lane + 64 * r] = y[r];
  if (lane == 0 && iters) iters[c] = it;
}

// sampleparIndex (MK.R:141), 0-based: idx_j = min(floor(u_j * n_levels), n_levels - 1),
// u_j from Philox key (seed, 0), counter (j, 0, TAG_RESAMPLE, 0) -- oracle/post.py resample_index.
__global__ __launch_bounds__(256) void k_post_index(uint64_t seed, int samplesize, int n_levels, int* __restrict__ idx) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= samplesize) return;
  const uint4 w = philox((uint32_t)j, 0u, MK_TAG_RESAMPLE, 0u, make_key(seed, 0u));
  const double u = u01_open(w.x, w.y);
  idx[j] = min((int)floor(u * (double)n_levels), n_levels - 1);
}

// out[j + c*S] = approx(probs, grid[, c], xout = Xout[idx_j])$y  (MK.R:142-146).  Per Xout level
// the host ran R's approx1 bisection: mode 0 -> y[hi] (v == x[j]), 1 -> y[lo] (v == x[i]),
// 2 -> y[lo] + (y[hi] - y[lo]) * t  with t = (v - x[i]) / (x[j] - x[i]).
__global__ __launch_bounds__(256) void k_post_interp(const double* __restrict__ grid, int L, long C,
                                                     const int* __restrict__ idx, int S, const int* __restrict__ lo,
                                                     const int* __restrict__ hi, const int* __restrict__ mode,
                                                     const double* __restrict__ t, double* __restrict__ out) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long)S * C) return;
  const int j = (int)(e % S);
  const long c = e / S;
  const int lv = idx[j];
  const double* y = grid + c * L;
  double v;
  const int m = mode[lv];
  if (m == 0) {
    v = y[hi[lv]];
  } else if (m == 1) {
    v = y[lo[lv]];
  } else {
    const double yi = y[lo[lv]], yj = y[hi[lv]];
    v = yi + (yj - yi) * t[lv];
  }
  out[e] = v;
}

// p.sample[j, c] = 1 / (1 + exp(-(x.test[c, ] %*% SamplePar[j, 1:p] + Samplew[j, c])))  (MK.R:156-161),
// x.test %*% B.s summed in column order.  All matrices column-major (R).
// link = MK_LINK_PROBIT (north-star extension; the reference is logit): Phi(eta) = erfc(-eta/sqrt 2)/2.
__global__ __launch_bounds__(256) void k_post_prob(const double* __restrict__ sample_par, int S,
                                                   const double* __restrict__ x_test, long C, int p,
                                                   const double* __restrict__ sample_w, int link,
                                                   double* __restrict__ pout) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long)S * C) return;
  const int j = (int)(e % S);
  const long c = e / S;
  double xb = 0.0;
  for (int m = 0; m < p; ++m) xb = xb + x_test[c + (long)m * C] * sample_par[j + (long)m * S];
  const double eta = xb + sample_w[e];
  pout[e] = (link == MK_LINK_PROBIT) ? norm_cdf(eta) : 1.0 / (1.0 + exp(-eta));
}

// ---------------------------------------------------------------- glm.fit IRLS pass (binomial)
// logit: R's family.c logit link with its eta thresholds (binomial()$linkinv / $mu.eta);
// probit: make.link("probit") -- linkinv = pnorm(eta clamped to +-(-qnorm(eps))),
// mu.eta = max(dnorm(eta), eps), linkfun = qnorm.
#define GLM_THRESH 30.0
#define GLM_EPS 2.220446049250313e-16
#define GLM_PROBIT_THRESH 8.125890664701906   // -qnorm(.Machine$double.eps)
#define GLM_INV_SQRT_2PI 0.3989422804014327
__device__ inline double glm_linkinv(double eta, int link) {
  if (link == MK_LINK_PROBIT) return norm_cdf(fmin(fmax(eta, -GLM_PROBIT_THRESH), GLM_PROBIT_THRESH));
  const double tmp = (eta < -GLM_THRESH) ? GLM_EPS : ((eta > GLM_THRESH) ? 1.0 / GLM_EPS : exp(eta));
  return tmp / (1.0 + tmp);
}
__device__ inline double glm_mu_eta(double eta, int link) {
  if (link == MK_LINK_PROBIT) return fmax(GLM_INV_SQRT_2PI * exp(-0.5 * eta * eta), GLM_EPS);
  const double opexp = 1.0 + exp(eta);
  return (eta > GLM_THRESH || eta < -GLM_THRESH) ? GLM_EPS : exp(eta) / (opexp * opexp);
}
__device__ inline double y_log_y(double y, double mu) { return (y != 0.0) ? y * log(y / mu) : 0.0; }

// mode 0: eta from binomial()$initialize (mustart = (wt*y + 0.5)/(wt + 1)); mode 1: eta = X coef.
// Per block b: part[b*NP + 0] = deviance, then the packed lower triangle of X'WX, then X'Wz,
// where W, z are the IRLS weights / working response at this eta (the next solve's system).
#define GLM_PMAX 8
__global__ __launch_bounds__(256) void k_glm_pass(const double* __restrict__ yprop, const double* __restrict__ wt,
                                                  const double* __restrict__ X, long n, int p,
                                                  const double* __restrict__ coef, int mode, int link,
                                                  double* __restrict__ part) {
  __shared__ double red[8];
  const int np_tri = p * (p + 1) / 2;
  const int NP = 1 + np_tri + p;
  double loc[1 + GLM_PMAX * (GLM_PMAX + 1) / 2 + GLM_PMAX];
  for (int i = 0; i < NP; ++i) loc[i] = 0.0;
  for (long r = (long)blockIdx.x * 256 + threadIdx.x; r < n; r += (long)gridDim.x * 256) {
    const double y = yprop[r], w = wt[r];
    double eta, mu;
    if (mode == 0) {
      mu = (w * y + 0.5) / (w + 1.0);
      eta = (link == MK_LINK_PROBIT) ? normcdfinv(mu) : log(mu / (1.0 - mu));
    } else {
      eta = 0.0;
      for (int j = 0; j < p; ++j) eta += X[r + (long)j * n] * coef[j];
      mu = glm_linkinv(eta, link);
    }
    loc[0] += 2.0 * w * (y_log_y(y, mu) + y_log_y(1.0 - y, 1.0 - mu));
    if (w > 0.0) {
      const double me = glm_mu_eta(eta, link);
      const double z = eta + (y - mu) / me;
      const double ww = w * me * me / (mu * (1.0 - mu));   // (sqrt-weight)^2
      int k = 1;
      for (int a = 0; a < p; ++a) {
        const double xa = X[r + (long)a * n];
        for (int b = a; b < p; ++b) loc[k++] += ww * xa * X[r + (long)b * n];
      }
      for (int a = 0; a < p; ++a) loc[1 + np_tri + a] += ww * X[r + (long)a * n] * z;
    }
  }
  for (int i = 0; i < NP; ++i) {
    const double tot = block_sum<256>(loc[i], red);
    if (threadIdx.x == 0) part[(long)blockIdx.x * NP + i] = tot;
  }
}

}  // namespace mk
