// Spatial correlation functions (spBayes spCor semantics):
//   exponential  rho(d) = exp(-phi d)
//   Matern       rho(d) = (phi d)^nu / (2^(nu-1) Gamma(nu)) K_nu(phi d),  rho(0) = 1
// K_nu for real nu >= 0 in fp64: nu = n + mu, |mu| <= 1/2; K_mu, K_mu+1 from
// Temme's series (x <= 2) or Steed's continued fraction CF2 (x > 2) (Temme
// 1975, J. Comput. Phys. 19; the bessik scheme), then forward recurrence in nu.
// 1/Gamma(1 +- mu) differences use the reciprocal-gamma Taylor series
// (Abramowitz & Stegun 6.1.34) for |mu| < 0.1 to avoid cancellation.
#pragma once
#include "mk_common.hpp"

namespace mk {

#define MK_COV_EXPONENTIAL 0
#define MK_COV_MATERN 1
#define MK_BK_NTAB 64   // terms of the reciprocal tables (CorrFn::fill_tables)

// 1/y from the hardware reciprocal estimate and two Newton steps (within an ulp of 1.0/y;
// ~5 dependent fp64 ops instead of the IEEE division sequence).
__device__ inline double rcp_nr(double y) {
  double r = __builtin_amdgcn_rcp(y);
  double e = fma(-y, r, 1.0);
  r = fma(r, e, r);
  e = fma(-y, r, 1.0);
  return fma(r, e, r);
}

__device__ inline void temme_gammas(double mu, double* gam1, double* gam2, double* gampl, double* gammi) {
  // 1/Gamma(1+z) = sum_k a_k z^(k-1)  (A&S 6.1.34)
  const double a[15] = {1.0, 0.5772156649015329, -0.6558780715202538, -0.0420026350340952,
                        0.1665386113822915, -0.0421977345555443, -0.0096219715278770, 0.0072189432466630,
                        -0.0011651675918591, -0.0002152416741149, 0.0001280502823882, -0.0000201348547807,
                        -0.0000012504934821, 0.0000011330272320, -0.0000002056338417};
  *gampl = 1.0 / tgamma(1.0 + mu);
  *gammi = 1.0 / tgamma(1.0 - mu);
  *gam2 = 0.5 * (*gammi + *gampl);
  if (fabs(mu) < 0.1) {
    const double m2 = mu * mu;
    double s = 0.0, pw = 1.0;
    for (int k = 1; k < 15; k += 2) {  // a_2, a_4, ... (0-based odd indices)
      s += a[k] * pw;
      pw *= m2;
    }
    *gam1 = -s;
  } else {
    *gam1 = (*gammi - *gampl) / (2.0 * mu);
  }
}

// Correlation function of one (phi, nu): the nu-only pieces -- Matern's normaliser
// 2^(nu-1) Gamma(nu), Temme's reciprocal gammas, pi mu / sin(pi mu), the CF2 constant and the
// recurrence count -- are computed once per candidate (init), so an element costs only its
// x-dependent series / continued fraction.  The arithmetic per element is the classic
// bessik scheme, operation for operation.
struct CorrFn {
  int model;
  double phi, nu;
  int nl;
  double mu, mu2, gam1, gam2, gampl, gammi, fact, a1, den;
  // Optional reciprocal tables of the candidate's mu (LDS, filled by fill_tables): the series
  // and CF2 divisions by i - mu, i + mu, i^2 - mu^2, i and a_i = -a1 - i(i-1) become
  // multiplications for i < MK_BK_NTAB (a division costs ~10 dependent fp64 ops; these loops
  // dominate the Matern candidate kernel).  nullptr: divide (host, parity entry points).
  const double* tab;

  __device__ void init(double phi_, double nu_, int model_) {
    model = model_;
    phi = phi_;
    nu = nu_;
    tab = nullptr;
    if (model != MK_COV_MATERN) return;
    const double EPS = 1e-16, PI = 3.141592653589793;
    nl = (int)(nu + 0.5);
    mu = nu - nl;
    mu2 = mu * mu;
    const double pimu = PI * mu;
    fact = (fabs(pimu) < EPS) ? 1.0 : pimu / sin(pimu);
    temme_gammas(mu, &gam1, &gam2, &gampl, &gammi);
    a1 = 0.25 - mu2;
    den = pow(2.0, nu - 1.0) * tgamma(nu);
  }

  // tab[j * MK_BK_NTAB + i]: j = 0 1/(i-mu), 1 1/(i+mu), 2 1/(i^2-mu^2), 3 1/i, 4 1/a_i
  __device__ void fill_tables(double* t, int tid, int nthreads) const {
    for (int i = tid; i < MK_BK_NTAB; i += nthreads) {
      const double di = (double)i;
      t[i] = 1.0 / (di - mu);
      t[MK_BK_NTAB + i] = 1.0 / (di + mu);
      t[2 * MK_BK_NTAB + i] = 1.0 / (di * di - mu2);
      t[3 * MK_BK_NTAB + i] = (i > 0) ? 1.0 / di : 0.0;
      t[4 * MK_BK_NTAB + i] = 1.0 / (-a1 - di * (di - 1.0));
    }
  }

  // K_nu(x), x > 0 (Temme series for x < 2, Steed's CF2 above, forward recurrence in nu).
  // lx = log(x).  sinh, cosh and exp of e = mu log(2/x) come from one expm1.
  __device__ double bessel_k(double x, double lx) const {
    const double EPS = 1e-16, PI = 3.141592653589793, LN2 = 0.6931471805599453;
    const double xi = 1.0 / x, xi2 = 2.0 * xi;
    double rkmu, rk1;
    if (x < 2.0) {
      const double x2 = 0.5 * x;
      double d = LN2 - lx;
      const double e = mu * d;
      const double em1 = expm1(e), E = em1 + 1.0, iE = 1.0 / E;
      const double fact2 = (fabs(e) < EPS) ? 1.0 : 0.5 * em1 * (1.0 + iE) / e;   // sinh(e) / e
      double ff = fact * (gam1 * (0.5 * (E + iE)) + gam2 * fact2 * d);
      double sum = ff;
      double p = 0.5 * E / gampl, q = 0.5 * iE / gammi;
      double c = 1.0;
      d = x2 * x2;
      double sum1 = p;
      int i = 1;
      bool done = false;
      if (tab) {
        for (; i < MK_BK_NTAB; ++i) {
          ff = (i * ff + p + q) * tab[2 * MK_BK_NTAB + i];
          c *= d * tab[3 * MK_BK_NTAB + i];
          p *= tab[i];
          q *= tab[MK_BK_NTAB + i];
          const double del = c * ff;
          sum += del;
          sum1 += c * (p - i * ff);
          if (fabs(del) < fabs(sum) * EPS) { done = true; break; }
        }
      }
      for (; !done && i <= 500; ++i) {
        ff = (i * ff + p + q) / (i * (double)i - mu2);
        c *= d / i;
        p /= (i - mu);
        q /= (i + mu);
        const double del = c * ff;
        sum += del;
        sum1 += c * (p - i * ff);
        if (fabs(del) < fabs(sum) * EPS) break;
      }
      rkmu = sum;
      rk1 = sum1 * xi2;
    } else {
      double b = 2.0 * (1.0 + x), d = 1.0 / b, h = d, delh = d;
      double q1 = 0.0, q2 = 1.0;
      double q = a1, c = a1, a = -a1;
      double s = 1.0 + q * delh;
      int i = 2;
      bool done = false;
      if (tab) {
        for (; i < MK_BK_NTAB; ++i) {
          a -= 2 * (i - 1);
          c = -a * c * tab[3 * MK_BK_NTAB + i];
          const double qnew = (q1 - b * q2) * tab[4 * MK_BK_NTAB + i];
          q1 = q2;
          q2 = qnew;
          q += c * qnew;
          b += 2.0;
          d = rcp_nr(b + a * d);
          delh = (b * d - 1.0) * delh;
          h += delh;
          const double dels = q * delh;
          s += dels;
          if (fabs(dels) < fabs(s) * EPS) { done = true; break; }
        }
      }
      for (; !done && i <= 500; ++i) {
        a -= 2 * (i - 1);
        c = -a * c / i;
        const double qnew = (q1 - b * q2) / a;
        q1 = q2;
        q2 = qnew;
        q += c * qnew;
        b += 2.0;
        d = 1.0 / (b + a * d);
        delh = (b * d - 1.0) * delh;
        h += delh;
        const double dels = q * delh;
        s += dels;
        if (fabs(dels / s) < EPS) break;
      }
      h = a1 * h;
      rkmu = sqrt(PI / (2.0 * x)) * exp(-x) / s;
      rk1 = rkmu * (mu + x + 0.5 - h) * xi;
    }
    for (int i = 1; i <= nl; ++i) {
      const double t = (mu + i) * xi2 * rk1 + rkmu;
      rkmu = rk1;
      rk1 = t;
    }
    return rkmu;
  }

  // Matern rho at x = phi d: x^nu / (2^(nu-1) Gamma(nu)) K_nu(x), 1 at x = 0
  __device__ double matern_x(double x) const {
    if (!(x > 0.0)) return 1.0;
    const double lx = log(x);
    return exp(nu * lx) / den * bessel_k(x, lx);
  }

  // rho(d): exponential exp(-phi d); Matern (phi d)^nu / (2^(nu-1) Gamma(nu)) K_nu(phi d), 1 at d = 0
  __device__ double operator()(double d) const {
    if (model == MK_COV_EXPONENTIAL) return exp(-phi * d);
    return matern_x(d * phi);
  }
};

// ---------------------------------------------------------------- Matern by Chebyshev tables
// The exact K_nu above costs ~300-700 dependent fp64 operations per element (series / continued
// fraction); the candidate and kriging kernels instead interpolate rho(x) of their candidate's
// (phi, nu) from a table built per workgroup out of exact values: on x in [0.5, x_hi], where rho is
// analytic, piecewise Chebyshev series of MK_CH_N terms on intervals [0.5 * 1.25^g, 0.5 * 1.25^(g+1))
// (g < 7: the singularity of x^(2 nu) at 0 stays >= 9 half-widths away) and then of width 0.5
// (e^-x varies by e^-0.5 per interval).  Truncation error ~ rho_E^-12 ~ 1e-15 relative for these
// widths (Bernstein ellipse rho_E >= 17.9); measured against scipy kv: <= 1e-13 relative, nu in [0.05, 4], x in
// [0.5, 39] (the scipy reference's own accuracy).  x < 0.5 (the non-analytic part) and x beyond
// the table use the exact evaluation.  Clenshaw: ~2 fp64 operations per term.
#define MK_CH_N 12                         // Chebyshev terms per interval (degree 11)
#define MK_CH_LD (MK_CH_N + 2)             // per interval: coefficients, centre, 1 / half-width
#define MK_CH_NG 7                         // geometric intervals
#define MK_CH_NI_MAX 100                   // x < 2.384 + 0.5 * 93 = 48.88
#define MK_CH_E7 2.384185791015625         // 0.5 * 1.25^7 (exact)
#define MK_PT_RB 16                        // observation rows per workgroup of k_pred_PT_matern
#define MK_CH_TAB (MK_CH_NI_MAX * MK_CH_LD + 1)   // one stored table: intervals, then the interval count

// interval of x >= 0.5
__device__ inline int cheb_interval(double x) {
  if (x >= MK_CH_E7) return MK_CH_NG + (int)((x - MK_CH_E7) * 2.0);
  return (x >= 0.625) + (x >= 0.78125) + (x >= 0.9765625) + (x >= 1.220703125) + (x >= 1.52587890625) +
         (x >= 1.9073486328125);
}
// left edge of interval j
__device__ inline double cheb_edge(int j) {
  if (j >= MK_CH_NG) return MK_CH_E7 + 0.5 * (j - MK_CH_NG);
  double e = 0.5;
  for (int g = 0; g < j; ++g) e *= 1.25;   // 5/4 powers of 1/2: exact
  return e;
}
// intervals covering [0.5, x_hi] (x_hi = +inf or NaN: all)
__device__ inline int cheb_count(double x_hi) {
  if (x_hi < 0.5) return 0;
  if (!(x_hi < 0.5 + 0.5 * MK_CH_NI_MAX)) return MK_CH_NI_MAX;
  return min(MK_CH_NI_MAX, cheb_interval(x_hi) + 2);   // one interval of margin (rounding of x)
}

// Build the table of rho (tab: ni * MK_CH_LD doubles) with every thread of the workgroup; vals:
// ni * MK_CH_N scratch, cosm: MK_CH_N^2.  Ends with a barrier.
__device__ inline void cheb_build(const CorrFn& rho, int ni, double* tab, double* vals, double* cosm, int tid, int nth) {
  const double PI = 3.141592653589793;
  for (int i = tid; i < MK_CH_N * MK_CH_N; i += nth) {
    const int k = i / MK_CH_N, m = i % MK_CH_N;
    cosm[i] = cos(PI * k * (m + 0.5) / MK_CH_N);
  }
  __syncthreads();
  for (int i = tid; i < ni * MK_CH_N; i += nth) {
    const int j = i / MK_CH_N, m = i % MK_CH_N;
    const double a = cheb_edge(j), b = cheb_edge(j + 1);
    vals[i] = rho.matern_x(0.5 * (a + b) + 0.5 * (b - a) * cosm[MK_CH_N + m]);   // node t_m = cos(pi (m+1/2)/N)
  }
  __syncthreads();
  for (int i = tid; i < ni * MK_CH_LD; i += nth) {
    const int j = i / MK_CH_LD, k = i % MK_CH_LD;
    const double a = cheb_edge(j), b = cheb_edge(j + 1);
    double v;
    if (k < MK_CH_N) {
      v = 0.0;
      for (int m = 0; m < MK_CH_N; ++m) v += vals[j * MK_CH_N + m] * cosm[k * MK_CH_N + m];
      v *= (k == 0 ? 1.0 : 2.0) / MK_CH_N;
    } else {
      v = (k == MK_CH_N) ? 0.5 * (a + b) : 2.0 / (b - a);
    }
    tab[i] = v;
  }
  __syncthreads();
}

// rho(x) from the table; false when x is outside it (x < 0.5, beyond interval ni - 1, NaN)
__device__ inline bool cheb_eval(const double* tab, int ni, double x, double* out) {
  if (!(x >= 0.5)) return false;
  const int j = cheb_interval(x);
  if (j >= ni) return false;
  const double* c = tab + j * MK_CH_LD;
  const double t = (x - c[MK_CH_N]) * c[MK_CH_N + 1], t2 = 2.0 * t;
  double b1 = 0.0, b2 = 0.0;
#pragma unroll
  for (int k = MK_CH_N - 1; k >= 1; --k) {
    const double b0 = fma(t2, b1, c[k] - b2);
    b2 = b1;
    b1 = b0;
  }
  *out = fma(t, b1, c[0] - b2);
  return true;
}

__device__ inline double correlation(double d, double phi, double nu, int model) {
  CorrFn f;
  f.init(phi, nu, model);
  return f(d);
}

__device__ inline double dist2d(double x0, double y0, double x1, double y1) {
  const double dx = x0 - x1, dy = y0 - y1;
  return sqrt(dx * dx + dy * dy);
}

}  // namespace mk
