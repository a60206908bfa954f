// Chain initialisation and the plain-matrix helpers behind the parity-test entry points.
#include "mk_types.hpp"
#include "mk_corr.hpp"

namespace mk {

// eta = X beta + w and u = A^-1 w at the starting values (spMvGLM starting=, MK.R:60).
__global__ __launch_bounds__(256) void k_init_state(Model md) {
  const int s = blockIdx.x, q = md.q, ns = md.n_s[s];
  const double* w = md.w + (long)s * md.Np;
  double* eta = md.eta + (long)s * md.Np;
  const double* beta = md.beta + (long)s * md.p;
  const double* Ai = md.Ainv + (long)s * q * q;
  for (int k = threadIdx.x; k < ns * q; k += 256) {
    double v = 0.0;
    for (int j = 0; j < md.p; ++j) v += md.X[((long)s * md.p + j) * md.Np + k] * beta[j];
    eta[k] = v + w[k];
  }
  for (int i = threadIdx.x; i < ns; i += 256)
    for (int h = 0; h < q; ++h) {
      double v = 0.0;
      for (int a = 0; a < q; ++a) v += Ai[h + a * q] * w[i * q + a];
      md.u[((long)s * q + h) * md.n_pad + i] = v;
    }
}

// Accept the starting-value factorisations of outcomes h0 .. h0+hc-1 unconditionally.
__global__ __launch_bounds__(64) void k_theta_init(Model md, MatSet ms, int h0, int hc) {
  const int e = blockIdx.x * 64 + threadIdx.x;
  if (e >= md.S * hc) return;
  const int s = e / hc, h = h0 + e % hc;
  const int sh = s * md.q + h;
  double ld = 0.0;
  for (int k = 0; k < md.nt; ++k) ld += md.ld_part[(long)sh * md.nt + k];
  md.logdetR[sh] = ld;
  md.quad[sh] = md.quad_c[sh];
  ms.cur[sh] ^= 1;
  md.dirty[sh] = 1;
  md.info[sh] = 0;
}

// Copy S dense n x n matrices into the candidate slot, identity-padded, zero border row.
__global__ __launch_bounds__(256) void k_load_plain(MatSet ms, const double* A, int n, int S) {
  const long ld = ms.ld, tot = (long)S * ld * ld;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < tot; e += (long)gridDim.x * 256) {
    const int s = (int)(e / (ld * ld));
    const long rem = e % (ld * ld);
    const int r = (int)(rem % ld), c = (int)(rem / ld);
    double v;
    if (r < n && c < n) v = A[(long)s * n * n + r + (long)c * n];
    else v = (r == c && r != n) ? 1.0 : 0.0;
    mat_slot(ms, s, 1 - ms.cur[s])[rem] = v;
  }
}

// Dense symmetric n x n image of the candidate slot's lower tiles (k_cov_candidate output: the
// upper half of its diagonal tiles is never written), for the correlation parity entry point.
__global__ __launch_bounds__(256) void k_extract_candidate(MatSet ms, int n, int S, double* out) {
  const long tot = (long)S * n * n;
  const long ld = ms.ld;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < tot; e += (long)gridDim.x * 256) {
    const int s = (int)(e / ((long)n * n));
    const long rem = e % ((long)n * n);
    const int r = (int)(rem % n), c = (int)(rem / n);
    const double* M = mat_slot(ms, s, 1 - ms.cur[s]);
    out[e] = (r >= c) ? M[r + (long)c * ld] : M[c + (long)r * ld];
  }
}

// mode 0: lower factor of the current slot (zeros above); mode 1: Q (full symmetric).
__global__ __launch_bounds__(256) void k_extract_L(MatSet ms, int n, int S, double* L, int mode) {
  const long tot = (long)S * n * n;
  const long ld = ms.ld;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < tot; e += (long)gridDim.x * 256) {
    const int s = (int)(e / ((long)n * n));
    const long rem = e % ((long)n * n);
    const int r = (int)(rem % n), c = (int)(rem / n);
    if (mode == 0) {
      const double* M = mat_slot(ms, s, ms.cur[s]);
      L[e] = (r >= c) ? M[r + (long)c * ld] : 0.0;
    } else {
      L[e] = ms.Q[(long)s * ld * ld + r + (long)c * ld];
    }
  }
}

}  // namespace mk
