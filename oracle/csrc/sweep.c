/* CPU restatement of the single-site latent-w sweep of oracle/spmvglm.py fit_subset step 5
 * (the oracle's own algorithm: R^-1 held explicitly as Q_h, g_h = Q_h u_h carried through the
 * sweep), in C so that the CPU baseline's iteration is native code end to end (LAPACK for the
 * factorisations, this loop for the sweep) instead of a Python loop.  TEST INFRASTRUCTURE: only
 * tests/ and bench.py's cpu_baseline leg load it.  Same operations in the same order as the
 * NumPy loop (build with -ffp-contract=off): bit-identical for q = 1 (tests/test_oracle.py).
 *
 * Layouts (NumPy C order): G, U, Qdiag [n][q]; Ainv [q][q]; Q[h] [n][n] (symmetric, so row i is
 * column i); w, eta, delta_w, dll, lu, accept_w [n q] (site-major, outcome-minor). */
#include <stddef.h>

void mk_oracle_sweep(int n, int q, const double* delta_w, const double* dll, const double* lu,
                     const double* Ainv, const double* Qdiag, const double* const* Q, double* G, double* U,
                     double* w, double* eta, double* accept_w) {
  const long N = (long)n * q;
  for (long k = 0; k < N; ++k) {
    const long i = k / q;
    const int a = (int)(k % q);
    const double dl = delta_w[k];
    double c = 0.0, d = 0.0;
    for (int h = 0; h < q; ++h) c += Ainv[h * q + a] * G[i * q + h];
    for (int h = 0; h < q; ++h) d += (Ainv[h * q + a] * Ainv[h * q + a]) * Qdiag[i * q + h];
    if (lu[k] <= dll[k] - (dl * c + 0.5 * dl * dl * d)) {
      w[k] += dl;
      eta[k] += dl;
      for (int h = 0; h < q; ++h) {
        const double coef = dl * Ainv[h * q + a];
        U[i * q + h] += coef;
        const double* Qi = Q[h] + (size_t)i * n;
        double* Gh = G + h;
        for (long r = 0; r < n; ++r) Gh[r * q] += coef * Qi[r];
      }
      accept_w[k] += 1.0;
    }
  }
}
