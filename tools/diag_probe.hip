// Development probe: k_chol_diag on the cfg3 shape (S=250 candidates of 2048^2, tile k),
// shader-clock stamps per phase (MK_DIAG_TIMING) averaged over the workgroups.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DMK_DIAG_TIMING tools/diag_probe.hip -o tools/diag_probe
#include <cstdio>
#include <vector>
#include <cmath>
#include "../laurabaracaldo-spatial-meta-kriging-for-distributed-inference-for-binary-response_amd/csrc/mk_linalg.hip"
using namespace mk;

__global__ void k_fill(double* p, long n, int ld) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const long e = i % ((long)ld * ld);
    const int r = (int)(e % ld), c = (int)(e / ld);
    p[i] = (r == c) ? 200.0 : 1e-3 * (double)(((long)(r + c) * 2654435761ull) % 1000) - 0.5;
  }
}

int main(int argc, char** argv) {
  const int S = argc > 1 ? atoi(argv[1]) : 250, ld = 2048, nt = 16;
  MatSet ms{};
  ms.ld = ld; ms.nt = nt; ms.q = 1;
  const long me = (long)ld * ld;
  hipMalloc(&ms.L, (size_t)S * 2 * me * 8);
  hipMalloc(&ms.Winv, (size_t)S * 2 * nt * MK_NB * MK_NB * 8);
  hipMemset(ms.Winv, 0, (size_t)S * 2 * nt * MK_NB * MK_NB * 8);
  hipMalloc(&ms.cur, S * 4);
  hipMemset(ms.cur, 0, S * 4);
  int* ns; double *ldp, *qc; int* info;
  hipMalloc(&ns, S * 4); hipMalloc(&ldp, (size_t)S * nt * 8); hipMalloc(&qc, S * 8); hipMalloc(&info, S * 4);
  std::vector<int> hn(S, 2000);
  hipMemcpy(ns, hn.data(), S * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, ms.L, (long)S * 2 * me, ld);
  long long* ts;
  hipMalloc(&ts, (size_t)S * 128 * 8);
  hipMemset(ts, 0, (size_t)S * 128 * 8);
  hipMemcpyToSymbol(HIP_SYMBOL(mk_diag_ts), &ts, sizeof(ts));
  hipFuncSetAttribute((const void*)k_chol_diag, hipFuncAttributeMaxDynamicSharedMemorySize, MK_DIAG_LDS_BYTES);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int k : {0, 8, 15}) {
    float best = 1e9;
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(k_chol_diag, dim3(S), dim3(256), MK_DIAG_LDS_BYTES, 0, ms, ns, 0, 1, k, ldp, qc, info,
                         (const int*)nullptr, (const int*)nullptr);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float t; hipEventElapsedTime(&t, e0, e1);
      if (t < best) best = t;
    }
    // correctness: refill, one launch, check L L^T = A (lower) and W L = I on workgroup 0's tile
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, ms.L, (long)S * 2 * me, ld);
    hipLaunchKernelGGL(k_chol_diag, dim3(S), dim3(256), MK_DIAG_LDS_BYTES, 0, ms, ns, 0, 1, k, ldp, qc, info,
                       (const int*)nullptr, (const int*)nullptr);
    hipDeviceSynchronize();
    if (k < 15) {
      std::vector<double> Lh(128 * 128), Wh(128 * 128);
      const int base = k * 128;
      for (int c = 0; c < 128; ++c)
        hipMemcpy(Lh.data() + c * 128, ms.L + me + base + (long)(base + c) * ld, 128 * 8, hipMemcpyDeviceToHost);
      hipMemcpy(Wh.data(), ms.Winv + (size_t)(1 * nt + k) * MK_NB * MK_NB, 128 * 128 * 8, hipMemcpyDeviceToHost);
      double e1 = 0, e2 = 0;
      for (int r = 0; r < 128; ++r)
        for (int c = 0; c <= r; ++c) {
          double a = 0, w = 0;
          for (int m = 0; m <= c; ++m) a += Lh[r + m * 128] * Lh[c + m * 128];
          for (int m = c; m <= r; ++m) w += Wh[r + m * 128] * Lh[m + c * 128];
          const int R = base + r, C = base + c;
          const double A = (R == C) ? 200.0 : 1e-3 * (double)(((long)(R + C) * 2654435761ull) % 1000) - 0.5;
          e1 = fmax(e1, fabs(a - A) / 200.0);
          e2 = fmax(e2, fabs(w - (r == c ? 1.0 : 0.0)));
        }
      printf("  check k=%d: max|LL^T - A|/200 %.2e  max|WL - I| %.2e\n", k, e1, e2);
    }
    std::vector<long long> h((size_t)S * 128);
    hipMemcpy(h.data(), ts, h.size() * 8, hipMemcpyDeviceToHost);
    double avg[128] = {0};
    for (int b = 0; b < S; ++b)
      for (int i = 0; i < 128; ++i) avg[i] += (double)(h[b * 128 + i] - h[b * 128]) / S;
    printf("k=%d best %.1f us  (cycles since start, avg over %d WGs)\n", k, best * 1e3, S);
    printf("  load %.0f\n", avg[40]);
    for (int p = 0; p < 8; ++p)
      printf("  p%d ph1 %.0f ph2 %.0f | w0 pivot %.0f-%.0f | w1 start %.0f S-end %.0f end %.0f | w2 end %.0f | w3 end %.0f\n",
             p, avg[1 + 3 * p], avg[2 + 3 * p], avg[44 + 4 * p], avg[45 + 4 * p], avg[96 + p], avg[47 + 4 * p],
             avg[46 + 4 * p], avg[80 + p], avg[88 + p]);
    printf("  logdet %.0f store %.0f\n", avg[41], avg[42]);
  }
  return 0;
}
