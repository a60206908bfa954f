// Development probe: k_chol_diag on the cfg3 shape (S=250 candidates of 2048^2, tile k),
// shader-clock stamps per phase (MK_DIAG_TIMING) averaged over the workgroups.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DMK_DIAG_TIMING tools/diag_probe.hip -o tools/diag_probe
#include <cstdio>
#include <vector>
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
  hipMalloc(&ts, (size_t)S * 64 * 8);
  hipMemset(ts, 0, (size_t)S * 64 * 8);
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
    std::vector<long long> h((size_t)S * 64);
    hipMemcpy(h.data(), ts, h.size() * 8, hipMemcpyDeviceToHost);
    double avg[64] = {0};
    for (int b = 0; b < S; ++b)
      for (int i = 0; i < 64; ++i) avg[i] += (double)(h[b * 64 + i] - h[b * 64]) / S;
    printf("k=%d best %.1f us  (cycles since start, avg over %d WGs)\n", k, best * 1e3, S);
    printf("  load %.0f\n", avg[40]);
    for (int p = 0; p < 8; ++p) printf("  p%d phase1 %.0f phase2 %.0f\n", p, avg[1 + 3 * p], avg[2 + 3 * p]);
  
    printf("  logdet %.0f store %.0f\n", avg[41], avg[42]);
  }
  return 0;
}
