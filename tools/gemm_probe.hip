// Micro-benchmark for the fp64 MFMA tile GEMM (development tool, not shipped).
// 1) raw v_mfma_f64_16x16x4 throughput (registers only)
// 2) mk::gemm_128 on batched 128 x K panels: operands from HBM (distinct per tile) vs L2 (shared)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cstdlib>
#include "../laurabaracaldo-spatial-meta-kriging-for-distributed-inference-for-binary-response_amd/csrc/mk_gemm.hpp"
using namespace mk;

__global__ __launch_bounds__(256) void k_mfma_peak(double* out, int iters) {
  d4 acc[16];
  for (int i = 0; i < 16; ++i) acc[i] = (d4){0, 0, 0, 0};
  double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 12345.0) out[threadIdx.x] = s;
}

__global__ void k_fill(double* p, long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    p[i] = 1e-3 * (double)((i * 2654435761ull) % 1000) - 0.5;
}

template <bool BNU>
__global__ __launch_bounds__(256, 2) void k_probe(const double* A, const double* B, double* C, int K, long strideA,
                                               long strideB, int lda) {
  extern __shared__ __attribute__((aligned(16))) double lds[];   // GB_LDS_BYTES
  const double* a = A + blockIdx.x * strideA;
  const double* b = B + blockIdx.x * strideB;
  Acc acc;
  acc_zero(acc);
  gemm_128<true, BNU>(a, lda, b, BNU ? 128 : K, K, K, acc, lds);
  store_tile(C + (long)blockIdx.x * 128 * 128, 128, acc);
}

int main() {
  double* out;
  hipMalloc(&out, 4096 * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 4000;
  // 1) raw MFMA rate: 16 independent accumulators per wave, 1 or 2 waves per SIMD
  for (int wps : {1, 2}) {
    const int grid = 256 * wps;
    hipLaunchKernelGGL(k_mfma_peak, dim3(grid), dim3(256), 0, 0, out, iters);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_mfma_peak, dim3(grid), dim3(256), 0, 0, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double fl = 5.0 * grid * 4.0 * 64 * 16.0 * iters * 2048 / 64;   // 2048 flops per wave-MFMA
    printf("raw v_mfma_f64_16x16x4: %d wave(s)/SIMD  %.2f TFLOP/s  (%.3f ms/launch)\n", wps, fl / ms / 1e9, ms / 5);
  }
  // GEMM probe: ntile tiles of 128x128, K deep.  distinct: every tile streams its own
  // 128 x K A panel from HBM (B shared, L2); shared: both operands shared (L2 resident).
  for (int bnu : {1, 0})
  for (int K : {256, 1024}) {
    for (int shared : {0, 1}) {
      const int ntile = 2000;
      const long nA = shared ? (long)128 * K : (long)ntile * 128 * K;
      double *A, *B, *C;
      hipMalloc(&A, nA * 8);
      hipMalloc(&B, (long)128 * K * 8);
      hipMalloc(&C, (long)ntile * 128 * 128 * 8);
      if (getenv("ZERO")) { hipMemset(A, 0, nA * 8); hipMemset(B, 0, (long)128 * K * 8); }
      else {
        hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, A, nA);
        hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, B, (long)128 * K);
      }
      const long sA = shared ? 0 : (long)128 * K;
      auto kern = bnu ? k_probe<true> : k_probe<false>;
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, GB_LDS_BYTES);
      hipLaunchKernelGGL(kern, dim3(ntile), dim3(256), GB_LDS_BYTES, 0, A, B, C, K, sA, 0L, 128);
      hipEventRecord(e0);
      for (int r = 0; r < 3; ++r)
        hipLaunchKernelGGL(kern, dim3(ntile), dim3(256), GB_LDS_BYTES, 0, A, B, C, K, sA, 0L, 128);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      double fl = 3.0 * ntile * 2.0 * 128 * 128 * K;
      double by = 3.0 * (shared ? 0.0 : (double)nA * 8);
      printf("B_NU=%d gemm K=%d shared=%d: %.2f TFLOP/s  A-stream %.2f TB/s (%.3f ms/launch)\n", bnu, K, shared,
             fl / ms / 1e9, by / ms / 1e9, ms / 3);
      hipFree(A); hipFree(B); hipFree(C);
    }
  }
  return 0;
}
