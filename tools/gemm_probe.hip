// Micro-benchmark for the fp64 MFMA tile GEMM (development tool, not shipped).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/gemm_probe.hip -o tools/gemm_probe
// 1) raw v_mfma_f64_16x16x4 throughput (registers only): NACC independent accumulators per
//    wave, W waves per SIMD -- how many independent chains hide the MFMA latency
// 2) mk::gemm_tile<TM, TM> (the Cholesky update's NT form) on batched TM x K panels, operands
//    distinct per tile (streamed) or shared (L2-resident), TM = 128 / 64 / 32
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../laurabaracaldo-spatial-meta-kriging-for-distributed-inference-for-binary-response_amd/csrc/mk_gemm.hpp"
using namespace mk;

template <int NACC>
__global__ __launch_bounds__(256) void k_mfma_peak(double* out, int iters) {
  d4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = (d4){0, 0, 0, 0};
  double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 12345.0) out[threadIdx.x] = s;
}

__global__ void k_fill(double* p, long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    p[i] = 1e-3 * (double)((i * 2654435761ull) % 1000) - 0.5;
}

template <int TM>
__global__ __launch_bounds__(256, 2) void k_probe(const double* A, const double* B, double* C, int K, long strideA,
                                               int lda) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const double* a = A + blockIdx.x * strideA;
  AccT<TM / 32, TM / 32> acc;
  acc_zero(acc);
  gemm_tile<TM, TM, true, true, true>(a, lda, B, lda, K, K, acc, lds);
  store_tile(C + (long)blockIdx.x * TM * TM, TM, acc);
}

template <int NACC>
static void raw(double* out, hipEvent_t e0, hipEvent_t e1) {
  const int iters = 2000;
  for (int wps : {1, 2, 4}) {
    const int grid = 256 * wps;
    hipLaunchKernelGGL(k_mfma_peak<NACC>, dim3(grid), dim3(256), 0, 0, out, iters);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_mfma_peak<NACC>, dim3(grid), dim3(256), 0, 0, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double fl = 5.0 * grid * 4.0 * NACC * (double)iters * 2048;   // 2048 flops per wave-MFMA
    printf("raw mfma_f64_16x16x4: %2d acc/wave %d wave(s)/SIMD  %.2f TFLOP/s\n", NACC, wps, fl / ms / 1e9);
  }
}

template <int TM>
static void probe(int K, int shared, int ntile) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const long nA = shared ? (long)TM * K : (long)ntile * TM * K;
  double *A, *B, *C;
  hipMalloc(&A, nA * 8);
  hipMalloc(&B, (long)TM * K * 8);
  hipMalloc(&C, (long)ntile * TM * TM * 8);
  hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, A, nA);
  hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, B, (long)TM * K);
  const long sA = shared ? 0 : (long)TM * K;
  const int lds = gb_lds_bytes(TM, TM);
  hipFuncSetAttribute((const void*)k_probe<TM>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipLaunchKernelGGL(k_probe<TM>, dim3(ntile), dim3(256), lds, 0, A, B, C, K, sA, TM);
  hipEventRecord(e0);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k_probe<TM>, dim3(ntile), dim3(256), lds, 0, A, B, C, K, sA, TM);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double fl = 3.0 * ntile * 2.0 * TM * TM * K;
  printf("gemm_tile<%3d> K=%4d %s tiles=%5d: %.2f TFLOP/s  (%.3f ms/launch)\n", TM, K, shared ? "L2 " : "HBM", ntile,
         fl / ms / 1e9, ms / 3);
  hipFree(A);
  hipFree(B);
  hipFree(C);
}

int main() {
  double* out;
  hipMalloc(&out, 4096 * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  raw<1>(out, e0, e1);
  raw<2>(out, e0, e1);
  raw<4>(out, e0, e1);
  raw<16>(out, e0, e1);
  for (int K : {256, 1024})
    for (int shared : {0, 1}) {
      probe<128>(K, shared, 2048);
      probe<64>(K, shared, 8192);
      probe<64>(K, shared, 1024);
      probe<32>(K, shared, 32768);
    }
  return 0;
}
