// Development probe: the left-looking Cholesky panel update k_chol_update on the real
// cfg3 shape (S=250 matrices of 2048^2, random data), block->tile mapping variants.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../laurabaracaldo-spatial-meta-kriging-for-distributed-inference-for-binary-response_amd/csrc/mk_gemm.hpp"
using namespace mk;

__global__ void k_fill(double* p, long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    p[i] = 1e-3 * (double)((i * 2654435761ull) % 1000) - 0.5;
}

// mode 0: s = b / ntk ; mode 1: XCD-aware (matrices m with m % 8 == x served by blocks b % 8 == x)
template <int VAR>
__global__ __launch_bounds__(256, VAR == 0 ? 1 : 2) void k_upd(double* L, int S, int ld, long mstride, int nt, int k, int mode) {
  __shared__ __attribute__((aligned(16))) double lds[GB_LDS_DOUBLES];
  const int ntk = nt - k;
  int s, i;
  if (mode == 0) {
    s = blockIdx.x / ntk; i = k + blockIdx.x % ntk;
  } else {
    const int x = blockIdx.x % 8, j = blockIdx.x / 8;
    const int ms = j / ntk;
    s = x + 8 * ms; i = k + j % ntk;
    if (s >= S) return;
  }
  double* M = L + (long)s * mstride;
  Acc acc;
  double* C = M + i * MK_NB + (long)k * MK_NB * ld;
  if (VAR == 0) {
    acc_zero(acc);
    gemm_128<true, true>(M + i * MK_NB, ld, M + k * MK_NB, ld, k * MK_NB, k * MK_NB, acc, lds);
    store_tile(C, ld, acc, -1.0, 1.0);
  } else {
    acc_load(acc, C, ld);
    gemm_128<true, true, true>(M + i * MK_NB, ld, M + k * MK_NB, ld, k * MK_NB, k * MK_NB, acc, lds);
    store_tile(C, ld, acc, 1.0, 0.0);
  }
}

int main() {
  const int S = 250, nt = 16;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int pad : {0}) {
    const int ld = 2048 + pad;
    const long mstride = (long)ld * 2048 + (pad ? 512 : 0);
    double* L;
    hipMalloc(&L, (size_t)S * mstride * 8);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, L, (long)S * mstride);
    for (int var : {0, 1}) for (int mode : {1}) {
      double tot_ms = 0, tot_fl = 0;
      printf("var %d mode %d:", var, mode);
      for (int k = 1; k < nt; ++k) {
        const int ntk = nt - k;
        const int grid = (mode == 0) ? S * ntk : 8 * ((S + 7) / 8) * ntk;
        hipEventRecord(e0);
        if (var == 0) hipLaunchKernelGGL(k_upd<0>, dim3(grid), dim3(256), 0, 0, L, S, ld, mstride, nt, k, mode);
        else hipLaunchKernelGGL(k_upd<1>, dim3(grid), dim3(256), 0, 0, L, S, ld, mstride, nt, k, mode);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double fl = 2.0 * 128 * 128 * 128.0 * k * ntk * S;
        tot_ms += ms; tot_fl += fl;
        if (k % 3 == 1 || k == 15) printf(" k%d %.1fTF", k, fl / ms / 1e9);
      }
      printf(" | total %.2f ms %.1f TF\n", tot_ms, tot_fl / tot_ms / 1e9);
    }
    hipFree(L);
  }
  return 0;
}
