// Tile-GEMM body variants for the left-looking Cholesky update (development tool, not shipped).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 tools/gemm_probe2.hip -o tools/gemm_probe2
//
// The update's access pattern: S matrices of ld x ld (column-major), column k of 128-tiles,
// C(i,k) -= L(i, 0:k) L(k, 0:k)^T for the tiles i = k .. k+T-1 (A: the tile's own row panel,
// streamed; B: the column's row panel, shared by the subset's tiles).  Output to a separate buffer
// (acc preloaded from C), so every variant sees the same inputs and the results compare bit for bit.
//
// Variants (per element the same MFMA sequence as mk::gemm_tile: 16-deep chunks in k order, four
// k-steps of 4, operands issued (B-fragment, A-fragment)):
//   V0  mk::gemm_tile<128,128>           4 waves, 2 LDS stages, 2 workgroups / CU (the shipped body)
//   G<TM, WM, WN, ST>                    TM x 128 tile, WM x WN waves, ST LDS stages (prefetch ST-1
//                                        chunks ahead, one barrier per chunk)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../laurabaracaldo-spatial-meta-kriging-for-distributed-inference-for-binary-response_amd/csrc/mk_gemm.hpp"
using namespace mk;

__host__ __device__ constexpr int stride_of(int len) { return len == 256 ? 272 : (len == 128 ? 144 : 80); }

__global__ void k_fill(double* p, long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    p[i] = 1e-3 * (double)((i * 2654435761ull) % 1000) - 0.5;
}

// V0: the shipped body, one 128 x 128 tile per workgroup
__global__ __launch_bounds__(256, 2) void k_v0(const double* M, double* out, int ld, long mstride, int k, int T) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int s = blockIdx.x / T, i = k + blockIdx.x % T;
  const double* Ms = M + s * mstride;
  const double* C = Ms + i * 128 + (long)(k * 128) * ld;
  Acc acc;
  acc_load(acc, C, ld);
  gemm_tile<128, 128, true, true, true>(Ms + i * 128, ld, Ms + k * 128, ld, k * 128, k * 128, acc, lds);
  store_tile(out + (long)blockIdx.x * 128 * 128, 128, acc);
}

template <int LEN, int NW>
__device__ inline void dma(const double* X, long s, int k0, double* img) {
  constexpr int PER_ROW = LEN / 128;              // wave instructions per k-row (1 KiB each)
  constexpr int R = 16 * PER_ROW;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < R / NW; ++j) {
    const int r = w + NW * j;
    const int row = r / PER_ROW, half = r % PER_ROW;
    __builtin_amdgcn_global_load_lds((const void*)(X + (long)(k0 + row) * s + half * 128 + 2 * lane),
                                     (void*)(img + row * stride_of(LEN) + half * 128), 16, 0, 0);
  }
}

template <int N>
__device__ inline void wait_vm() {
  static_assert(N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

template <int TM, int WM, int WN, int ST>
__global__ __launch_bounds__(64 * WM * WN, 1) void k_g(const double* M, double* out, int ld, long mstride, int k,
                                                       int T) {
  constexpr int NW = WM * WN, TN = 128;
  constexpr int BM = TM / WM / 16, BN = TN / WN / 16;
  constexpr int SA = stride_of(TM), SB = stride_of(TN);
  constexpr int STAGE = 16 * SA + 16 * SB;
  constexpr int PER = (16 * (TM / 128) + 16) / NW;   // DMA instructions per wave per chunk
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int RT = TM / 128;                           // 128-row tiles per workgroup
  const int TW = (T + RT - 1) / RT;
  const int s = blockIdx.x / TW, i = k + (blockIdx.x % TW) * RT;
  const double* Ms = M + s * mstride;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w % WM, wn = w / WM;
  const int li = lane & 15, lk = lane >> 4;
  d4 acc[BM][BN];
#pragma unroll
  for (int bm = 0; bm < BM; ++bm)
#pragma unroll
    for (int bn = 0; bn < BN; ++bn)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = wm * (TM / WM) + bm * 16 + li, n = wn * (TN / WN) + bn * 16 + lk + 4 * r;
        acc[bm][bn][r] = Ms[i * 128 + m + (long)(k * 128 + n) * ld];
      }
  const double* A = Ms + i * 128;
  const double* B = Ms + k * 128;
  const int nch = k * 128 / 16;
#pragma unroll
  for (int c = 0; c < ST - 1; ++c)
    if (c < nch) {
      dma<TM, NW>(A, ld, 16 * c, lds + c * STAGE);
      dma<TN, NW>(B, ld, 16 * c, lds + c * STAGE + 16 * SA);
    }
  for (int c = 0; c < nch; ++c) {
    // chunk c landed (chunks c+1 .. c+ST-2 may still be in flight), and every wave is past chunk c-1
    if (c + ST - 2 < nch) wait_vm<PER * (ST - 2)>();
    else wait_vm<0>();
    __syncthreads();
    if (c + ST - 1 < nch) {
      double* st = lds + ((c + ST - 1) % ST) * STAGE;
      dma<TM, NW>(A, ld, 16 * (c + ST - 1), st);
      dma<TN, NW>(B, ld, 16 * (c + ST - 1), st + 16 * SA);
    }
    const double* As = lds + (c % ST) * STAGE;
    const double* Bs = As + 16 * SA;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int kk = ks * 4 + lk;
      double ya[BM], xb[BN];
#pragma unroll
      for (int b = 0; b < BM; ++b) ya[b] = -As[kk * SA + wm * (TM / WM) + b * 16 + li];
#pragma unroll
      for (int b = 0; b < BN; ++b) xb[b] = Bs[kk * SB + wn * (TN / WN) + b * 16 + li];
#pragma unroll
      for (int bm = 0; bm < BM; ++bm)
#pragma unroll
        for (int bn = 0; bn < BN; ++bn)
          acc[bm][bn] = __builtin_amdgcn_mfma_f64_16x16x4f64(xb[bn], ya[bm], acc[bm][bn], 0, 0, 0);
    }
  }
  // out: the 128-tiles of this workgroup in V0's order (tile index blockIdx-equivalent)
#pragma unroll
  for (int bm = 0; bm < BM; ++bm)
#pragma unroll
    for (int bn = 0; bn < BN; ++bn)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = wm * (TM / WM) + bm * 16 + li, n = wn * (TN / WN) + bn * 16 + lk + 4 * r;
        const int sub = m / 128;
        const long tile = (long)s * T + (i - k) + sub;
        if (i - k + sub < T) out[tile * 128 * 128 + (m % 128) + n * 128] = acc[bm][bn][r];
      }
}

static double run(const char* name, void (*kern)(const double*, double*, int, long, int, int), int wgs, int threads,
                  int lds, const double* M, double* out, int ld, long ms, int k, int T, double flops) {
  hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipLaunchKernelGGL(kern, dim3(wgs), dim3(threads), lds, 0, M, out, ld, ms, k, T);
  if (hipDeviceSynchronize() != hipSuccess) {
    printf("%s: launch failed\n", name);
    exit(1);
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(wgs), dim3(threads), lds, 0, M, out, ld, ms, k, T);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms_;
  hipEventElapsedTime(&ms_, e0, e1);
  const double t = ms_ / reps;
  printf("%-34s k=%2d T=%2d wgs=%5d lds=%6d: %7.3f ms  %6.2f TFLOP/s\n", name, k, T, wgs, lds, t, flops / t / 1e9);
  return t;
}

int main() {
  const int S = 250, ld = 2048;
  const long mstride = (long)ld * ld;
  double *M, *o0, *o1;
  hipMalloc(&M, S * mstride * 8);
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, M, S * mstride);
  const long omax = (long)S * 16 * 128 * 128;
  hipMalloc(&o0, omax * 8);
  hipMalloc(&o1, omax * 8);
  std::vector<double> h0(omax), h1(omax);
  for (int k : {2, 8, 12}) {
    const int T = 15 - k + 1;                     // tiles k .. 15
    const long n_out = (long)S * T * 128 * 128;
    const double flops = 2.0 * S * T * 128.0 * 128.0 * (k * 128.0);
    run("V0 gemm_tile<128,128> 4w 2st x2", k_v0, S * T, 256, gb_lds_bytes(128, 128), M, o0, ld, mstride, k, T, flops);
    hipMemcpy(h0.data(), o0, n_out * 8, hipMemcpyDeviceToHost);
    auto check = [&](const char* name) {
      hipMemcpy(h1.data(), o1, n_out * 8, hipMemcpyDeviceToHost);
      const bool same = memcmp(h0.data(), h1.data(), n_out * 8) == 0;
      printf("    %s %s\n", name, same ? "bit-identical to V0" : "DIFFERS from V0");
    };
    constexpr int L3_128 = 3 * (16 * 144 + 16 * 144) * 8, L2_256 = 2 * (16 * 272 + 16 * 144) * 8,
                  L3_256 = 3 * (16 * 272 + 16 * 144) * 8, L2_128 = 2 * (16 * 144 + 16 * 144) * 8;
    run("G<128,2,2,3> 4w 3st x1", k_g<128, 2, 2, 3>, S * T, 256, L3_128, M, o1, ld, mstride, k, T, flops);
    check("G<128,2,2,3>");
    run("G<128,2,4,3> 8w 3st x1", k_g<128, 2, 4, 3>, S * T, 512, L3_128, M, o1, ld, mstride, k, T, flops);
    check("G<128,2,4,3>");
    run("G<128,2,4,2> 8w 2st", k_g<128, 2, 4, 2>, S * T, 512, L2_128, M, o1, ld, mstride, k, T, flops);
    check("G<128,2,4,2>");
    const int TW = (T + 1) / 2;
    run("G<256,4,2,2> 8w 2st x1", k_g<256, 4, 2, 2>, S * TW, 512, L2_256, M, o1, ld, mstride, k, T, flops);
    check("G<256,4,2,2>");
    run("G<256,4,2,3> 8w 3st x1", k_g<256, 4, 2, 3>, S * TW, 512, L3_256, M, o1, ld, mstride, k, T, flops);
    check("G<256,4,2,3>");
  }
  return 0;
}
