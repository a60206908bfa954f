// Development probe: HBM write rate of the candidate kernel's store pattern (one 128 x 128 fp64
// tile per 256-thread workgroup, 16-byte row-pair stores, column stride ld) with and without the
// exp(-phi d) arithmetic, over 250 matrices of 2048^2 (lower tiles only, as k_cov_candidate).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/store_probe.hip -o tools/store_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ __launch_bounds__(256) void k_store(double* M, const double* cx, const double* cy, int nt, long ld, double phi) {
  const int ntiles = nt * (nt + 1) / 2;
  const int e = blockIdx.x / ntiles, t = blockIdx.x % ntiles;
  int ti = 0;
  while ((ti + 1) * (ti + 2) / 2 <= t) ++ti;
  const int tj = t - ti * (ti + 1) / 2;
  double* Mm = M + (long)e * ld * ld;
  const double* x = cx + (long)e * ld;
  const double* y = cy + (long)e * ld;
  const int R = ti * 128 + (threadIdx.x & 63) * 2;
  const double x0 = x[R], y0 = y[R], x1 = x[R + 1], y1 = y[R + 1];
  for (int cc = threadIdx.x >> 6; cc < 128; cc += 4) {
    const int C = tj * 128 + cc;
    if (ti == tj && R + 1 < C) continue;
    d2 v;
    if (MODE == 0) {
      v.x = 0.5; v.y = 0.25;
    } else {
      const double xc = x[C], yc = y[C];
      const double dx0 = x0 - xc, dy0 = y0 - yc, dx1 = x1 - xc, dy1 = y1 - yc;
      v.x = exp(-phi * sqrt(dx0 * dx0 + dy0 * dy0));
      v.y = exp(-phi * sqrt(dx1 * dx1 + dy1 * dy1));
    }
    *reinterpret_cast<d2*>(Mm + R + (long)C * ld) = v;
  }
}

int main() {
  const int S = 250, nt = 16;
  const long ld = 2048;
  double *M, *cx, *cy;
  hipMalloc(&M, (size_t)S * ld * ld * 8);
  hipMalloc(&cx, (size_t)S * ld * 8);
  hipMalloc(&cy, (size_t)S * ld * 8);
  hipMemset(cx, 0, (size_t)S * ld * 8);
  hipMemset(cy, 0, (size_t)S * ld * 8);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  const int grid = S * nt * (nt + 1) / 2;
  const double bytes = (double)S * (nt * (nt - 1) / 2 * 128.0 * 128.0 + nt * (128.0 * 129.0 / 2 + 64)) * 8;
  for (int mode = 0; mode < 2; ++mode) {
    float best = 1e9;
    for (int r = 0; r < 6; ++r) {
      hipEventRecord(a);
      if (mode == 0) hipLaunchKernelGGL(k_store<0>, dim3(grid), dim3(256), 0, 0, M, cx, cy, nt, ld, 6.0);
      else hipLaunchKernelGGL(k_store<1>, dim3(grid), dim3(256), 0, 0, M, cx, cy, nt, ld, 6.0);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      if (ms < best) best = ms;
    }
    printf("mode %d (%s): %.3f ms, %.2f TB/s of stores\n", mode, mode ? "exp(-phi d)" : "constants", best,
           bytes / (best * 1e-3) / 1e12);
  }
  return 0;
}
