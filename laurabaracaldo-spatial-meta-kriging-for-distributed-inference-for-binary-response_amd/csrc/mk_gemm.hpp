// Batched fp64 128x128 tile GEMM on CDNA4 MFMA (v_mfma_f64_16x16x4_f64).
//
// One 256-thread workgroup (4 waves, 2x2) owns one 128x128 output tile; each
// wave owns a 64x64 quadrant = 4x4 MFMA blocks (64 fp64 accumulators/lane).
// K is streamed in chunks of 16 through LDS ([k][m] images, row stride 144
// doubles so the two 16-lane halves of a ds_read_b64 group land on disjoint
// banks), register-prefetching chunk c+1 while chunk c is multiplied.  Kernels
// built on it stay within 256 registers (__launch_bounds__(256, 2)) so two
// workgroups share a CU and one's HBM stalls hide behind the other's MFMAs
// (measured on the cfg3 Cholesky update: 35.8 -> 56.2 TFLOP/s).
//
// Operands are described by strides so that every product the Cholesky /
// inverse / kriging code needs (NT, NN, TN) is the same kernel body:
//   op(A)(m,k) = A[m + k*sA]  (A_MU)   or  A[m*sA + k]  (!A_MU)
//   op(B)(k,n) = B[k*sB + n]  (B_NU)   or  B[k + n*sB]  (!B_NU)
// The MFMA is issued with (B-fragment, A-fragment) so the accumulator holds
// C^T: lane l, register r of block (bm,bn) is C[m = 16bm + (l&15)][n = 16bn +
// (l>>4) + 4r] -- consecutive lanes walk consecutive rows of a column-major C
// (coalesced 128-B stores) instead of consecutive columns.
#pragma once
#include "mk_common.hpp"

namespace mk {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));

#ifndef MK_GB_K
#define MK_GB_K 16
#endif
constexpr int GB_K = MK_GB_K;  // K chunk
constexpr int GB_SM = 144;     // LDS row stride (doubles) for m-contiguous operands
// k-contiguous operands are transposed while stored to LDS; an odd stride spreads
// the 8 k values a 16-lane ds_write group stores for one m over distinct banks.
constexpr int GB_SMT = 145;
template <bool MU> constexpr int sm_of() { return MU ? GB_SM : GB_SMT; }
constexpr int GB_LDS_DOUBLES = 2 * GB_K * GB_SMT;
constexpr int GB_PER = GB_K / 4;   // d2 loads per thread per operand per chunk

struct Acc {
  d4 v[4][4];
};

__device__ inline void acc_zero(Acc& a) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) a.v[i][j] = (d4){0.0, 0.0, 0.0, 0.0};
}

// Load one 128 x 16 chunk of op(X) into registers (8 doubles per thread).
// `kvalid`: elements with chunk-relative k >= kvalid are zero (K masking).
template <bool MU>
__device__ inline void load_chunk(const double* __restrict__ X, long s, int k0, int kvalid, d2 (&r)[GB_PER]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < GB_PER; ++i) {
    const int e = t + 256 * i;
    if (MU) {
      const int k = e >> 6, m = (e & 63) * 2;
      r[i] = (k < kvalid) ? *reinterpret_cast<const d2*>(X + m + (long)(k0 + k) * s) : (d2){0.0, 0.0};
    } else {
      const int k = (e % (GB_K / 2)) * 2, m = e / (GB_K / 2);
      d2 v = *reinterpret_cast<const d2*>(X + (long)m * s + k0 + k);
      if (k >= kvalid) v.x = 0.0;
      if (k + 1 >= kvalid) v.y = 0.0;
      r[i] = v;
    }
  }
}

template <bool MU>
__device__ inline void store_chunk(double* lds, const d2 (&r)[GB_PER]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < GB_PER; ++i) {
    const int e = t + 256 * i;
    if (MU) {
      const int k = e >> 6, m = (e & 63) * 2;
      *reinterpret_cast<d2*>(lds + k * GB_SM + m) = r[i];
    } else {
      const int k = (e % (GB_K / 2)) * 2, m = e / (GB_K / 2);
      lds[k * GB_SMT + m] = r[i].x;
      lds[(k + 1) * GB_SMT + m] = r[i].y;
    }
  }
}

// Structural zeros (wave-uniform skips; the skipped MFMAs would add exact zeros or feed
// outputs nobody reads, so results are unchanged and the SIMD's matrix pipe goes to the
// co-resident wave instead):
//   SKIP_UPPER  output tile on the diagonal of a symmetric update: 16-blocks above the
//               diagonal (column block > row block) are never read   (flag = tile is diagonal)
//   SKIP_TRI_B  op(B) lower-triangular in (n, k) over one 128-deep K: chunk c only touches
//               output column blocks >= c                             (flag = chunk index c)
//   SKIP_WAVE   the calling wave's whole 64x64 quadrant is unused        (flag = skip this wave)
enum { SKIP_NONE = 0, SKIP_UPPER = 1, SKIP_TRI_B = 2, SKIP_WAVE = 3 };

template <bool NEG = false, int SA = GB_SM, int SB = GB_SM, int SKIP = SKIP_NONE>
__device__ inline void mma_chunk(const double* As, const double* Bs, Acc& acc, int flag = 0) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w & 1, wn = w >> 1;
  const int li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int ks = 0; ks < GB_K / 4; ++ks) {
    double ya[4], xb[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const double av = As[(ks * 4 + lk) * SA + wm * 64 + b * 16 + li];
      ya[b] = NEG ? -av : av;
      xb[b] = Bs[(ks * 4 + lk) * SB + wn * 64 + b * 16 + li];
    }
#pragma unroll
    for (int bm = 0; bm < 4; ++bm)
#pragma unroll
      for (int bn = 0; bn < 4; ++bn) {
        if (SKIP == SKIP_UPPER && flag && wn * 4 + bn > wm * 4 + bm) continue;
        if (SKIP == SKIP_TRI_B && flag > wn * 4 + bn) continue;
        acc.v[bm][bn] = __builtin_amdgcn_mfma_f64_16x16x4f64(xb[bn], ya[bm], acc.v[bm][bn], 0, 0, 0);
      }
  }
}

// acc += (NEG ? -1 : 1) op(A)[128 x K] * op(B)[K x 128], K % GB_K == 0; k >= kvalid_total zeroed.
// REV: K chunks in descending order -- tiles of one launch whose K ranges share their END
// (triangular operands) then stream the same chunks at the same time, so an XCD's L2
// serves the shared panels once.  SAME: op(B) = op(A)^T read from the same memory (A'A
// products): one load and one LDS image serve both fragments.
// SKIP (see mma_chunk): SKIP_UPPER with diag_tile != 0; SKIP_TRI_B for K = 128.
template <bool A_MU, bool B_NU, bool NEG = false, bool REV = false, bool SAME = false, int SKIP = SKIP_NONE>
__device__ inline void gemm_128(const double* __restrict__ A, long sA, const double* __restrict__ B, long sB,
                                int K, int kvalid_total, Acc& acc, double* lds, int diag_tile = 0) {
  double* As = lds;
  double* Bs = SAME ? lds : lds + GB_K * GB_SMT;
  d2 ra[GB_PER], rb[GB_PER];
  if (K <= 0) return;
  const int k_first = REV ? K - GB_K : 0;
  load_chunk<A_MU>(A, sA, k_first, kvalid_total - k_first, ra);
  if (!SAME) load_chunk<B_NU>(B, sB, k_first, kvalid_total - k_first, rb);
  for (int kc = 0; kc < K; kc += GB_K) {
    __syncthreads();
    store_chunk<A_MU>(As, ra);
    if (!SAME) store_chunk<B_NU>(Bs, rb);
    __syncthreads();
    if (kc + GB_K < K) {
      const int k1 = REV ? K - 2 * GB_K - kc : kc + GB_K;
      load_chunk<A_MU>(A, sA, k1, kvalid_total - k1, ra);
      if (!SAME) load_chunk<B_NU>(B, sB, k1, kvalid_total - k1, rb);
    }
    if (SKIP == SKIP_WAVE) {
      if (!diag_tile) mma_chunk<NEG, sm_of<A_MU>(), sm_of<B_NU>()>(As, Bs, acc);
    } else {
      mma_chunk<NEG, sm_of<A_MU>(), sm_of<B_NU>(), SKIP>(As, Bs, acc,
                                                         SKIP == SKIP_TRI_B ? (REV ? K - GB_K - kc : kc) / GB_K : diag_tile);
    }
  }
}

// LDS-DMA variant for operands whose 128 m (n) values per k are contiguous (A_MU, B_NU) and
// K fully valid: each k-row of a chunk is ONE global_load_lds_dwordx4 wave instruction
// (64 lanes x 16 B = the 1 KiB row; rows padded to GB_SM, no instruction crosses a row), so
// the chunk lands in LDS with no staging registers and no ds_write pass.  Two stages: chunk
// c+1 streams in while chunk c is multiplied; one barrier per chunk (its vmcnt(0) retires
// the DMA, and every wave has finished reading the stage the next DMA overwrites).
constexpr int GD_STAGE = 2 * GB_K * GB_SM;                 // A + B images of one chunk
constexpr int GD_LDS_BYTES = 2 * GD_STAGE * 8;             // two stages
static_assert(GD_LDS_BYTES == MK_GD_LDS_BYTES, "mk_common.hpp LDS size");
template <bool NEG = false, int SKIP = SKIP_NONE>
__device__ inline void gemm_128_dma(const double* __restrict__ A, long sA, const double* __restrict__ B, long sB,
                                    int K, Acc& acc, double* lds) {
  if (K <= 0) return;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  auto issue = [&](int k0, double* st) {
#pragma unroll
    for (int r = w; r < GB_K; r += 4) {
      __builtin_amdgcn_global_load_lds((const void*)(A + (long)(k0 + r) * sA + 2 * lane), (void*)(st + r * GB_SM),
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(B + (long)(k0 + r) * sB + 2 * lane),
                                       (void*)(st + (GB_K + r) * GB_SM), 16, 0, 0);
    }
  };
  issue(0, lds);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int cur = 0;
  for (int kc = 0; kc < K; kc += GB_K) {
    double* st = lds + cur * GD_STAGE;
    if (kc + GB_K < K) issue(kc + GB_K, lds + (cur ^ 1) * GD_STAGE);
    mma_chunk<NEG, GB_SM, GB_SM, SKIP>(st, st + GB_K * GB_SM, acc, SKIP == SKIP_TRI_B ? kc / GB_K : 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    cur ^= 1;
  }
}

// acc = C (column-major, ldc): preload for C -= A B^T updates (no read-modify-write epilogue).
__device__ inline void acc_load(Acc& acc, const double* C, long ldc);

// Element coordinates of accumulator (bm,bn,r) for this lane.
__device__ inline int acc_row(int bm) {
  const int lane = threadIdx.x & 63, wm = (threadIdx.x >> 6) & 1;
  return wm * 64 + bm * 16 + (lane & 15);
}
__device__ inline int acc_col(int bn, int r) {
  const int lane = threadIdx.x & 63, wn = threadIdx.x >> 7;
  return wn * 64 + bn * 16 + (lane >> 4) + 4 * r;
}

__device__ inline void acc_load(Acc& acc, const double* C, long ldc) {
#pragma unroll
  for (int bm = 0; bm < 4; ++bm)
#pragma unroll
    for (int bn = 0; bn < 4; ++bn)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc.v[bm][bn][r] = C[acc_row(bm) + (long)acc_col(bn, r) * ldc];
}

// C = acc (column-major, ldc); optional mirrored store C^T at Ct.  Pure stores only:
// accumulating updates preload C into the accumulators (acc_load) and negate the A
// fragment (gemm_128<..., NEG>), which keeps the kernels at <= 256 registers (2 waves/SIMD).
__device__ inline void store_tile(double* C, long ldc, const Acc& acc, double* Ct = nullptr) {
#pragma unroll
  for (int bm = 0; bm < 4; ++bm)
#pragma unroll
    for (int bn = 0; bn < 4; ++bn)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = acc_row(bm), n = acc_col(bn, r);
        C[m + (long)n * ldc] = acc.v[bm][bn][r];
        if (Ct) Ct[n + (long)m * ldc] = acc.v[bm][bn][r];
      }
}

}  // namespace mk
