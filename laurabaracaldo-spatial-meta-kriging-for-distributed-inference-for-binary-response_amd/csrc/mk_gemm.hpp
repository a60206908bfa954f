// Batched fp64 tile GEMM on CDNA4 MFMA (v_mfma_f64_16x16x4_f64).
//
// One 256-thread workgroup (4 waves, 2x2) owns one TM x TN output tile (TM, TN in {32, 64, 128});
// each wave owns a (TM/2) x (TN/2) quadrant = BM x BN MFMA blocks of 16x16.  K is streamed in
// chunks of 16 straight from HBM into LDS by global_load_lds (LDS-DMA: no staging registers,
// no ds_write pass), two stages deep: chunk c+1 streams in while chunk c is multiplied, one
// barrier per chunk.  128 x 128 kernels stay within 256 registers (__launch_bounds__(256, 2))
// and 2 x 72 KiB of LDS, so two workgroups share a CU and one's waits hide behind the other's
// MFMAs.
//
// Tile shape and bits: every output element accumulates the same MFMA sequence -- the same
// 16-deep chunks in the same order, four k-steps of 4 per chunk, the same fragment values and
// operand order -- whatever TM x TN tile it belongs to.  A 128-tile split into 64-sub-tiles
// therefore gives bit-identical results; the launch code picks the tile shape from how many
// workgroups the launch would have (small shards: 64-sub-tiles fill the 256 CUs), and the
// chains stay independent of the sharding.
//
// Operands are described by strides so that every product the Cholesky / inverse / kriging
// code needs (NT, NN, TN) is the same kernel body:
//   op(A)(m,k) = A[m + k*sA]  (A_MU)   or  A[m*sA + k]  (!A_MU)
//   op(B)(k,n) = B[k*sB + n]  (B_NU)   or  B[k + n*sB]  (!B_NU)
// LDS images (a DMA wave instruction writes 64 lanes x 16 B = 1 KiB lane-linearly):
//   m-contiguous: [k][m], k-row stride 144 / 80 / 48 doubles (128 / 64 / 32-long operand); one
//     instruction per k-row (a shorter row uses the first lanes).  Every stride is 32 mod 64
//     dwords, so the two 16-lane halves of a ds_read_b64 group hit disjoint banks.
//   k-contiguous: [m][16], the 8 k-pairs of row m XOR-swizzled by (m >> 1) & 7.  One
//     instruction fills 8 rows (lane L: row L>>3, slot L&7 holds pair (L&7)^swz); the
//     swizzle is applied to the SOURCE address, so the image stays lane-linear while a
//     fragment read (16 m x 2 k per half-wave) touches 64 distinct banks.
// The MFMA is issued with (B-fragment, A-fragment) so the accumulator holds
// C^T: lane l, register r of block (bm,bn) is C[m = row0 + 16bm + (l&15)][n = col0 + 16bn +
// (l>>4) + 4r] -- consecutive lanes walk consecutive rows of a column-major C
// (coalesced 128-B stores) instead of consecutive columns.
#pragma once
#include "mk_common.hpp"

namespace mk {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));

constexpr int GB_K = 16;                       // K chunk (the k-contiguous image assumes 8 pairs per row)
// m-contiguous image k-row stride: 32 mod 64 dwords for every operand length (bank-disjoint halves)
__host__ __device__ constexpr int gb_stride(int len) {
  return len == 256 ? 272 : (len == 128 ? 144 : (len == 64 ? 80 : 48));
}
__host__ __device__ constexpr int gb_img(int len) { return GB_K * gb_stride(len); }   // >= len * GB_K
// dynamic LDS of a TM x TN tile GEMM: two stages of (A image, B image)
__host__ __device__ constexpr int gb_lds_bytes(int tm, int tn) { return 2 * (gb_img(tm) + gb_img(tn)) * 8; }
static_assert(gb_lds_bytes(128, 128) == MK_GD_LDS_BYTES, "mk_common.hpp LDS size");
static_assert(128 * GB_K <= gb_img(128) && 64 * GB_K <= gb_img(64) && 32 * GB_K <= gb_img(32),
              "k-contiguous images fit their slots");

template <int BM, int BN>
struct AccT {
  d4 v[BM][BN];
};
typedef AccT<4, 4> Acc;   // 128 x 128

template <int BM, int BN>
__device__ inline void acc_zero(AccT<BM, BN>& a) {
#pragma unroll
  for (int i = 0; i < BM; ++i)
#pragma unroll
    for (int j = 0; j < BN; ++j) a.v[i][j] = (d4){0.0, 0.0, 0.0, 0.0};
}

__device__ inline int ku_swz(int m) { return (m >> 1) & 7; }

// LDS-DMA wave instructions one dma_chunk issues per wave (4 waves)
template <bool MU, int LEN>
__host__ __device__ constexpr int dma_count() { return MU ? 4 * (LEN > 128 ? LEN / 128 : 1) : (LEN + 31) / 32; }

// DMA one LEN x 16 chunk of op(X) (k = k0 .. k0+15) into an LDS image.
template <bool MU, int LEN>
__device__ inline void dma_chunk(const double* __restrict__ X, long s, int k0, double* img) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (MU) {
    static_assert(!MU || LEN <= 128 || LEN % 128 == 0, "m-contiguous rows of 128-double pieces");
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = w + 4 * j;
#pragma unroll
      for (int pc = 0; pc < (LEN > 128 ? LEN / 128 : 1); ++pc)   // 1 KiB per wave instruction
        if (LEN >= 128 || lane < LEN / 2)
          __builtin_amdgcn_global_load_lds((const void*)(X + (long)(k0 + r) * s + 128 * pc + 2 * lane),
                                           (void*)(img + r * gb_stride(LEN) + 128 * pc), 16, 0, 0);
    }
  } else {
#pragma unroll
    for (int j = 0; j < (LEN + 31) / 32; ++j) {
      const int m8 = (w + 4 * j) * 8;
      const int m = m8 + (lane >> 3);
      const int pr = (lane & 7) ^ ku_swz(m);
      __builtin_amdgcn_global_load_lds((const void*)(X + (long)m * s + k0 + 2 * pr), (void*)(img + m8 * GB_K), 16, 0,
                                       0);
    }
  }
}

template <bool MU, int LEN>
__device__ inline double frag(const double* img, int m, int k) {
  return MU ? img[k * gb_stride(LEN) + m] : img[m * GB_K + 2 * ((k >> 1) ^ ku_swz(m)) + (k & 1)];
}

// Structural zeros (wave-uniform skips; the skipped MFMAs would add exact zeros or feed
// outputs nobody reads, so results are unchanged and the SIMD's matrix pipe goes to the
// co-resident wave instead).  Block indices are absolute within the 128-tile (rb0 / cb0: the
// sub-tile's offset in 16-blocks), so a sub-tile skips exactly what its 128-tile would:
//   SKIP_UPPER  output tile on the diagonal of a symmetric update: 16-blocks above the
//               diagonal (column block > row block) are never read   (flag = tile is diagonal)
//   SKIP_TRI_B  op(B) lower-triangular in (n, k) over one 128-deep K: chunk c only touches
//               output column blocks >= c                             (flag = chunk index c)
//   SKIP_TRI_A  op(A) lower-triangular in (m, k) over the 128-deep K block starting at diag_tile
//               (gemm_tile): chunk c' of that block only touches output row blocks >= c'
//               (flag = c' inside the block, -1 elsewhere)
//   SKIP_TRI_BL op(B) lower-triangular in (k, n) over the 128-deep K block starting at diag_tile:
//               chunk c' of that block only touches output column blocks <= c'
//               (flag = c' inside the block, SKIP_FLAG_NONE elsewhere)
enum { SKIP_NONE = 0, SKIP_UPPER = 1, SKIP_TRI_B = 2, SKIP_TRI_A = 3, SKIP_TRI_BL = 4 };
constexpr int SKIP_FLAG_NONE = 1 << 20;

// MASK: fragments with chunk-relative k >= kvalid read as zero.
template <int TM, int TN, bool NEG, bool A_MU, bool B_NU, int SKIP, bool MASK>
__device__ inline void mma_chunk(const double* As, const double* Bs, AccT<TM / 32, TN / 32>& acc, int flag,
                                 int kvalid, int rb0, int cb0) {
  constexpr int BM = TM / 32, BN = TN / 32;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w & 1, wn = w >> 1;
  const int li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int ks = 0; ks < GB_K / 4; ++ks) {
    const int k = ks * 4 + lk;
    const bool live = !MASK || k < kvalid;
    double ya[BM], xb[BN];
#pragma unroll
    for (int b = 0; b < BM; ++b) {
      const double av = live ? frag<A_MU, TM>(As, wm * (TM / 2) + b * 16 + li, k) : 0.0;
      ya[b] = NEG ? -av : av;
    }
#pragma unroll
    for (int b = 0; b < BN; ++b) xb[b] = live ? frag<B_NU, TN>(Bs, wn * (TN / 2) + b * 16 + li, k) : 0.0;
#pragma unroll
    for (int bm = 0; bm < BM; ++bm)
#pragma unroll
      for (int bn = 0; bn < BN; ++bn) {
        if (SKIP == SKIP_UPPER && flag && cb0 + wn * BN + bn > rb0 + wm * BM + bm) continue;
        if (SKIP == SKIP_TRI_B && flag > cb0 + wn * BN + bn) continue;
        if (SKIP == SKIP_TRI_A && flag > rb0 + wm * BM + bm) continue;
        if (SKIP == SKIP_TRI_BL && flag < cb0 + wn * BN + bn) continue;
        acc.v[bm][bn] = __builtin_amdgcn_mfma_f64_16x16x4f64(xb[bn], ya[bm], acc.v[bm][bn], 0, 0, 0);
      }
  }
}

// acc += (NEG ? -1 : 1) op(A)[TM x K] * op(B)[K x TN], K % GB_K == 0 (MASK: k >= kvalid_total
// read as zero; the chunk's memory must still be addressable).
// REV: K chunks in descending order -- tiles of one launch whose K ranges share their END
// (triangular operands) then stream the same chunks at the same time, so an XCD's L2
// serves the shared panels once.  SAME: op(B) = op(A)^T read from the same memory (A'A
// products, TM == TN): one DMA and one LDS image serve both fragments.
// SKIP (see mma_chunk): SKIP_UPPER with diag_tile != 0; SKIP_TRI_B for K = 128; SKIP_TRI_A /
// SKIP_TRI_BL with diag_tile = the K offset of the triangular 128-deep block.
// lds: gb_lds_bytes(TM, TN) of dynamic LDS.  Ends with a barrier (the caller may reuse the LDS).
template <int TM, int TN, bool A_MU, bool B_NU, bool NEG = false, bool REV = false, bool SAME = false,
          int SKIP = SKIP_NONE, bool MASK = false>
__device__ inline void gemm_tile(const double* __restrict__ A, long sA, const double* __restrict__ B, long sB, int K,
                                 int kvalid_total, AccT<TM / 32, TN / 32>& acc, double* lds, int diag_tile = 0,
                                 int rb0 = 0, int cb0 = 0) {
  static_assert(!SAME || TM == TN, "SAME needs a square tile");
  constexpr int STAGE = gb_img(TM) + gb_img(TN);
  if (K <= 0) return;
  const int nch = K / GB_K;
  auto k_of = [&](int c) { return REV ? K - GB_K * (c + 1) : GB_K * c; };
  auto issue = [&](int c) {
    double* st = lds + (c & 1) * STAGE;
    dma_chunk<A_MU, TM>(A, sA, k_of(c), st);
    if (!SAME) dma_chunk<B_NU, TN>(B, sB, k_of(c), st + gb_img(TM));
  };
  issue(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    const double* st = lds + (c & 1) * STAGE;
    // the stage chunk c+1 overwrites was last read in iteration c-1, which every wave has left
    if (c + 1 < nch) issue(c + 1);
    const int k0 = k_of(c);
    int flag = diag_tile;
    if (SKIP == SKIP_TRI_B) {
      flag = k0 / GB_K;
    } else if (SKIP == SKIP_TRI_A || SKIP == SKIP_TRI_BL) {
      const int rel = k0 - diag_tile;
      flag = (rel >= 0 && rel < 128) ? rel / GB_K : (SKIP == SKIP_TRI_A ? -1 : SKIP_FLAG_NONE);
    }
    mma_chunk<TM, TN, NEG, A_MU, B_NU, SKIP, MASK>(st, SAME ? st : st + gb_img(TM), acc, flag, kvalid_total - k0,
                                                   rb0, cb0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
}

// acc += op(A)[TM x K] * B[K x TN] with B GENERATED into LDS rather than streamed: gen(k0, img)
// writes chunk k0's [16][TN] m-contiguous image (k-row stride gb_stride(TN)) with plain LDS stores.
// A streams by LDS-DMA as in gemm_tile; chunk c+1's B is generated while chunk c multiplies (the
// stage it overwrites was last read before the previous barrier).  Same MFMA sequence per element
// as gemm_tile<..., A_MU, B_NU = true> on a stored copy of the same values.
template <int TM, int TN, bool A_MU, class Gen>
__device__ inline void gemm_tile_genb(const double* __restrict__ A, long sA, int K, AccT<TM / 32, TN / 32>& acc,
                                      double* lds, Gen&& gen) {
  constexpr int STAGE = gb_img(TM) + gb_img(TN);
  if (K <= 0) return;
  const int nch = K / GB_K;
  dma_chunk<A_MU, TM>(A, sA, 0, lds);
  gen(0, lds + gb_img(TM));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    const double* st = lds + (c & 1) * STAGE;
    if (c + 1 < nch) {
      double* nx = lds + ((c + 1) & 1) * STAGE;
      dma_chunk<A_MU, TM>(A, sA, GB_K * (c + 1), nx);
      gen(GB_K * (c + 1), nx + gb_img(TM));
    }
    mma_chunk<TM, TN, false, A_MU, true, SKIP_NONE, false>(st, st + gb_img(TM), acc, 0, GB_K, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
}

// Row-wave form of a TM x 128 tile, TM in {128, 64} (k_chol_update_trsm): wave w owns rows
// TM/4 * w .. of all 128 columns (TM/64 x 8 MFMA blocks) instead of a quadrant -- the same MFMA
// sequence per element (same chunks, k-steps, fragment values), so the same bits; what changes is
// which wave holds which rows, and a wave then holds whole rows of C: the operand of a solve
// applied from the right.
// Accumulator: lane l, register r of block (bm, bn) is C[TM/4 w + 16bm + (l & 15)][16bn + (l >> 4) + 4r].
template <int TM>
using AccRW = AccT<TM / 64, 8>;
template <int TM>
__device__ inline int rw_row(int bm) { return (threadIdx.x >> 6) * (TM / 4) + bm * 16 + (threadIdx.x & 15); }
__device__ inline int rw_col(int bn, int r) { return bn * 16 + ((threadIdx.x & 63) >> 4) + 4 * r; }

template <int TM, bool NEG>
__device__ inline void mma_chunk_rw(const double* As, const double* Bs, AccRW<TM>& acc) {
  constexpr int BM = TM / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int ks = 0; ks < GB_K / 4; ++ks) {
    const int k = ks * 4 + lk;
    double ya[BM], xb[8];
#pragma unroll
    for (int b = 0; b < BM; ++b) {
      const double av = frag<true, TM>(As, w * (TM / 4) + b * 16 + li, k);
      ya[b] = NEG ? -av : av;
    }
#pragma unroll
    for (int b = 0; b < 8; ++b) xb[b] = frag<true, 128>(Bs, b * 16 + li, k);
#pragma unroll
    for (int bm = 0; bm < BM; ++bm)
#pragma unroll
      for (int bn = 0; bn < 8; ++bn)
        acc.v[bm][bn] = __builtin_amdgcn_mfma_f64_16x16x4f64(xb[bn], ya[bm], acc.v[bm][bn], 0, 0, 0);
  }
}

// gemm_tile<TM, 128, true, true, NEG> in the row-wave form (A m-contiguous, B n-contiguous), K > 0.
template <int TM, bool NEG>
__device__ inline void gemm_tile_rw(const double* __restrict__ A, long sA, const double* __restrict__ B, long sB, int K,
                                    AccRW<TM>& acc, double* lds) {
  constexpr int STAGE = gb_img(TM) + gb_img(128);
  const int nch = K / GB_K;   // K > 0
  auto issue = [&](int c) {
    double* st = lds + (c & 1) * STAGE;
    dma_chunk<true, TM>(A, sA, GB_K * c, st);
    dma_chunk<true, 128>(B, sB, GB_K * c, st + gb_img(TM));
  };
  issue(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    const double* st = lds + (c & 1) * STAGE;
    if (c + 1 < nch) issue(c + 1);
    mma_chunk_rw<TM, NEG>(st, st + gb_img(TM), acc);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
}

template <int TM>
__device__ inline void acc_load_rw(AccRW<TM>& acc, const double* C, long ldc) {
#pragma unroll
  for (int bm = 0; bm < TM / 64; ++bm)
#pragma unroll
    for (int bn = 0; bn < 8; ++bn)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc.v[bm][bn][r] = C[rw_row<TM>(bm) + (long)rw_col(bn, r) * ldc];
}

// The 128 x 128 form every kernel started from.
template <bool A_MU, bool B_NU, bool NEG = false, bool REV = false, bool SAME = false, int SKIP = SKIP_NONE,
          bool MASK = false>
__device__ inline void gemm_128(const double* __restrict__ A, long sA, const double* __restrict__ B, long sB, int K,
                                int kvalid_total, Acc& acc, double* lds, int diag_tile = 0) {
  gemm_tile<128, 128, A_MU, B_NU, NEG, REV, SAME, SKIP, MASK>(A, sA, B, sB, K, kvalid_total, acc, lds, diag_tile);
}

// Element coordinates of accumulator (bm,bn,r) for this lane (within the TM x TN tile).
template <int TM = 128>
__device__ inline int acc_row(int bm) {
  const int lane = threadIdx.x & 63, wm = (threadIdx.x >> 6) & 1;
  return wm * (TM / 2) + bm * 16 + (lane & 15);
}
template <int TN = 128>
__device__ inline int acc_col(int bn, int r) {
  const int lane = threadIdx.x & 63, wn = threadIdx.x >> 7;
  return wn * (TN / 2) + bn * 16 + (lane >> 4) + 4 * r;
}

// acc = C (column-major, ldc): preload for C -= A B^T updates (no read-modify-write epilogue).
template <int BM, int BN>
__device__ inline void acc_load(AccT<BM, BN>& acc, const double* C, long ldc) {
#pragma unroll
  for (int bm = 0; bm < BM; ++bm)
#pragma unroll
    for (int bn = 0; bn < BN; ++bn)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc.v[bm][bn][r] = C[acc_row<BM * 32>(bm) + (long)acc_col<BN * 32>(bn, r) * ldc];
}

// C = acc (column-major, ldc); optional mirrored store C^T at Ct.  Pure stores only:
// accumulating updates preload C into the accumulators (acc_load) and negate the A
// fragment (gemm_tile<..., NEG>), which keeps the kernels at <= 256 registers (2 waves/SIMD).
template <int BM, int BN>
__device__ inline void store_tile(double* C, long ldc, const AccT<BM, BN>& acc, double* Ct = nullptr) {
#pragma unroll
  for (int bm = 0; bm < BM; ++bm)
#pragma unroll
    for (int bn = 0; bn < BN; ++bn)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = acc_row<BM * 32>(bm), n = acc_col<BN * 32>(bn, r);
        C[m + (long)n * ldc] = acc.v[bm][bn][r];
        if (Ct) Ct[n + (long)m * ldc] = acc.v[bm][bn][r];
      }
}

}  // namespace mk
