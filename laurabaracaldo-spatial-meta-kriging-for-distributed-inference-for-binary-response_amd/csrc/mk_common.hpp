// Shared device helpers for libmk (gfx950 / CDNA4 only).
//
// Philox4x32-10 is the bit-exact twin of oracle/philox.py; every random draw
// of the sampler and of the kriging step is a pure function of
// (seed, subset, index, iteration, tag) so the device chain can be replayed on
// the host.  Stream layout documented in oracle/philox.py and DESIGN.md.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MK_NB 128          // Cholesky / GEMM tile edge (fp64)
#define MK_SS_T 256        // threads of the site sweep workgroup (k_sweep_site: one wave per SIMD)
#define MK_SW_T 1024       // threads of the latent-w sweep workgroup (one per subset): loads in flight for the W panels
// k_sweep_mg's per-subset admission word: arrival count | aborted | swept (k_sweep's fallback skips it)
constexpr int MK_ADM_COUNT = 0xffff, MK_ADM_ABORT = 1 << 16, MK_ADM_DONE = 1 << 17;
// bounded admission wait: ~2^15 x s_sleep 2 (~128 cycles) ~ 2 ms -- above the other streams' longest
// kernels at small shards, which the sweep's missing workgroups may wait behind for CUs
constexpr int MK_ADM_SPINS = 1 << 15;   // MK_ADM_SPINS overrides (tests: 0 sends some subsets to the fallback, -1 all)
// dynamic LDS of the LDS-DMA GEMM (k_chol_update): 2 stages x (A, B) x 16 k-rows x 144 doubles
#define MK_GD_LDS_BYTES (2 * 2 * 16 * 144 * 8)
#define MK_CAND_NOBORDER 4  // k_cov_candidate `which` flag: no bordered row (lookahead schedule)
                            // (MK_COV_FUSE: the update kernel generates every other tile at its first touch)
#define MK_TLD 129         // LDS column stride of the diagonal-tile factor/inverse (k_chol_diag)
// dynamic LDS of k_chol_diag: tile + diag(L) + diag(L^-1) + 7 16 x 17 inverse stagings
#define MK_DIAG_LDS_BYTES ((MK_NB * MK_TLD + 2 * MK_NB + 7 * 16 * 17) * 8)
#define MK_TAG_PROPOSAL 1u
#define MK_TAG_PREDICT 2u
#define MK_TAG_RESAMPLE 3u

#define MK_TWO_PI 6.283185307179586
#define MK_SQRT1_2 0.7071067811865476
// binomial links: logit is the reference's (spMvGLM's binomial family, MK.R:80-84, 160);
// probit is the north-star extension ("logit/probit latent-GP"), no reference parity target
#define MK_LINK_LOGIT 0
#define MK_LINK_PROBIT 1
#define MK_TWO_M52 2.220446049250313e-16   // 2^-52

namespace mk {

typedef double d2 __attribute__((ext_vector_type(2)));   // 16-byte fp64 pair loads/stores

struct Key { uint32_t k0, k1; };

__host__ __device__ inline Key make_key(uint64_t seed, uint32_t subset) {
  Key k;
  k.k0 = (uint32_t)(seed & 0xFFFFFFFFull);
  k.k1 = (uint32_t)(seed >> 32) + subset;
  return k;
}

__device__ inline uint4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, Key key) {
  uint32_t k0 = key.k0, k1 = key.k1;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
  }
  return make_uint4(c0, c1, c2, c3);
}

__device__ inline double u01_open(uint32_t hi, uint32_t lo) {
  const uint64_t top52 = ((((uint64_t)hi) << 32) | (uint64_t)lo) >> 12;
  return ((double)top52 + 0.5) * MK_TWO_M52;
}

__device__ inline double normal_from(uint4 w) {
  const double u1 = u01_open(w.x, w.y), u2 = u01_open(w.z, w.w);
  return sqrt(-2.0 * log(u1)) * cos(MK_TWO_PI * u2);
}

// N(0,1) proposal for MH parameter j at iteration s.
__device__ inline double proposal_normal(Key key, uint32_t j, uint32_t s) {
  return normal_from(philox(j, s, MK_TAG_PROPOSAL, 0u, key));
}
// log U accept draw for MH parameter j at iteration s.
__device__ inline double accept_log_uniform(Key key, uint32_t j, uint32_t s) {
  const uint4 w = philox(j, s, MK_TAG_PROPOSAL, 1u, key);
  return log(u01_open(w.x, w.y));
}
__device__ inline double predict_normal(Key key, uint32_t idx, uint32_t s) {
  return normal_from(philox(idx, s, MK_TAG_PREDICT, 0u, key));
}

__device__ inline double softplus(double x) { return fmax(x, 0.0) + log1p(exp(-fabs(x))); }
// Phi(x) and log Phi(x): erfc for x >= 0 (log1p keeps the digits near 1), the scaled erfcx
// below 0 (no underflow: log Phi(-40) is finite).  oracle/spmvglm.py log_ndtr states the same.
__device__ inline double norm_cdf(double x) { return 0.5 * erfc(-x * MK_SQRT1_2); }
__device__ inline double log_norm_cdf(double x) {
  return (x >= 0.0) ? log1p(-0.5 * erfc(x * MK_SQRT1_2)) : log(0.5 * erfcx(-x * MK_SQRT1_2)) - 0.5 * x * x;
}
// Binomial log-likelihood of y successes in wt trials at linear predictor eta (constants dropped):
// logit  y eta - wt log(1 + e^eta);  probit  y log Phi(eta) + (wt - y) log Phi(-eta).
__device__ inline double loglik_term(double y, double wt, double eta, int link) {
  if (link == MK_LINK_PROBIT) return y * log_norm_cdf(eta) + (wt - y) * log_norm_cdf(-eta);
  return y * eta - wt * softplus(eta);
}

// spBayes util logitInv(z, a, b) = b - (b-a)/(1+exp(z))
__device__ __host__ inline double logit_inv(double z, double a, double b) { return b - (b - a) / (1.0 + exp(z)); }
__device__ inline double unif_jacobian(double v, double a, double b) { return log(v - a) + log(b - v); }

// Deterministic block reduction (fixed tree, wave64 shuffles then LDS).
template <int NT>
__device__ inline double block_sum(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) t += red[w];
    red[NT / 64] = t;
  }
  __syncthreads();
  return red[NT / 64];
}

}  // namespace mk
