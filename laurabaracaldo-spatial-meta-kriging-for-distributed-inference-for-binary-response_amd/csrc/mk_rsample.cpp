// R's default RNG stream and the reference's partition loop (MK.R:15-41), host side.
//
// The reference draws its subsets with `sample(a, n.part[i], replace=FALSE)` and then
// `a <- setdiff(a, index.part[[i]])` (MK.R:29-41).  Given the seed of a preceding
// `set.seed(seed)`, mk_partition_r returns the index sets R would, so a run driven from
// Python (or from C) can fit exactly the subsets an R session fits.  R >= 3.6.0 defaults:
// RNGkind("Mersenne-Twister", "Inversion", "Rejection").
//   set.seed      RNG.c RNG_Init: 50 LCG scramblings s = 69069 s + 1, then 625 more fill
//                 dummy[0..624] (dummy[0] is mti), FixupSeeds sets mti = 624
//   unif_rand     MT19937 word * 2^-32, fixup() into the open interval (0, 1)
//   unif_index    R_unif_index: rejection over rbits(ceil(log2 n)), 16 bits per draw
//   sample        do_sample, uniform without replacement: x = 0..n-1, j = unif_index(n),
//                 take x[j], x[j] = x[--n]; with replacement: unif_index(n) + 1 per draw
// The partition is a sequential RNG stream, so it stays on the host: per subset O(|a|)
// (the selection plus an order-keeping compaction for setdiff), 1.25e8 simple steps at
// n = 500k, K = 250.
#include <cmath>
#include <cstdint>
#include <vector>
#include "../../include/mk.h"

namespace mk {
int host_error(int code, const char* msg);   // mk_api.hip: sets mk_last_error()
}

namespace {

class RRng {
 public:
  explicit RRng(int32_t seed) {
    uint32_t s = (uint32_t)seed;
    for (int j = 0; j < 50; ++j) s = 69069u * s + 1u;
    s = 69069u * s + 1u;   // dummy[0] (mti slot, overwritten by FixupSeeds)
    for (int j = 0; j < N; ++j) {
      s = 69069u * s + 1u;
      mt_[j] = s;
    }
    mti_ = N;
  }

  double unif_rand() {
    const double v = genrand();
    constexpr double i2_32m1 = 2.328306437080797e-10;   // RNG.c fixup()
    if (v <= 0.0) return 0.5 * i2_32m1;
    if (1.0 - v <= 0.0) return 1.0 - 0.5 * i2_32m1;
    return v;
  }

  // R_unif_index(dn), Rejection kind
  int64_t unif_index(int64_t n) {
    if (n <= 0) return 0;
    const int bits = (int)std::ceil(std::log2((double)n));
    for (;;) {
      int64_t v = 0;
      for (int b = 0; b <= bits; b += 16) v = 65536 * v + (int64_t)std::floor(unif_rand() * 65536);
      v &= ((int64_t)1 << bits) - 1;
      if (n > v) return v;
    }
  }

 private:
  static constexpr int N = 624, M = 397;
  uint32_t mt_[N];
  int mti_;

  double genrand() {
    constexpr uint32_t mag01[2] = {0x0u, 0x9908B0DFu};
    constexpr uint32_t upper = 0x80000000u, lower = 0x7FFFFFFFu;
    if (mti_ >= N) {
      int kk;
      uint32_t y;
      for (kk = 0; kk < N - M; ++kk) {
        y = (mt_[kk] & upper) | (mt_[kk + 1] & lower);
        mt_[kk] = mt_[kk + M] ^ (y >> 1) ^ mag01[y & 1];
      }
      for (; kk < N - 1; ++kk) {
        y = (mt_[kk] & upper) | (mt_[kk + 1] & lower);
        mt_[kk] = mt_[kk + (M - N)] ^ (y >> 1) ^ mag01[y & 1];
      }
      y = (mt_[N - 1] & upper) | (mt_[0] & lower);
      mt_[N - 1] = mt_[M - 1] ^ (y >> 1) ^ mag01[y & 1];
      mti_ = 0;
    }
    uint32_t y = mt_[mti_++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9D2C5680u;
    y ^= (y << 15) & 0xEFC60000u;
    y ^= y >> 18;
    return (double)y * 2.3283064365386963e-10;
  }
};

int rs_fail(const char* msg) { return mk::host_error(MK_E_ARG, msg); }

// sample.int(n, size) without replacement into out (1-based); x is scratch of >= n.
void sample_noreplace(RRng& rng, int64_t n, int64_t size, std::vector<int32_t>& x, int32_t* out) {
  for (int64_t i = 0; i < n; ++i) x[i] = (int32_t)i;
  for (int64_t i = 0; i < size; ++i) {
    const int64_t j = rng.unif_index(n);
    out[i] = x[j] + 1;
    x[j] = x[--n];
  }
}

}  // namespace

extern "C" int mk_r_sample(int32_t seed, int32_t n, int32_t size, int32_t* out) {
  if (n < 0 || size < 0 || (size > 0 && !out)) return rs_fail("invalid arguments");
  if (size > n) return rs_fail("cannot take a sample larger than the population when 'replace = FALSE'");
  RRng rng(seed);
  std::vector<int32_t> x((size_t)n);
  sample_noreplace(rng, n, size, x, out);
  return MK_OK;
}

// sample(x, size, replace = TRUE) with length(x) = n > 1 (MK.R:141: sample(seq(1, length(Xout), 1),
// samplesize, replace=TRUE)): do_sample's with-replacement branch, iy[i] = R_unif_index(n) + 1.
extern "C" int mk_r_sample_replace(int32_t seed, int32_t n, int32_t size, int32_t* out) {
  if (n < 1 || size < 0 || (size > 0 && !out)) return rs_fail("invalid arguments");
  RRng rng(seed);
  for (int32_t i = 0; i < size; ++i) out[i] = (int32_t)(rng.unif_index(n) + 1);
  return MK_OK;
}

extern "C" int mk_partition_r(int32_t n, int32_t n_core, int32_t seed, int32_t* n_part, int32_t* index_out) {
  if (n < 1 || n_core < 1 || !n_part || !index_out) return rs_fail("invalid arguments");
  const int32_t per = n / n_core;   // floor(n.sample / n.core), MK.R:17
  for (int32_t i = 0; i < n_core; ++i) n_part[i] = (i < n_core - 1) ? per : n - per * (n_core - 1);   // MK.R:18
  RRng rng(seed);
  std::vector<int32_t> a((size_t)n), x((size_t)n), pick;
  std::vector<uint8_t> taken((size_t)n + 1, 0);
  for (int32_t v = 0; v < n; ++v) a[v] = v + 1;   // a <- 1:n.sample (MK.R:20)
  int64_t len = n, off = 0;
  for (int32_t i = 0; i < n_core; ++i) {
    const int64_t m = n_part[i];
    int32_t* idx = index_out + off;
    if (len == 1 && a[0] >= 1) {
      // sample(x, size) with length(x) == 1 and x >= 1 means sample.int(x, size): R's quirk
      const int64_t pop = a[0];
      if (m > pop) return rs_fail("cannot take a sample larger than the population when 'replace = FALSE'");
      if ((int64_t)x.size() < pop) x.resize((size_t)pop);
      sample_noreplace(rng, pop, m, x, idx);
    } else {
      if (m > len) return rs_fail("cannot take a sample larger than the population when 'replace = FALSE'");
      pick.resize((size_t)m);
      sample_noreplace(rng, len, m, x, pick.data());
      for (int64_t t = 0; t < m; ++t) idx[t] = a[pick[t] - 1];   // a[sample.int(length(a), m)]
    }
    // a <- setdiff(a, index.part[[i]]): keep a's order, drop the drawn values
    for (int64_t t = 0; t < m; ++t)
      if (idx[t] >= 1 && idx[t] <= n) taken[idx[t]] = 1;
    int64_t w = 0;
    for (int64_t t = 0; t < len; ++t)
      if (!taken[a[t]]) a[w++] = a[t];
    len = w;
    off += m;
  }
  return MK_OK;
}
