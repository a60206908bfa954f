"""R's default RNG and sample() restated in Python (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.

The reference partitions the data with `sample(a, n.part[i], replace=FALSE)` followed by
`a <- setdiff(a, index.part[[i]])` (MK.R:29-41).  R is not installed here, so
this restates R >= 3.6.0's published algorithms for the defaults RNGkind("Mersenne-Twister",
"Inversion", "Rejection"):
  set_seed      -- src/main/RNG.c RNG_Init: 50 LCG scramblings (69069 s + 1), then 625
                   more fill dummy[0..624]; FixupSeeds sets mti = dummy[0] = 624
  unif_rand     -- MT_genrand (Matsumoto-Nishimura MT19937, tempering) * 2^-32, then fixup()
                   into the open interval (0, 1)
  unif_index    -- R_unif_index: rejection sampling over rbits(ceil(log2 n)), 16 bits per
                   unif_rand draw (floor(u * 65536))
  sample_int    -- do_sample, uniform without replacement: x = 0..n-1; j = unif_index(n);
                   pick x[j]; x[j] = x[--n]
  sample_int_replace -- do_sample with replacement: unif_index(n) + 1 per draw (MK.R:141)
  partition     -- MK.R:15-41 verbatim (1-based indices, setdiff keeps a's order)
Pinned by R's published known answers (tests/test_rrng.py): set.seed(1); runif(3) and
set.seed(42|123|1); sample(1:10).  The product implementation is `mk_partition_r` in libmk.
"""
import math

import numpy as np

_N, _M = 624, 397
_MATRIX_A, _UPPER, _LOWER = 0x9908B0DF, 0x80000000, 0x7FFFFFFF
_I2_32M1 = 2.328306437080797e-10      # 1 / (2^32 - 1), RNG.c fixup()


class RRng:
    """RNGkind("Mersenne-Twister", "Inversion", "Rejection") after set.seed(seed)."""

    def __init__(self, seed):
        s = int(seed) & 0xFFFFFFFF
        for _ in range(50):
            s = (69069 * s + 1) & 0xFFFFFFFF
        dummy = []
        for _ in range(_N + 1):
            s = (69069 * s + 1) & 0xFFFFFFFF
            dummy.append(s)
        self.mt = dummy[1:]
        self.mti = _N                    # FixupSeeds(initial): dummy[0] = 624

    def _genrand(self):
        mt = self.mt
        if self.mti >= _N:
            for kk in range(_N):
                y = (mt[kk] & _UPPER) | (mt[(kk + 1) % _N] & _LOWER)
                mt[kk] = mt[(kk + _M) % _N] ^ (y >> 1) ^ (_MATRIX_A if y & 1 else 0)
            self.mti = 0
        y = mt[self.mti]
        self.mti += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y * 2.3283064365386963e-10

    def unif_rand(self):
        v = self._genrand()
        if v <= 0.0:
            return 0.5 * _I2_32M1
        if 1.0 - v <= 0.0:
            return 1.0 - 0.5 * _I2_32M1
        return v

    def _rbits(self, bits):
        v = 0
        for _ in range(0, bits + 1, 16):
            v = 65536 * v + int(math.floor(self.unif_rand() * 65536))
        return v & ((1 << bits) - 1)

    def unif_index(self, dn):
        if dn <= 0:
            return 0
        bits = int(math.ceil(math.log2(dn)))
        while True:
            dv = self._rbits(bits)
            if dn > dv:
                return dv

    def sample_int(self, n, size):
        """sample.int(n, size) without replacement, 1-based (n <= 1e7: no hash path)."""
        if size > n:
            raise ValueError("cannot take a sample larger than the population when 'replace = FALSE'")
        x = list(range(n))
        out = []
        for _ in range(size):
            j = self.unif_index(n)
            out.append(x[j] + 1)
            n -= 1
            x[j] = x[n]
        return out

    def sample_int_replace(self, n, size):
        """sample.int(n, size, replace=TRUE), 1-based: do_sample's R_unif_index(n) + 1 per draw
        (MK.R:141 draws sampleparIndex this way)."""
        return [self.unif_index(n) + 1 for _ in range(size)]

    def runif(self, k):
        return [self.unif_rand() for _ in range(k)]


def partition(n, n_core, seed):
    """MK.R:15-41 after set.seed(seed): (n.part, index.part) with 1-based int64 index arrays."""
    per = n // n_core
    n_part = [per] * (n_core - 1) + [n - per * (n_core - 1)]
    rng = RRng(seed)
    a = np.arange(1, n + 1, dtype=np.int64)
    index_part = []
    for m in n_part:
        if len(a) == 1 and a[0] >= 1:
            # sample(x, size) with one number x >= 1 is sample.int(x, size) (R's quirk)
            idx = np.asarray(rng.sample_int(int(a[0]), m), dtype=np.int64)
        else:
            # sample(a, m): a[sample.int(length(a), m)]
            if m > len(a):
                raise ValueError("cannot take a sample larger than the population when 'replace = FALSE'")
            idx = a[np.asarray(rng.sample_int(len(a), m), dtype=np.int64) - 1]
        index_part.append(idx)
        a = a[~np.isin(a, idx)]            # setdiff(a, idx): a's order, idx removed
    return n_part, index_part
