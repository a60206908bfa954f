"""Philox4x32-10 counter-based RNG, NumPy restatement (TEST INFRASTRUCTURE ONLY).

The reference draws every random number from R's Mersenne-Twister through
spBayes' ``rnorm``/``runif`` calls (MetaKriging_BinaryResponse.R:80-87 call
into spBayes; MK.R:31 and MK.R:141 call ``sample``).  R is absent from this
build, so identical-draw parity is only possible between this oracle and the
HIP library: both derive every draw from the same
(key, counter) pairs through Philox4x32-10 (Salmon et al., SC'11, the
Random123 algorithm).  This file is the bit-exact host restatement of
``csrc/philox.hpp``; it is pinned by the Random123 known-answer vectors in
tests/test_oracle_philox.py.

Stream layout (shared with the device):
  key  = (lo32(seed), hi32(seed) + subset)                 -- one stream per subset
  ctr  = (c0, c1, c2, c3) = (index, iteration, tag, word)  -- one call per draw
  TAG_PROPOSAL : c0 = MH parameter index j, c1 = iteration s
                 word 0 -> N(0,1) proposal (Box-Muller), word 1 -> U(0,1) accept draw
  TAG_PREDICT  : c0 = test-site*q + outcome, c1 = iteration s, word 0 -> N(0,1)
  TAG_RESAMPLE : c0 = draw index, c1 = 0 -> resample index (post-processing)
"""
import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)

TAG_PROPOSAL = 1
TAG_PREDICT = 2
TAG_RESAMPLE = 3

TWO_PI = 6.283185307179586          # nearest double to 2*pi (device uses the same literal)
TWO_M52 = 2.0 ** -52


def philox4x32_10(ctr, key):
    """ctr: (..., 4) uint32 array; key: (..., 2) uint32 (broadcastable). Returns (..., 4) uint32."""
    ctr = np.asarray(ctr, dtype=np.uint32)
    key = np.asarray(key, dtype=np.uint32)
    c0 = ctr[..., 0].astype(np.uint64)
    c1 = ctr[..., 1].astype(np.uint32)
    c2 = ctr[..., 2].astype(np.uint64)
    c3 = ctr[..., 3].astype(np.uint32)
    k0 = np.broadcast_to(key[..., 0], c1.shape).astype(np.uint32)
    k1 = np.broadcast_to(key[..., 1], c1.shape).astype(np.uint32)
    with np.errstate(over="ignore"):
        for r in range(10):
            if r > 0:
                k0 = (k0 + W0).astype(np.uint32)
                k1 = (k1 + W1).astype(np.uint32)
            p0 = M0 * c0
            p1 = M1 * c2
            hi0 = (p0 >> np.uint64(32)).astype(np.uint32)
            lo0 = (p0 & MASK32).astype(np.uint32)
            hi1 = (p1 >> np.uint64(32)).astype(np.uint32)
            lo1 = (p1 & MASK32).astype(np.uint32)
            n0 = hi1 ^ c1 ^ k0
            n1 = lo1
            n2 = hi0 ^ c3 ^ k1
            n3 = lo0
            c0 = n0.astype(np.uint64)
            c1 = n1
            c2 = n2.astype(np.uint64)
            c3 = n3
    return np.stack([c0.astype(np.uint32), c1, c2.astype(np.uint32), c3], axis=-1)


def make_key(seed, subset):
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    return np.array([seed & 0xFFFFFFFF, ((seed >> 32) + int(subset)) & 0xFFFFFFFF], dtype=np.uint32)


def u01_open(hi, lo):
    """Two 32-bit words -> double in (0,1): (top52 + 0.5) * 2^-52 (exact in fp64)."""
    hi = np.asarray(hi, dtype=np.uint64)
    lo = np.asarray(lo, dtype=np.uint64)
    top52 = ((hi << np.uint64(32)) | lo) >> np.uint64(12)
    return (top52.astype(np.float64) + 0.5) * TWO_M52


def normal_from_words(w):
    """Box-Muller on one Philox output block: u1 from (w0,w1), u2 from (w2,w3)."""
    u1 = u01_open(w[..., 0], w[..., 1])
    u2 = u01_open(w[..., 2], w[..., 3])
    return np.sqrt(-2.0 * np.log(u1)) * np.cos(TWO_PI * u2)


def _ctr(c0, c1, tag, word):
    c0 = np.asarray(c0, dtype=np.int64)
    c1 = np.broadcast_to(np.asarray(c1, dtype=np.int64), c0.shape)
    out = np.empty(c0.shape + (4,), dtype=np.uint32)
    out[..., 0] = (c0 & 0xFFFFFFFF).astype(np.uint32)
    out[..., 1] = (c1 & 0xFFFFFFFF).astype(np.uint32)
    out[..., 2] = np.uint32(tag)
    out[..., 3] = np.uint32(word)
    return out


def proposal_normal(key, j, s):
    """N(0,1) used for the random-walk proposal of MH parameter(s) j at iteration s."""
    return normal_from_words(philox4x32_10(_ctr(j, s, TAG_PROPOSAL, 0), key))


def accept_log_uniform(key, j, s):
    """log(U), U~U(0,1), the accept draw of MH parameter(s) j at iteration s."""
    w = philox4x32_10(_ctr(j, s, TAG_PROPOSAL, 1), key)
    return np.log(u01_open(w[..., 0], w[..., 1]))


def predict_normal(key, idx, s):
    """N(0,1) for the kriging draw of (test-site*q + outcome) idx at iteration s."""
    return normal_from_words(philox4x32_10(_ctr(idx, s, TAG_PREDICT, 0), key))


def resample_uniform(key, idx):
    w = philox4x32_10(_ctr(idx, 0, TAG_RESAMPLE, 0), key)
    return u01_open(w[..., 0], w[..., 1])
