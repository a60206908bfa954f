"""R's RNG stream and the reference's partition loop (MK.R:15-41).

oracle/rrng.py is pinned by R's published known answers (R >= 3.6.0 defaults); libmk's host
implementation (mk_partition_r / mk_r_sample, no GPU work) is checked against it exactly.
"""
import time

import numpy as np
import pytest

from oracle import rrng


# R >= 3.6.0 console output (RNGkind defaults), 7 significant digits as R prints them
KNOWN_RUNIF = {1: [0.2655087, 0.3721239, 0.5728534], 123: [0.2875775, 0.7883051, 0.4089769], 42: [0.914806]}
KNOWN_SAMPLE = {(42, 10, 10): [1, 5, 10, 8, 2, 4, 6, 9, 7, 3],
                (123, 10, 10): [3, 10, 2, 8, 6, 9, 1, 7, 5, 4],
                (1, 10, 10): [9, 4, 7, 1, 2, 5, 3, 10, 6, 8],
                (42, 100, 5): [49, 65, 25, 74, 18],
                (123, 100, 5): [31, 79, 51, 14, 67]}


@pytest.mark.parametrize("seed", sorted(KNOWN_RUNIF))
def test_oracle_runif_known_answers(seed):
    got = rrng.RRng(seed).runif(len(KNOWN_RUNIF[seed]))
    np.testing.assert_allclose(got, KNOWN_RUNIF[seed], atol=5e-7, rtol=0)


@pytest.mark.parametrize("key", sorted(KNOWN_SAMPLE))
def test_oracle_sample_known_answers(key):
    seed, n, size = key
    assert rrng.RRng(seed).sample_int(n, size) == KNOWN_SAMPLE[key]


@pytest.mark.parametrize("key", sorted(KNOWN_SAMPLE))
def test_lib_sample_known_answers(mk, key):
    seed, n, size = key
    lib = mk._lib.load()
    out = np.zeros(size, dtype=np.int32)
    mk._lib.check(lib.mk_r_sample(seed, n, size, mk._lib.iptr(out)))
    assert out.tolist() == KNOWN_SAMPLE[key]


def test_lib_sample_large_population_matches_oracle(mk):
    # n > 2^16: two unif_rand draws per rbits (the bits > 16 path), plus rejections
    lib = mk._lib.load()
    out = np.zeros(300, dtype=np.int32)
    mk._lib.check(lib.mk_r_sample(20250114, 500_000, 300, mk._lib.iptr(out)))
    assert out.tolist() == rrng.RRng(20250114).sample_int(500_000, 300)


@pytest.mark.parametrize("n,k,seed", [(2000, 5, 20250114), (103, 7, 3), (7, 3, 11), (3, 5, 2), (5, 5, 9),
                                      (1, 1, 4), (12001, 6, -77)])
def test_partition_matches_oracle(mk, n, k, seed):
    n_part, idx = mk.metakriging.partition(n, k, seed=seed, method="R")
    o_part, o_idx = rrng.partition(n, k, seed)
    assert n_part.tolist() == o_part
    for a, b in zip(idx, o_idx):
        assert (a + 1).tolist() == b.tolist()


def test_partition_covers_and_is_disjoint(mk):
    n, k = 20_000, 9
    n_part, idx = mk.metakriging.partition(n, k, seed=5, method="R")
    assert n_part.tolist() == [2222] * 8 + [2224]                 # MK.R:17-18
    allidx = np.concatenate(idx)
    assert np.array_equal(np.sort(allidx), np.arange(n))


def test_partition_cfg3_is_fast(mk):
    t = time.perf_counter()
    n_part, idx = mk.metakriging.partition(500_000, 250, seed=20250114, method="R")
    assert time.perf_counter() - t < 5.0
    assert len(idx) == 250 and all(len(i) == 2000 for i in idx)
    assert np.array_equal(np.sort(np.concatenate(idx)), np.arange(500_000))
    # first subset: R draws it straight from 1:n, so it is sample.int(n, 2000)
    assert (idx[0] + 1).tolist() == rrng.RRng(20250114).sample_int(500_000, 2000)


def test_partition_errors(mk):
    with pytest.raises(mk.MkError):
        mk.metakriging.partition(0, 3, seed=1, method="R")
    with pytest.raises(ValueError):
        mk.metakriging.partition(10, 3, seed=1, method="bogus")


# sample(1:n, size, replace = TRUE) after set.seed(seed), R >= 3.6.0 console output
KNOWN_SAMPLE_REPLACE = {(123, 6, 10): [3, 6, 3, 2, 2, 6, 3, 5, 4, 6],
                        (42, 10, 5): [1, 5, 1, 9, 10]}


@pytest.mark.parametrize("key", sorted(KNOWN_SAMPLE_REPLACE))
def test_oracle_sample_replace_known_answers(key):
    seed, n, size = key
    assert rrng.RRng(seed).sample_int_replace(n, size) == KNOWN_SAMPLE_REPLACE[key]


@pytest.mark.parametrize("key", sorted(KNOWN_SAMPLE_REPLACE) + [(20250114, 996, 1000), (7, 70000, 50)])
def test_lib_sample_replace_matches_oracle(mk, key):
    """mk_r_sample_replace: MK.R:141's sampleparIndex (sample(seq(1, 996, 1), 1000, replace=TRUE))
    as R draws it right after set.seed(seed); n > 2^16 takes the two-draw rbits path."""
    seed, n, size = key
    lib = mk._lib.load()
    out = np.zeros(size, dtype=np.int32)
    mk._lib.check(lib.mk_r_sample_replace(seed, n, size, mk._lib.iptr(out)))
    assert out.tolist() == rrng.RRng(seed).sample_int_replace(n, size)
    if key in KNOWN_SAMPLE_REPLACE:
        assert out.tolist() == KNOWN_SAMPLE_REPLACE[key]
