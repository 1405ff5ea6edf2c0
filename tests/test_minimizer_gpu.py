"""The device minimizer hash at full width.

k_minimizer_hash (kcount_owner.hip) decides KmerDHT::get_kmer_target_rank for the owner hand-off and the
supermer exchange: quick_hash(get_minimizer_fast(m)) (src/kmer.cpp:344-393,454-463; src/kcount/kmer_dht.cpp:
193-196). It is checked through the C ABI (mhmkc_minimizer_hashes) on the SURVEY.md Appendix A keys (the values
the reference's own kmer.cpp gave) and on 10^5 random canonical keys per k against the oracle's
orc_minimizer_hash_fast, all 64 bits.
"""
import numpy as np
import pytest

import mhm2_proxy_amd as m
import oracle_lib as O
from test_oracle import APPENDIX_A

pytestmark = pytest.mark.gpu


def random_canonical_keys(n: int, k: int, nl: int, seed: int) -> np.ndarray:
    """(n, nl) Kmer<MAX_K>::longs of uniform random canonical k-mers (2-bit MSB-first, zero below base k)."""
    rng = np.random.default_rng(seed)
    codes = rng.integers(0, 4, size=(n, k), dtype=np.uint8)
    rc = 3 - codes[:, ::-1]
    diff = codes != rc
    first = np.argmax(diff, axis=1)  # odd k: never a palindrome, so some position differs
    take_rc = rc[np.arange(n), first] < codes[np.arange(n), first]
    canon = np.where(take_rc[:, None], rc, codes).astype(np.uint64)
    keys = np.zeros((n, nl), dtype=np.uint64)
    for i in range(k):
        keys[:, i // 32] |= canon[:, i] << np.uint64(2 * (31 - i % 32))
    return keys


@pytest.mark.parametrize("kmer,nl,longs,h,mini,mhash", APPENDIX_A)
def test_minimizer_hash_appendix_a(kmer, nl, longs, h, mini, mhash):
    k = len(kmer)
    with m.KmerCounter(k, n_longs=nl, device=0) as c:
        got = c.minimizer_hashes(np.array([longs], dtype=np.uint64))
        assert int(got[0]) == mhash, f"{kmer}: {int(got[0]):016x} != {mhash:016x}"
        assert int(c.target_ranks(np.array([longs], dtype=np.uint64), 7)[0]) == mhash % 7


@pytest.mark.parametrize("k", [21, 33, 55, 63, 77, 99, 127])
def test_minimizer_hash_random_keys_full_width(k):
    nl = k // 32 + 1
    n = 100_000
    keys = random_canonical_keys(n, k, nl, seed=k)
    mlen = O.oracle().orc_minimizer_len(k)
    with m.KmerCounter(k, device=0) as c:
        got = c.minimizer_hashes(keys)
    L = O.oracle()
    exp = np.fromiter((L.orc_minimizer_hash_fast(keys[i].ctypes.data, k, nl, mlen) for i in range(n)),
                      dtype=np.uint64, count=n)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"k={k}: {bad.size} of {n} differ, first row {bad[:1]}"


def test_minimizer_hash_explicit_m_and_wide_longs():
    """An explicit m (1..min(k, 28)) and keys given with more longs than k needs (a larger MAX_K)."""
    k = 45
    keys = random_canonical_keys(20_000, k, 2, seed=5)
    wide = np.zeros((keys.shape[0], 3), dtype=np.uint64)
    wide[:, :2] = keys
    L = O.oracle()
    with m.KmerCounter(k, n_longs=3, device=0) as c:
        for mm in (1, 11, 19, 28):
            got = c.minimizer_hashes(wide, m=mm)
            exp = np.fromiter((L.orc_minimizer_hash_fast(wide[i].ctypes.data, k, 3, mm) for i in range(len(wide))),
                              dtype=np.uint64, count=len(wide))
            assert (got == exp).all(), f"m={mm}"
