"""The order-independent table digest used by the large multi-rank tests (common.table_digest)."""
import numpy as np

import mhm2_proxy_amd as m
from common import assert_digests_equal, merge_digests, oracle_table, synth_set, table_digest


def test_digest_is_order_independent_and_sensitive():
    b, o = synth_set(3000, 20000, 77)
    t = oracle_table(b, o, 21)
    perm = np.random.default_rng(1).permutation(len(t))
    p = m.KmerTable(21, t.keys[perm], t.counts[perm], t.left[perm], t.right[perm])
    d = table_digest(t, sample_bits=3)
    assert d["keys"].shape[0] > 0
    half = len(t) // 2
    parts = [m.KmerTable(21, p.keys[s], p.counts[s], p.left[s], p.right[s]) for s in (slice(0, half), slice(half, None))]
    assert_digests_equal(merge_digests([table_digest(x, sample_bits=3) for x in parts]), d, 21, "split + permuted")
    c = t.counts.copy()
    c[len(t) // 3] += 1
    bad = table_digest(m.KmerTable(21, t.keys, c, t.left, t.right), sample_bits=3)
    assert (bad["s1"], bad["s2"]) != (d["s1"], d["s2"])
