"""world_size-2 gloo rehearsal of the multi-GPU hash-range exchange (CPU).

The union of the owners' tables must equal the single-rank table of all reads, and the owners' key
sets must be disjoint (each k-mer finalized by exactly one rank, like the reference's owner rank).
"""
import socket

import numpy as np
import pytest

import mhm2_proxy_amd as m
from common import assert_tables_equal, oracle_table, synth_set


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("k,world", [(21, 2), (63, 2), (33, 3)])
def test_hash_range_exchange_equals_single_rank(k, world, tmp_path):
    import torch.multiprocessing as mp

    import mr_worker

    mp.spawn(mr_worker.run, args=(world, free_port(), k, str(tmp_path)), nprocs=world, join=True)
    parts = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    keys = np.concatenate([p["keys"] for p in parts])
    union = m.KmerTable(k, keys, np.concatenate([p["counts"] for p in parts]),
                        np.concatenate([p["left"] for p in parts]), np.concatenate([p["right"] for p in parts]))
    assert sum(int(p["n_recv"]) for p in parts) == sum(int(p["n_sent"]) for p in parts)
    assert len({tuple(r) for r in keys.tolist()}) == len(keys), "owners' key sets overlap"
    b, o = synth_set(1200, 9000, 600 + k)
    assert_tables_equal(union, oracle_table(b, o, k), f"union of {world} owners")
