"""Worker of the world_size-2 gloo tests (TEST INFRASTRUCTURE): the hash-range exchange protocol of
libmhmkc's multi-GPU path (mhmkc_host.cpp exchange()), restated over the CPU oracle.

Each rank extracts (canonical key, ext code) records from its own shard of reads, sends every record to
the owner of its coarse bucket (coarse = Kmer::hash() >> (64 - CB), CB = 8 + ceil(log2 G), owner ranges
[ceil(r*2^CB/G), ceil((r+1)*2^CB/G))) with one all_to_all, and counts what it owns.
"""
import bisect
import os
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
sys.path.insert(0, str(HERE.parent))


def coarse_bits(world: int) -> int:
    extra = 0
    while (1 << extra) < world:
        extra += 1
    return 8 + extra


def owner_of(coarse: np.ndarray, world: int) -> np.ndarray:
    nb = 1 << coarse_bits(world)
    lo = [(r * nb + world - 1) // world for r in range(world + 1)]
    return np.array([bisect.bisect_right(lo, int(c)) - 1 for c in coarse], dtype=np.int64)


def run(rank: int, world: int, port: int, k: int, out_dir: str):
    import torch
    import torch.distributed as dist

    import oracle_lib as O
    from common import synth_set

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b, o = synth_set(1200, 9000, 600 + k)
    n = o.size - 1
    lo, hi = n * rank // world, n * (rank + 1) // world
    mb, mo = b[int(o[lo]):int(o[hi])], (o[lo:hi + 1] - o[lo]).astype(np.uint64)
    nl = k // 32 + 1
    keys, exts = O.extract(mb, mo, k)
    h = np.empty(len(keys), dtype=np.uint64)
    O.oracle().orc_kmer_hash_many.argtypes = [O.C.c_void_p, O.C.c_uint64, O.C.c_int, O.C.c_void_p]
    O.oracle().orc_kmer_hash_many(np.ascontiguousarray(keys).ctypes.data, len(keys), nl, h.ctypes.data)
    coarse = h >> np.uint64(64 - coarse_bits(world))
    owner = owner_of(coarse, world)
    order = np.argsort(owner, kind="stable")
    send_keys, send_ext = keys[order], exts[order]
    send_counts = np.bincount(owner, minlength=world).astype(np.int64)
    recv_counts = torch.empty(world, dtype=torch.int64)
    dist.all_to_all_single(recv_counts, torch.from_numpy(send_counts))
    rc = recv_counts.numpy()
    rk = torch.empty((int(rc.sum()), nl), dtype=torch.int64)
    dist.all_to_all_single(rk, torch.from_numpy(send_keys.view(np.int64)), rc.tolist(), send_counts.tolist())
    re_ = torch.empty(int(rc.sum()), dtype=torch.uint8)
    dist.all_to_all_single(re_, torch.from_numpy(send_ext), rc.tolist(), send_counts.tolist())
    t = O.count_records(rk.numpy().view(np.uint64), re_.numpy(), k)
    tk, tc, tl, tr = t.fetch()
    np.savez(Path(out_dir) / f"rank{rank}.npz", keys=tk, counts=tc, left=tl, right=tr, n_recv=rc.sum(),
             n_sent=len(keys))
    dist.barrier()
    dist.destroy_process_group()
