"""Multi-GPU sharding of a packet batch.

The soft-RSS result of a packet depends only on its own bytes, the key and the
config, so a batch splits into contiguous shards, one per GPU/rank, with no
collective on the data path.  The reference's per-queue ``rte_ring`` is FIFO
(fs/lib/ff_dpdk_if.c:1087-1093), so the global per-queue lists are the
per-shard lists concatenated in shard order — that is the only host-side
step, and it is what :func:`merge_queue_lists` does.
"""
from __future__ import annotations

import numpy as np


def shard_range(n_total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [first, first+count) slice of n_total for rank (balanced)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(n_total, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def merge_queue_lists(parts):
    """Concatenate per-shard bucket lists in shard order.

    ``parts``: iterable of (first, qidx, qstart) per shard, in shard order, with
    qidx holding shard-local indices.  Returns (qidx, qstart) over global
    indices, bucket b = qidx[qstart[b]:qstart[b+1]].
    """
    parts = list(parts)
    if not parts:
        raise ValueError("no shards")
    nbk = len(parts[0][2]) - 1
    counts = np.zeros(nbk, dtype=np.int64)
    for _, _, qs in parts:
        qs = np.asarray(qs, dtype=np.int64)
        if len(qs) != nbk + 1:
            raise ValueError("shards disagree on bucket count")
        counts += np.diff(qs)
    qstart = np.zeros(nbk + 1, dtype=np.int64)
    qstart[1:] = np.cumsum(counts)
    out = np.empty(int(qstart[-1]), dtype=np.int64)
    fill = qstart[:-1].copy()
    for first, qi, qs in parts:
        qi = np.asarray(qi, dtype=np.int64)
        qs = np.asarray(qs, dtype=np.int64)
        for b in range(nbk):
            seg = qi[qs[b]:qs[b + 1]]
            out[fill[b]:fill[b] + len(seg)] = seg + first
            fill[b] += len(seg)
    return out, qstart
