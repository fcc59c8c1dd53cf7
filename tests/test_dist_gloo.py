"""World-size-2 gloo run of the multi-GPU path's host logic on CPU.

bench.py shards the packet stream contiguously across ranks, runs every shard
independently (no data-path collective), and reduces only the step time
(max) and packet count (sum).  Here each rank classifies its shard with the
oracle standing in for its GPU, the per-queue lists are gathered and merged
in shard order, and the result must equal the single-process answer.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

N_TOTAL = 40_000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(root))
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import bench
    from oracle import oracle
    from yastack_amd.shard import merge_queue_lists, shard_range

    w, r, _ = bench.dist_setup(world)
    assert (w, r) == (world, rank)
    first, cnt = shard_range(N_TOTAL, world, rank)
    win, lens = oracle.synth(6, cnt, first, stride=80)
    c = oracle.cfg(5, 4, 1, 1)
    qv, hv = oracle.dispatch_windows(win, 80, lens, c)
    qi, qs = oracle.process_burst(qv, 4)
    bench.barrier(world)
    tmax = bench.max_over_ranks(float(rank + 1), world)
    tsum = bench.sum_over_ranks(float(cnt), world)
    gathered = [None] * world
    dist.all_gather_object(gathered, (first, qi.tolist(), qs.tolist(), qv.tolist()))
    if rank == 0:
        merged_qi, merged_qs = merge_queue_lists(
            [(f, np.array(a), np.array(b)) for f, a, b, _ in gathered])
        q_all = np.concatenate([np.array(x[3], np.int16) for x in gathered])
        win_a, lens_a = oracle.synth(6, N_TOTAL, 0, stride=80)
        q_ref, _ = oracle.dispatch_windows(win_a, 80, lens_a, c)
        qi_ref, qs_ref = oracle.process_burst(q_ref, 4)
        q.put(dict(tmax=tmax, tsum=tsum,
                   q_ok=bool(np.array_equal(q_all, q_ref)),
                   qi_ok=bool(np.array_equal(merged_qi, qi_ref.astype(np.int64))),
                   qs_ok=bool(np.array_equal(merged_qs, qs_ref.astype(np.int64)))))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shard_and_merge():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = q.get(timeout=5)
    assert res["tmax"] == 2.0
    assert res["tsum"] == N_TOTAL
    assert res["q_ok"] and res["qi_ok"] and res["qs_ok"]
