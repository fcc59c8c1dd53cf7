"""Soak test of the host-burst fan-out (not part of the pytest suite): one
dispatcher thread, 2-3 contexts on the device, random burst sizes (0..1024),
mbuf and frames submissions, non-blocking hand-offs, idle gaps past the
workers' idle limit (launches leave and are relaunched), and device batches on
a separate context in between.  Bursts come back strictly in submission order;
every burst is checked against the oracle and the per-queue lists, merged in
hand-off order, must equal the oracle's lists over the whole stream.

    python tools/fanout_soak.py --seconds 60
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle import oracle  # noqa: E402  (checker only)
from yastack_amd import FanOut, SoftRss, abi  # noqa: E402

from test_gpu_parity import _fake_mbufs  # noqa: E402
from test_gpu_small_burst import _expect, _frames  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=30.0)
    ap.add_argument("--seed", type=int, default=3)
    args = ap.parse_args()
    os.environ.setdefault("YRSS_WORKER_IDLE_MS", "3")
    os.environ.setdefault("YRSS_WORKER_LIFE_MS", "150")
    import torch

    rng = np.random.default_rng(args.seed)
    cfg = (6, 5, 1, 1)
    npool = 1 << 15
    frames = _frames(oracle, npool, 4321)
    pool, ptrs, _ = _fake_mbufs(frames, headroom=128)
    data = (ptrs + np.uint64(256)).astype(np.uint64)
    flen = np.array([len(f) for f in frames], np.uint16)
    q_all, h_all, _, _ = _expect(oracle, frames, cfg)
    stats = dict(bursts=0, pkts=0, nonblock=0, gaps=0, dev_batches=0, runs=0)
    t_end = time.time() + args.seconds
    with SoftRss(*cfg, device=0, max_burst=0) as dev_eng:
        win_d, lens_d = dev_eng.synth(abi.SYN_TCP4, 1 << 16)
        while time.time() < t_end:
            nctx = int(rng.choice([2, 3]))
            nslots = int(rng.choice([8, 16]))
            stats["runs"] += 1
            with FanOut([0] * nctx, *cfg, nslots=nslots, nblocks=int(rng.choice([2, 4, 8]))) as fo:
                fo.register_host_memory(pool.ctypes.data, pool.nbytes)
                order, pend = [], {}
                stream_q = []          # q of the whole stream, in submission order
                lists = {b: [] for b in range(cfg[1] + 1)}
                base = 0
                t_run = min(t_end, time.time() + 5.0)
                while time.time() < t_run or pend:
                    full = len(pend) >= nctx * nslots
                    if time.time() < t_run and not full and rng.random() < 0.6:
                        n = int(rng.choice([0, 1, 32, 32, 100, 1024, int(rng.integers(1, 1025))]))
                        off = int(rng.integers(0, npool - n))
                        if rng.random() < 0.5:
                            t = fo.submit_frames(data[off:off + n], flen[off:off + n])
                        else:
                            t = fo.submit(ptrs[off:off + n])
                        pend[t] = (off, n)
                        order.append(t)
                        stats["bursts"] += 1
                        stats["pkts"] += n
                        continue
                    if pend and rng.random() < 0.9:
                        got = fo.next(wait=rng.random() < 0.7)
                        if got is None:
                            stats["nonblock"] += 1
                            continue
                        t, r = got
                        assert t == min(pend), (t, min(pend))   # strictly in order
                        off, n = pend.pop(t)
                        q = q_all[off:off + n]
                        qi, qs = oracle.process_burst(q, cfg[1])
                        assert np.array_equal(r.q, q) and np.array_equal(r.hash, h_all[off:off + n])
                        assert np.array_equal(r.qidx, qi) and np.array_equal(r.qstart[:qs.size], qs)
                        for b in range(cfg[1] + 1):
                            lists[b].extend(base + int(x) for x in qi[qs[b]:qs[b + 1]])
                        stream_q.append(q)
                        base += n
                        continue
                    if rng.random() < 0.3:
                        time.sleep(0.006)   # past the idle limit: launches leave
                        stats["gaps"] += 1
                    else:
                        dev_eng.dispatch_dev(win_d, lens_d, 64, 1 << 16)
                        torch.cuda.synchronize()
                        stats["dev_batches"] += 1
                qi_ref, _ = oracle.process_burst(
                    np.concatenate(stream_q) if stream_q else np.zeros(0, np.int16), cfg[1])
                merged = [x for b in range(cfg[1] + 1) for x in lists[b]]
                assert np.array_equal(np.array(merged, np.int64), qi_ref.astype(np.int64))
                fo.unregister_host_memory(pool.ctypes.data)
    print("fanout soak ok", stats, flush=True)


if __name__ == "__main__":
    main()
