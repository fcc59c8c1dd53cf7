"""Soak test of the host-resident burst paths (not part of the pytest suite):
random sizes on both sides of the one-launch threshold (1..9000 packets),
yrss_dispatch_burst / _burst_zc / _frames / _frames_zc, synchronous and
YRSS_F_ASYNC over two contexts with waits in random order, optional outputs
left out, and the hash.rss write-back.  Every burst is checked against the
oracle.

    python tools/burst_soak.py --seconds 60
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle import oracle  # noqa: E402  (checker only)
from yastack_amd import SoftRss, abi  # noqa: E402

from test_gpu_parity import _fake_mbufs  # noqa: E402
from test_gpu_small_burst import _expect, _frames  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=30.0)
    ap.add_argument("--seed", type=int, default=2)
    args = ap.parse_args()
    rng = np.random.default_rng(args.seed)
    cfg = (5, 4, 1, 1)
    npool = 1 << 15
    frames = _frames(oracle, npool, 4321)
    pool, ptrs, stride = _fake_mbufs(frames, headroom=128)
    data = (ptrs + np.uint64(256)).astype(np.uint64)
    flen = np.array([len(f) for f in frames], np.uint16)
    q_all, h_all, _, _ = _expect(oracle, frames, cfg)
    lib = abi.load()
    stats = dict(bursts=0, pkts=0, small=0, big=0, asyncs=0, writeback=0)
    engs = [SoftRss(*cfg, device=0, max_burst=0) for _ in range(2)]
    try:
        for e in engs:
            e.register_host_memory(pool.ctypes.data, pool.nbytes)
        pend = [None, None]   # per context: (off, n, outputs, writeback)
        t_end = time.time() + args.seconds
        while time.time() < t_end or any(pend):
            k = int(rng.integers(0, 2))
            if pend[k] is not None:
                assert lib.yrss_wait(engs[k]._ctx) == 0
                check(pend[k], q_all, h_all, cfg, pool, stride)
                pend[k] = None
                continue
            if time.time() >= t_end:
                continue
            n = int(rng.choice([1, 32, 1024, 4095, 4096, 4097, int(rng.integers(1, 9001))]))
            half = npool // 2   # each context owns half the pool (write-back checks)
            off = k * half + int(rng.integers(0, half - n))
            m = max(n, 1)
            q = np.zeros(m, np.int16)
            h = np.zeros(m, np.uint32) if rng.random() < 0.8 else None
            compact = rng.random() < 0.8
            qi = np.zeros(m, np.uint32) if compact else None
            qs = np.zeros(cfg[1] + 2, np.uint32) if compact else None
            api = int(rng.integers(0, 4))
            asy = rng.random() < 0.5
            wb = api in (0, 1) and rng.random() < 0.2
            flags = (abi.F_ASYNC if asy else 0) | (abi.F_WRITE_RSS if wb else 0)
            ptr = lambda a: None if a is None else a.ctypes.data  # noqa: E731
            mb = np.ascontiguousarray(ptrs[off:off + n])
            dp = np.ascontiguousarray(data[off:off + n])
            ln = np.ascontiguousarray(flen[off:off + n])
            if wb:   # the write-back must be seen fresh
                pool.reshape(-1, stride)[off:off + n, 44:48] = 0
            c = engs[k]._ctx
            if api == 0:
                rc = lib.yrss_dispatch_burst(c, mb.ctypes.data, n, q.ctypes.data, ptr(h), ptr(qi),
                                             ptr(qs), flags)
            elif api == 1:
                rc = lib.yrss_dispatch_burst_zc(c, mb.ctypes.data, n, q.ctypes.data, ptr(h),
                                                ptr(qi), ptr(qs), flags)
            elif api == 2:
                asy = False   # yrss_dispatch_frames is synchronous
                bufs = [frames[i] for i in range(off, off + n)]
                arrs = [np.frombuffer(b, np.uint8) for b in bufs]
                dps = np.array([a.ctypes.data for a in arrs], np.uint64)
                rc = lib.yrss_dispatch_frames(c, dps.ctypes.data, ln.ctypes.data, n,
                                              q.ctypes.data, ptr(h), ptr(qi), ptr(qs))
            else:
                rc = lib.yrss_dispatch_frames_zc_ex(c, dp.ctypes.data, ln.ctypes.data, n,
                                                    q.ctypes.data, ptr(h), ptr(qi), ptr(qs),
                                                    abi.F_ASYNC if asy else 0)
            assert rc == 0, (api, n, rc)
            item = (off, n, (q, h, qi, qs), wb, (mb, dp, ln))
            stats["bursts"] += 1
            stats["pkts"] += n
            stats["small" if n <= 4096 else "big"] += 1
            stats["writeback"] += wb
            if asy:
                stats["asyncs"] += 1
                pend[k] = item
            else:
                check(item, q_all, h_all, cfg, pool, stride)
        for e in engs:
            e.unregister_host_memory(pool.ctypes.data)
    finally:
        for e in engs:
            e.close()
    print("soak ok", stats, flush=True)


def check(item, q_all, h_all, cfg, pool, stride):
    off, n, (q, h, qi, qs), wb, _ = item
    qr = q_all[off:off + n]
    assert np.array_equal(q[:n], qr), (off, n)
    if h is not None:
        assert np.array_equal(h[:n], h_all[off:off + n]), (off, n)
    if qi is not None:
        qi_ref, qs_ref = oracle.process_burst(qr, cfg[1])
        assert np.array_equal(qi[:n], qi_ref), (off, n)
        assert np.array_equal(qs[: qs_ref.size], qs_ref), (off, n)
    if wb:
        rss = pool.reshape(-1, stride)[off:off + n, 44:48].copy().view(np.uint32).ravel()
        assert np.array_equal(rss, h_all[off:off + n]), (off, n)


if __name__ == "__main__":
    main()
