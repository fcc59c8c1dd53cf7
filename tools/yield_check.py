#!/usr/bin/env python3
"""Latency of a 2^24-packet device batch on context B while context A's
persistent worker (128 workgroups, idle exit 3 s) is resident, and the
latency of A's next burst.  --filter runs B's batch through the KNI-filter
parse kernel (the largest LDS footprint).  The commit that built a device-wide
yield read YRSS_NO_YIELD for its A/B (profiles/r02_v4_worker_yield_ab.log)."""
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."),
                os.path.join(os.path.dirname(__file__), "..", "tests")]
os.environ.setdefault("YRSS_WORKER_IDLE_MS", "3000")
os.environ.setdefault("YRSS_WORKER_LIFE_MS", "6000")
import torch  # noqa: E402

from oracle import oracle  # noqa: E402
from test_gpu_parity import _fake_mbufs  # noqa: E402
from test_gpu_small_burst import _frames  # noqa: E402
from yastack_amd import SoftRss, abi  # noqa: E402

n = 1 << 24
frames = _frames(oracle, 256, 3)
pool, ptrs, _ = _fake_mbufs(frames)
filt = "--filter" in sys.argv
with SoftRss(3, 3, 1, 1, device=0, max_burst=0) as b, SoftRss(3, 3, 1, 1, device=0, max_burst=0) as a:
    win, lens = b.synth(abi.SYN_UDP4, n)
    if filt:
        b.set_kni(True, "reject", "80,443", "53")
    b.dispatch_dev(win, lens, 64, n, want_filter=filt)

    def batch():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        b.dispatch_dev(win, lens, 64, n, want_filter=filt)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3

    solo = min(batch() for _ in range(5))
    a.register_host_memory(pool.ctypes.data, pool.nbytes)
    a.worker_start(512, 128)
    a.worker_poll(a.worker_submit(ptrs[:128]))
    shared = batch()
    t0 = time.perf_counter()
    a.worker_poll(a.worker_submit(ptrs[128:]))
    relaunch = (time.perf_counter() - t0) * 1e3
    a.worker_stop()
    a.unregister_host_memory(pool.ctypes.data)
print(f"filter={int(filt)} "
      f"solo_ms={solo:.3f} "
      f"with_worker_ms={shared:.3f} next_burst_ms={relaunch:.3f}", flush=True)
