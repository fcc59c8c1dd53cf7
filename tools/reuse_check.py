"""Does re-reading the same batch every step flatter the device-path rate?
The 256 MB MALL sits in front of HBM; a 1.2 GB batch re-read step after step
could keep part of itself there.  Times the bench workload (2^24 packets of
64 B UDP, configs[1]) with ONE batch re-read every step, and with FOUR
distinct batches (4.8 GB) rotated, so that no line is re-read within 3.6 GB of
other traffic.  Alternates the two modes a few times.

    python tools/reuse_check.py
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from yastack_amd import SoftRss, abi  # noqa: E402


def main():
    import torch

    dev = torch.device("cuda", 0)
    n, nbuf, steps = 1 << 24, 4, 48
    lib = abi.load()
    with SoftRss(3, 3, 1, 1, device=0, max_burst=0) as eng:
        bufs = [eng.synth(abi.SYN_UDP4, n, first=k * n, stride=64) for k in range(nbuf)]
        outs = [eng.alloc_out(n, dev) for _ in range(nbuf)]
        torch.cuda.synchronize()

        def run(rotate):
            for i in range(8):   # warm-up
                k = i % nbuf if rotate else 0
                eng.dispatch_dev(bufs[k][0], bufs[k][1], 64, n, out=outs[k])
            torch.cuda.synchronize()
            lib.yrss_timing_enable(eng._ctx, 1 << abi.K_PARSE_HASH)
            t0 = time.perf_counter()
            for i in range(steps):
                k = i % nbuf if rotate else 0
                eng.dispatch_dev(bufs[k][0], bufs[k][1], 64, n, out=outs[k])
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / steps
            ms, cnt = ctypes.c_double(), ctypes.c_uint32()
            lib.yrss_timing_read(eng._ctx, abi.K_PARSE_HASH, ctypes.byref(ms), ctypes.byref(cnt))
            lib.yrss_timing_enable(eng._ctx, 0)
            k_us = ms.value / max(cnt.value, 1) * 1e3
            return {"mode": "rotate4" if rotate else "same", "step_us": round(dt * 1e6, 1),
                    "gpkt_s": round(n / dt / 1e9, 2), "parse_us": round(k_us, 1),
                    "parse_TBps": round(72 * n / (k_us * 1e-6) / 1e12, 3)}

        for _ in range(3):
            for rotate in (False, True):
                print(json.dumps(run(rotate)), flush=True)
        assert eng.status() == 0


if __name__ == "__main__":
    main()
