"""Device-path rate against batch size, 2^12 .. 2^31 packets of 64 B UDP
(BASELINE configs[1] traffic), one GPU: the full yrss_dispatch_dev step
(parse + hash + queue + per-queue lists) and the parse kernel alone (HIP
events on its launch stream).  The windows are generated once at the largest
size (128 GiB at 2^31); each size classifies a prefix.

    python tools/size_sweep.py [--max-log2 31] [--out gpurun_out/size_sweep.json]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from yastack_amd import SoftRss, abi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-log2", type=int, default=31)
    ap.add_argument("--out", default="gpurun_out/size_sweep.json")
    args = ap.parse_args()
    import torch

    dev = torch.device("cuda", 0)
    nmax = 1 << args.max_log2
    rows = []
    with SoftRss(3, 3, 1, 1, device=0, max_burst=0) as eng:
        win, lens = eng.synth(abi.SYN_UDP4, nmax, stride=64)
        out = eng.alloc_out(nmax, dev)
        torch.cuda.synchronize()
        lib = abi.load()
        sizes = sorted({lg for lg in list(range(12, args.max_log2 + 1, 2)) + [24, args.max_log2]
                        if lg <= args.max_log2})   # never past the buffers
        for lg in sizes:
            n = 1 << lg
            steps = max(5, min(200, (1 << 28) // n))
            for _ in range(3):
                eng.dispatch_dev(win, lens, 64, n, out=out)
            torch.cuda.synchronize()
            lib.yrss_timing_enable(eng._ctx, 1 << abi.K_PARSE_HASH)
            t0 = time.perf_counter()
            for _ in range(steps):
                eng.dispatch_dev(win, lens, 64, n, out=out)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / steps
            ms, cnt = ctypes.c_double(), ctypes.c_uint32()
            lib.yrss_timing_read(eng._ctx, abi.K_PARSE_HASH, ctypes.byref(ms), ctypes.byref(cnt))
            lib.yrss_timing_enable(eng._ctx, 0)
            k_us = ms.value / max(cnt.value, 1) * 1e3
            row = {"pkts": n, "steps": steps, "step_us": round(dt * 1e6, 2),
                   "gpkt_s": round(n / dt / 1e9, 2),
                   # batches of <= 4096 packets run as one untimed launch
                   "parse_us": round(k_us, 2) if cnt.value else None,
                   "parse_TBps": round(72 * n / (k_us * 1e-6) / 1e12, 3) if cnt.value else None}
            rows.append(row)
            print(json.dumps(row), flush=True)
        assert eng.status() == 0
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
