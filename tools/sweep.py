#!/usr/bin/env python3
"""Launch-shape sweep for yrss_parse_hash on one GPU.

Each configuration is a fresh context (the YRSS_* env knobs are read by
yrss_init).  Reports the parse kernel's average duration (hipEvents on its
stream), algorithmic GB/s and the full dispatch step time.

    python tools/sweep.py [--profile udp4] [--pkts N] [--out gpurun_out/sweep.json]
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--profile", default="udp4")
    ap.add_argument("--pkts", type=int, default=1 << 24)
    ap.add_argument("--stride", type=int, default=64)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--blocks", default="256,512,1024")
    ap.add_argument("--unroll", default="1,2")
    ap.add_argument("--nt", default="0,1")
    ap.add_argument("--wpc", default="16,24,32")
    ap.add_argument("--out", default=str(ROOT / "gpurun_out" / "sweep.json"))
    args = ap.parse_args()

    import torch

    import bench
    from yastack_amd import SoftRss, abi

    prof = bench.PROFILES[args.profile]
    n = args.pkts
    base = SoftRss(3, 3, 1, 1, device=0, max_burst=0)
    win, lens = base.synth(prof, n, 0, bench.SEED, bench.NFLOWS[args.profile], args.stride)
    out = base.alloc_out(n, win.device)
    torch.cuda.synchronize()
    ref_q = None
    rows = []
    combos = itertools.product([int(x) for x in args.blocks.split(",")],
                               [int(x) for x in args.unroll.split(",")],
                               [int(x) for x in args.nt.split(",")],
                               [int(x) for x in args.wpc.split(",")])
    for blk, unr, nt, wpc in combos:
        os.environ.update(YRSS_BLOCK=str(blk), YRSS_UNROLL=str(unr), YRSS_NT=str(nt),
                          YRSS_WAVES_PER_CU=str(wpc))
        eng = SoftRss(3, 3, 1, 1, device=0, max_burst=0)
        for _ in range(5):
            eng.dispatch_dev(win, lens, args.stride, n, out=out)
        torch.cuda.synchronize()
        eng.timing_enable(1 << abi.K_PARSE_HASH)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            eng.dispatch_dev(win, lens, args.stride, n, out=out)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ms, cnt = eng.timing_read(abi.K_PARSE_HASH)
        eng.timing_enable(0)
        q = out.q[:n].clone()
        if ref_q is None:
            ref_q = q
        same = bool(torch.equal(q, ref_q))
        k_us = ms / cnt * 1e3
        row = dict(block=blk, unroll=unr, nt=nt, wpc=wpc, grid=eng.grid_for(n),
                   kernel_us=round(k_us, 2), gbs=round(72 * n / (k_us * 1e-6) / 1e9, 1),
                   step_us=round(dt / args.steps * 1e6, 2),
                   mpps=round(n * args.steps / dt / 1e6, 1), same=same)
        rows.append(row)
        print(json.dumps(row), flush=True)
        eng.close()
    rows.sort(key=lambda r: r["kernel_us"])
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    Path(args.out).write_text(json.dumps({"profile": args.profile, "pkts": n, "rows": rows},
                                         indent=1))
    print("best:", json.dumps(rows[0]))


if __name__ == "__main__":
    main()
