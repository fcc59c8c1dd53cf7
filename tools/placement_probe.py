#!/usr/bin/env python3
"""Which buffer's placement moves the parse kernel?  One build, tcp4 at the
given nb_procs; per trial, only the chosen buffers are re-allocated behind a
random spacer (the rest stay put), and the parse / scatter kernel averages
are recorded.  Modes: win (windows + lens), out (q / hash / lists), ctx (the
context's internal buffers: ranks, counts), all.

    python tools/placement_probe.py --mode win,out,ctx,all --trials 8
"""
from __future__ import annotations

import argparse
import random
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

from yastack_amd import SoftRss, abi  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="win,out,ctx,all")
    ap.add_argument("--trials", type=int, default=8)
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--nb-procs", type=int, default=8)
    ap.add_argument("--pkts", type=int, default=1 << 24)
    ap.add_argument("--batches", type=int, default=4)
    args = ap.parse_args()
    n, stride, npr = args.pkts, 64, args.nb_procs
    rng = random.Random(7)
    keep = []

    def spacer():
        keep.append(torch.empty(rng.randrange(1, 64) << 21, dtype=torch.uint8, device="cuda"))

    def new_eng():
        return SoftRss(npr, npr, 1, 1, device=0, max_burst=0)

    def new_wins(e):
        spacer()
        return [e.synth(abi.SYN_TCP4, n, k * n, stride=stride) for k in range(args.batches)]

    def new_outs(e):
        spacer()
        return [e.alloc_out(n, torch.device("cuda", 0)) for _ in range(args.batches)]

    for mode in args.mode.split(","):
        e = new_eng()
        wins, outs = new_wins(e), new_outs(e)
        parse, scat = [], []
        for t in range(args.trials):
            if mode in ("win", "all"):
                wins = new_wins(e)
            if mode in ("out", "all"):
                outs = new_outs(e)
            if mode in ("ctx", "all"):
                e.close()
                spacer()
                e = new_eng()
            torch.cuda.synchronize()
            it = [0]

            def run(steps):
                for _ in range(steps):
                    k = it[0] % args.batches
                    it[0] += 1
                    e.dispatch_dev(wins[k][0], wins[k][1], stride, n, out=outs[k])

            run(4)
            e.timing_enable((1 << abi.K_PARSE_HASH) | (1 << abi.K_SCATTER))
            run(args.steps)
            torch.cuda.synchronize()
            ms, c = e.timing_read(abi.K_PARSE_HASH)
            parse.append(ms / max(c, 1) * 1e3)
            ms, c = e.timing_read(abi.K_SCATTER)
            scat.append(ms / max(c, 1) * 1e3)
            e.timing_enable(0)
            if len(keep) > 6:
                keep.pop(0)
        e.close()
        del wins, outs
        keep.clear()
        torch.cuda.empty_cache()
        print(f"q{npr} mode {mode:4s} parse mean {statistics.mean(parse):6.1f} sd "
              f"{statistics.pstdev(parse):4.1f} [{min(parse):.1f}-{max(parse):.1f}]  "
              f"scatter mean {statistics.mean(scat):5.1f} [{min(scat):.1f}-{max(scat):.1f}]  "
              f"parse trials {[round(x, 1) for x in parse]}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
