#!/usr/bin/env python3
"""Residency and look-back counters of the line scatter (a -DYRSS_LB_STATS
build): per batch, workgroups started / finished, the most finished any
starting workgroup saw (> 0: the grid was not resident at once), and the
look-back fallbacks taken (a granule not published within wait_ticks).

    python tools/lb_probe.py LIB [--nb-procs 3,64] [--tune k=v;...]
"""
import argparse
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

from yastack_amd import SoftRss, abi  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--nb-procs", default="3,8,64,255")
    ap.add_argument("--tune", default="")
    ap.add_argument("--pkts", type=int, default=1 << 24)
    args = ap.parse_args()
    lib = ctypes.CDLL(str(ROOT / args.lib))
    lib.yrss_debug_lb_stats.argtypes = [ctypes.POINTER(ctypes.c_uint32)]
    st = (ctypes.c_uint32 * 8)()
    for npr in (int(x) for x in args.nb_procs.split(",")):
        e = SoftRss(npr, npr, 1, 1, device=0, max_burst=0, lib_path=str(ROOT / args.lib))
        if args.tune:
            e.set_tuning(**{k: int(v) for k, v in (kv.split("=") for kv in args.tune.split(";"))})
        win, lens = e.synth(abi.SYN_TCP4, args.pkts, 0, stride=64)
        out = e.alloc_out(args.pkts, win.device)
        for it in range(3):
            lib.yrss_debug_lb_stats(st)   # clear
            e.dispatch_dev(win, lens, 64, args.pkts, out=out)
            torch.cuda.synchronize()
            lib.yrss_debug_lb_stats(st)
            print(f"q{npr} batch {it}: started {st[0]} finished {st[1]} "
                  f"max_finished_seen_at_start {st[2]} fallbacks {st[3]} status {e.status()}",
                  flush=True)
        e.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
