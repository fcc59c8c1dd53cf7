#!/usr/bin/env python3
"""Where the line scatter's lists go wrong, per bucket: the first list
position that differs from the oracle, the packet there and its span.

    python tools/lb_debug.py [--lib L] [--tune k=v;...] [--n N] [--cfg a,b,c,d]
        [--chunk 2 --span 2] [--profile 5]
"""
import argparse
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

from oracle import oracle  # noqa: E402
from yastack_amd import SoftRss  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--tune", default="chunk_tiles=2;span_tiles=2")
    ap.add_argument("--n", type=int, default=300001)
    ap.add_argument("--first", type=int, default=777)
    ap.add_argument("--cfg", default="5,5,1,1")
    ap.add_argument("--profile", type=int, default=5)
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    cfg = tuple(int(x) for x in args.cfg.split(","))
    tune = {k: int(v) for k, v in (kv.split("=") for kv in args.tune.split(";") if kv)}
    lib = str(ROOT / args.lib) if args.lib else None
    bad = 0
    for rep in range(args.reps):
        with SoftRss(*cfg, device=0, max_burst=0, lib_path=lib) as eng:
            if tune:
                eng.set_tuning(**tune)
            win, lens = eng.synth(args.profile, args.n, args.first, stride=64)
            res = eng.dispatch_dev(win, lens, 64, args.n)
            torch.cuda.synchronize()
            f = eng.fault_info()
            w_h = win[: args.n * 64].cpu().numpy()
            l_h = lens[: args.n].cpu().numpy().view(np.uint16)
            q_ref, _ = oracle.dispatch_windows(w_h, 64, l_h, oracle.cfg(*cfg))
            qi_ref, qs_ref = oracle.process_burst(q_ref, cfg[1])
            qi = res.qidx[: args.n].cpu().numpy().view(np.uint32)
            qs = res.qstart.cpu().numpy().view(np.uint32)
            print(f"rep {rep} fault {f} qstart ok {np.array_equal(qs, qs_ref)} "
                  f"qidx mismatches {(qi != qi_ref).sum()}", flush=True)
            for b in range(len(qs_ref) - 1):
                lo, hi = int(qs_ref[b]), int(qs_ref[b + 1])
                d = np.nonzero(qi[lo:hi] != qi_ref[lo:hi])[0]
                if d.size:
                    bad += 1
                    p = lo + int(d[0])
                    # which got value sits one before/after
                    print(f"  bucket {b}: {d.size} wrong of {hi - lo}, first at list pos {p} "
                          f"(pkt {qi_ref[p]} span@128 {qi_ref[p] // 128}); got {qi[p:p + 3]} "
                          f"want {qi_ref[p:p + 3]}; last wrong pos {lo + int(d[-1])}", flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
