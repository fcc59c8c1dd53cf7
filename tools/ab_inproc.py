#!/usr/bin/env python3
"""Paired A/B of library builds in ONE process on one GPU: every build gets
its own context (SoftRss(lib_path=...)) and fresh buffers placed behind a
random spacer, in shuffled order, round after round: box-level drift and the
placement of the buffers (worth up to ~5 % of the parse kernel for one and
the same build) hit all builds alike.  Per build and bucket count: mean over
rounds (and range) of the step time (no kernel events), and of the parse /
scan / scatter kernel averages (events on, a separate block).

    python tools/ab_inproc.py --nb-procs 8,64 --libs cur,ab/lib/libyrss_x.so \
        [--rounds 6] [--steps 20] [--profile tcp4] [--tune k=v,...]
"""
from __future__ import annotations

import argparse
import random
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

from yastack_amd import SoftRss, abi  # noqa: E402

PROFILES = {"udp4": abi.SYN_UDP4, "tcp4": abi.SYN_TCP4, "imix": abi.SYN_IMIX,
            "jumbo_tcp4": abi.SYN_JUMBO_TCP4}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nb-procs", default="8,64")
    ap.add_argument("--libs", default="cur")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--pkts", type=int, default=1 << 24)
    ap.add_argument("--batches", type=int, default=4)
    ap.add_argument("--profile", default="tcp4", choices=sorted(PROFILES))
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--ignore-faults", action="store_true",
                    help="measurement builds whose lists are wrong by design (a guard fires)")
    ap.add_argument("--tune", default="", help="k=v[;k=v] for every build, or per build "
                    "as lib@k=v in --libs (yrss_set_tuning fields; side=1 runs the "
                    "batches on a non-default stream)")
    args = ap.parse_args()
    n, stride = args.pkts, 64
    specs = []
    for s in args.libs.split(","):
        path, _, tune = s.partition("@")
        tune = tune or args.tune
        # "test": libyrss_test.so, whose hooks the dbg_* keys drive
        # (dbg_groups: yrss_debug_line_groups, dbg_merge: yrss_debug_partial_merge)
        lib = None if path == "cur" else str(abi.TEST_LIB_PATH) if path == "test" \
            else str(ROOT / path)
        specs.append((s, lib,
                      {k: int(v) for k, v in (kv.split("=") for kv in tune.split(";") if kv)}
                      if tune else {}))
    rng = random.Random(args.seed)
    for npr in (int(x) for x in args.nb_procs.split(",")):
        res = {name: {"step": [], "parse": [], "scan": [], "scatter": []} for name, _, _ in specs}
        for r in range(args.rounds):
            order = list(range(len(specs)))
            rng.shuffle(order)
            for i in order:
                name, path, tune = specs[i]
                # fresh buffers behind a random spacer each time: parse time
                # moves by up to ~5 % with where the buffers land (same build,
                # same process), so every build sees many placements
                spacer = torch.empty(rng.randrange(0, 64) << 21, dtype=torch.uint8,
                                     device="cuda")
                e = SoftRss(npr, npr, 1, 1, device=0, max_burst=0, lib_path=path)
                tn = dict(tune)
                # side=1: the caller's work on a non-default (non-blocking) stream
                st = torch.cuda.Stream() if tn.pop("side", 0) else None
                grp = tn.pop("dbg_groups", 0)
                if tn.pop("dbg_merge", 0):
                    assert e._lib.yrss_debug_partial_merge(e._ctx, 1) == 0
                if grp:
                    assert e._lib.yrss_debug_line_groups(e._ctx, grp, 0) == 0
                if tn:
                    e.set_tuning(**tn)
                wins = [e.synth(PROFILES[args.profile], n, k * n, stride=stride)
                        for k in range(args.batches)]
                outs = [e.alloc_out(n, wins[0][0].device) for _ in range(args.batches)]
                torch.cuda.synchronize()

                def run(steps, it=[0]):
                    for _ in range(steps):
                        k = it[0] % args.batches
                        it[0] += 1
                        e.dispatch_dev(wins[k][0], wins[k][1], stride, n, out=outs[k],
                                       stream=st)

                run(4)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                run(args.steps)
                torch.cuda.synchronize()
                res[name]["step"].append((time.perf_counter() - t0) / args.steps * 1e3)
                e.timing_enable((1 << abi.K_PARSE_HASH) | (1 << abi.K_SCAN) | (1 << abi.K_SCATTER))
                run(args.steps)
                torch.cuda.synchronize()
                for kname, k in (("parse", abi.K_PARSE_HASH), ("scan", abi.K_SCAN),
                                 ("scatter", abi.K_SCATTER)):
                    ms, cnt = e.timing_read(k)
                    res[name][kname].append(ms / max(cnt, 1) * 1e3)
                e.timing_enable(0)
                if e.status() != 0 and not args.ignore_faults:
                    print(f"{name}: device fault {e.fault_info()}")
                    return 1
                e.close()
                del wins, outs, spacer
                torch.cuda.empty_cache()
            print(f"round {r + 1} done", flush=True)
        for name, _, _ in specs:
            v = res[name]
            m = {k: statistics.mean(x) for k, x in v.items()}
            sd = statistics.stdev(v["parse"]) / len(v["parse"]) ** 0.5 if len(v["parse"]) > 1 else 0
            print(f"q{npr:<4d} {name:28s} step {m['step']:.4f} [{min(v['step']):.4f}-"
                  f"{max(v['step']):.4f}]  parse {m['parse']:6.1f} +-{sd:4.1f} "
                  f"[{min(v['parse']):.1f}-{max(v['parse']):.1f}]  scan {m['scan']:5.2f}  "
                  f"scatter {m['scatter']:6.2f}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
