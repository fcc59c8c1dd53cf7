#!/usr/bin/env python3
"""Phase clock of the line scatter (a YRSS_PROF_LINES build): per workgroup
and span, the 100 MHz realtime clock at each phase boundary, read by thread 0;
prints the mean time per phase over workgroups and spans, and the spread of
the workgroups' start and end.

    tools/build_ab_lib.sh prof -DYRSS_PROF_LINES=1
    python tools/line_prof.py --lib ab/lib/libyrss_prof.so --nb-procs 8,64
"""
from __future__ import annotations

import argparse
import ctypes
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

from yastack_amd import SoftRss, abi  # noqa: E402

PH = ["b1 tags/carried (and the next span's loads issued)", "b2 place", "wait + wave-0 layout + S2", "c copy-out", "d carry"]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--nb-procs", default="8,64")
    ap.add_argument("--pkts", type=int, default=1 << 24)
    ap.add_argument("--groups", type=int, default=0,
                    help="force the line-scatter kernel (yrss_debug_line_groups: 2 / 4 kG); "
                         "needs a -DYRSS_TEST_HOOKS build")
    ap.add_argument("--profile", default="tcp4", choices=("tcp4", "imix", "udp4"))
    ap.add_argument("--scan-kernel", type=int, default=0,
                    help="1: list prefixes from the scan kernel (yrss_tuning.scan_kernel)")
    args = ap.parse_args()
    lib = abi.load(str(ROOT / args.lib))
    lib.yrss_debug_line_prof.restype = ctypes.c_int
    lib.yrss_debug_line_prof.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    n = args.pkts
    for npr in (int(x) for x in args.nb_procs.split(",")):
        e = SoftRss(npr, npr, 1, 1, device=0, max_burst=0, lib_path=str(ROOT / args.lib))
        if args.groups:
            assert e._lib.yrss_debug_line_groups(e._ctx, args.groups, 0) == 0
        if args.scan_kernel:
            e.set_tuning(scan_kernel=1)
        w, l = e.synth({"tcp4": abi.SYN_TCP4, "imix": abi.SYN_IMIX, "udp4": abi.SYN_UDP4}[args.profile],
                       n, 0)
        out = e.alloc_out(n, w.device)
        buf = np.zeros(2048 * 8 * 8, np.uint64)
        for _ in range(4):
            e.dispatch_dev(w, l, 64, n, out=out)
        torch.cuda.synchronize()
        assert lib.yrss_debug_line_prof(buf.ctypes.data, buf.nbytes) > 0   # read + clear
        e.dispatch_dev(w, l, 64, n, out=out)
        torch.cuda.synchronize()
        assert lib.yrss_debug_line_prof(buf.ctypes.data, buf.nbytes) > 0
        p = buf.reshape(2048, 8, 8).astype(np.int64)
        used = p[:, :, 0] != 0
        blocks = int(used[:, 0].sum())
        spans = used.sum(axis=1)
        d = np.diff(p, axis=2) * 10  # ns
        m = used[:, :, None] & (p[:, :, 1:] != 0) & (p[:, :, :-1] != 0)
        if blocks == 0:
            print(f"q{npr}: no spans (one-list batch)")
            e.close()
            continue
        print(f"q{npr} {args.profile} groups {args.groups} scan_kernel {args.scan_kernel}: {blocks} workgroups, spans per workgroup {spans.min()}-{spans.max()}")
        for k, name in enumerate(PH):
            v = d[:, :, k][m[:, :, k]]
            if v.size == 0:
                continue
            print(f"   {name:20s} mean {v.mean():8.0f} ns  p90 {np.percentile(v, 90):8.0f}")
        first = p[:, 0, 0][used[:, 0]]
        lastidx = spans - 1
        ends = np.array([p[b, lastidx[b], len(PH)] for b in range(2048) if used[b, 0]])
        t0 = first.min()
        print(f"   workgroup start spread {(first.max() - t0) * 10:.0f} ns, "
              f"end {(ends.min() - t0) * 10:.0f}-{(ends.max() - t0) * 10:.0f} ns after the first start")
        per_span = (p[:, :, len(PH)] - p[:, :, 0])[used] * 10
        print(f"   span total mean {per_span.mean():.0f} ns")
        # slots 7 / 6 of span 0: kernel entry and the look-back's end
        entry = p[:, 0, 7][used[:, 0]]
        # slot 6: every thread done writing the next span's table (start of phase c)
        lay = (p[:, :, 6] - p[:, :, 3])[used & (p[:, :, 6] != 0)] * 10
        if lay.size:
            print(f"   next span's table write (start of c) mean {lay.mean():.0f} ns  "
                  f"p90 {np.percentile(lay, 90):.0f}")
        lbend = np.zeros(0)
        if (entry > 0).all():
            k0 = entry.min()
            pro = (first - entry) * 10
            print(f"   entry spread {(entry.max() - k0) * 10:.0f} ns; entry -> first span mean "
                  f"{pro.mean():.0f} p90 {np.percentile(pro, 90):.0f} ns")
            if lbend.size and (lbend > 0).all():
                print(f"   entry -> look-back done mean {((lbend - entry) * 10).mean():.0f} ns")
            # prologue milestones (slots 1-5 of the span-7 row): totals scanned,
            # one-list barrier passed, in-scatter prefixes done, first layout
            # barrier passed, first span's streams arrived
            pro_ms = p[:, 7, 1:6][used[:, 0]]
            names = ["totals scanned", "one-list barrier", "range prefixes", "first layout",
                     "streams arrived"]
            prev = entry
            for k, nm in enumerate(names):
                col = pro_ms[:, k]
                ok = col > 0
                if ok.any():
                    print(f"   prologue: -> {nm:18s} mean {((col - prev)[ok] * 10).mean():7.0f} ns")
                    prev = np.where(ok, col, prev)
            print(f"   prologue: -> first span         mean {((first - prev) * 10).mean():7.0f} ns")
            endk = (ends - k0) * 10
            ids = np.nonzero(used[:, 0])[0]
            print(f"   end after first entry: p10 {np.percentile(endk, 10):.0f} p50 "
                  f"{np.percentile(endk, 50):.0f} p90 {np.percentile(endk, 90):.0f} max "
                  f"{endk.max():.0f} ns")
            xcd = " ".join(f"{endk[ids % 8 == x].mean() / 1e3:.1f}" for x in range(8))
            print(f"   mean end by blockIdx % 8 (XCD), us: {xcd}")
            half = len(ids) // 2
            print(f"   mean end, first / second half of the grid: "
                  f"{endk[ids < half].mean() / 1e3:.1f} / {endk[ids >= half].mean() / 1e3:.1f} us")
        e.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
