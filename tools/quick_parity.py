#!/usr/bin/env python3
"""Quick GPU parity sweep of yrss_dispatch_dev against the oracle: bucket
counts x streams x ragged sizes, q / hash / qidx / qstart compared in full and
the fault record asserted empty after every batch.  Prints one line per case
and exits non-zero on the first mismatch.

    python tools/quick_parity.py [--big] [--lib ab/lib/libyrss_X.so] [--tune k=v;...]
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main() -> int:
    import torch

    from oracle import oracle
    from yastack_amd import SoftRss, abi

    big = "--big" in sys.argv
    lib = None
    tune = {}
    for i, a in enumerate(sys.argv):
        if a == "--lib":
            lib = str(ROOT / sys.argv[i + 1])
        if a == "--tune":
            tune = {k: int(v) for k, v in (kv.split("=") for kv in sys.argv[i + 1].split(";") if kv)}
    cfgs = [(3, 3, 1, 1), (2, 2, 1, 0), (8, 8, 1, 0), (8, 8, 1, 1), (16, 16, 1, 0),
            (64, 64, 1, 1), (255, 255, 1, 0), (4096, 256, 1, 1), (5, 3, 1, 0)]
    sizes = [4097, 5000, 300001] + ([1 << 22] if big else [])
    profs = [abi.SYN_TCP4, abi.SYN_FUZZ, abi.SYN_UDP4, abi.SYN_IMIX]
    bad = 0
    for cfg in cfgs:
        with SoftRss(*cfg, device=0, max_burst=0, lib_path=lib) as eng:
            if tune:
                eng.set_tuning(**tune)
            for prof in profs:
                for n in sizes:
                    win, lens = eng.synth(prof, n, 1234 + n, stride=64)
                    res = eng.dispatch_dev(win, lens, 64, n)
                    torch.cuda.synchronize()
                    f = eng.fault_info()
                    w_h = win[: n * 64].cpu().numpy()
                    l_h = lens[:n].cpu().numpy().view(np.uint16)
                    q_ref, h_ref = oracle.dispatch_windows(w_h, 64, l_h, oracle.cfg(*cfg))
                    qi_ref, qs_ref = oracle.process_burst(q_ref, cfg[1])
                    ok_q = np.array_equal(res.q[:n].cpu().numpy(), q_ref)
                    ok_h = np.array_equal(res.hash[:n].cpu().numpy().view(np.uint32), h_ref)
                    ok_s = np.array_equal(res.qstart.cpu().numpy().view(np.uint32), qs_ref)
                    qi = res.qidx[:n].cpu().numpy().view(np.uint32)
                    ok_i = np.array_equal(qi, qi_ref)
                    ok = ok_q and ok_h and ok_s and ok_i and f[0] == 0
                    line = f"cfg={cfg} prof={abi.SYN_NAMES[prof]} n={n} q={ok_q} h={ok_h} " \
                           f"qstart={ok_s} qidx={ok_i} fault={f}"
                    print(("ok   " if ok else "FAIL ") + line, flush=True)
                    if not ok:
                        bad += 1
                        if not ok_i:
                            d = np.nonzero(qi != qi_ref)[0]
                            print("   first qidx diffs at", d[:8], qi[d[:8]], qi_ref[d[:8]],
                                  "of", d.size, flush=True)
                        if bad > 3:
                            return 1
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
