"""Soak test of the persistent burst worker (not part of the pytest suite):
random burst sizes (0..1024), mbuf and frames submissions, outputs in
registered or plain memory, per-slot output reuse, polls in random order and
non-blocking, idle gaps past the idle limit (the launch leaves and is
relaunched), lifetime exits, and device-resident batches on the same context
(which retire the worker).  Every burst is checked against the oracle.

    python tools/worker_soak.py --seconds 60
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle import oracle  # noqa: E402  (checker only)
from yastack_amd import SoftRss, abi  # noqa: E402

from test_gpu_parity import _fake_mbufs  # noqa: E402
from test_gpu_small_burst import _expect, _frames  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=30.0)
    ap.add_argument("--seed", type=int, default=1)
    args = ap.parse_args()
    os.environ.setdefault("YRSS_WORKER_IDLE_MS", "3")
    os.environ.setdefault("YRSS_WORKER_LIFE_MS", "150")
    import torch

    rng = np.random.default_rng(args.seed)
    cfg = (6, 5, 1, 1)
    npool = 1 << 15
    frames = _frames(oracle, npool, 1234)
    pool, ptrs, _ = _fake_mbufs(frames, headroom=128)
    data = (ptrs + np.uint64(256)).astype(np.uint64)
    flen = np.array([len(f) for f in frames], np.uint16)
    q_all, h_all, _, _ = _expect(oracle, frames, cfg)
    lib = abi.load()
    nslots, nblocks = 32, 8
    arena = np.zeros(nslots * 16384, np.uint8)
    slot_reg = []
    for k in range(nslots):
        b = arena[k * 16384:(k + 1) * 16384]
        slot_reg.append((b[0:2048].view(np.int16), b[2048:6144].view(np.uint32),
                         b[6144:10240].view(np.uint32), b[10240:10240 + 64].view(np.uint32)))
    stats = dict(bursts=0, pkts=0, relaunch_gaps=0, dev_batches=0, nonblock=0, empty=0)
    with SoftRss(*cfg, device=0, max_burst=0) as eng:
        eng.register_host_memory(pool.ctypes.data, pool.nbytes)
        eng.register_host_memory(arena.ctypes.data, arena.nbytes)
        eng.worker_start(nslots, nblocks)
        pend = {}           # ticket -> (off, n, outputs)
        issued = 0          # tickets are consecutive from 1; slot = ticket % nslots
        t_end = time.time() + args.seconds
        win_d, lens_d = eng.synth(abi.SYN_TCP4, 1 << 16)
        while time.time() < t_end or pend:
            # a slot is free once its previous ticket was polled
            submit = (time.time() < t_end and (issued + 1 - nslots) not in pend
                      and rng.random() < 0.6)
            if submit:
                n = int(rng.choice([0, 1, 32, 32, 32, 100, 1024, int(rng.integers(1, 1025))]))
                off = int(rng.integers(0, npool - n)) if n < npool else 0
                mode = rng.random()
                t = ctypes.c_uint64()
                if mode < 0.4:
                    outs = None   # per-slot registered arrays, chosen after the ticket
                elif mode < 0.7:
                    m = max(n, 1)
                    outs = (np.zeros(m, np.int16), np.zeros(m, np.uint32),
                            np.zeros(m, np.uint32), np.zeros(cfg[1] + 2, np.uint32))
                else:
                    m = max(n, 1)
                    outs = (np.zeros(m, np.int16), None, np.zeros(m, np.uint32),
                            np.zeros(cfg[1] + 2, np.uint32))
                if outs is None:   # the next ticket's slot keeps one output set
                    outs = slot_reg[(issued + 1) % nslots]
                q, h, qi, qs = outs
                frames_mode = rng.random() < 0.5
                if frames_mode:
                    rc = lib.yrss_worker_submit_frames(
                        eng._ctx, data[off:].ctypes.data, flen[off:].ctypes.data, n,
                        q.ctypes.data, None if h is None else h.ctypes.data, qi.ctypes.data,
                        qs.ctypes.data, ctypes.byref(t))
                else:
                    mb = np.ascontiguousarray(ptrs[off:off + n]) if n else ptrs[:1]
                    rc = lib.yrss_worker_submit(eng._ctx, mb.ctypes.data, n, q.ctypes.data,
                                                None if h is None else h.ctypes.data,
                                                qi.ctypes.data, qs.ctypes.data, 0,
                                                ctypes.byref(t))
                assert rc == 0, rc
                issued += 1
                assert t.value == issued
                pend[t.value] = (off, n, outs)
                stats["bursts"] += 1
                stats["pkts"] += n
                stats["empty"] += n == 0
                continue
            if pend and rng.random() < 0.9:
                # poll a random pending ticket, sometimes without waiting
                t = int(rng.choice(list(pend)))
                wait = rng.random() < 0.7
                rc = lib.yrss_worker_poll(eng._ctx, t, 1 if wait else 0)
                if rc == -11:
                    stats["nonblock"] += 1
                    continue
                assert rc == 0, (t, rc)
                off, n, (q, h, qi, qs) = pend.pop(t)
                qr = q_all[off:off + n]
                qi_ref, qs_ref = oracle.process_burst(qr, cfg[1])
                assert np.array_equal(q[:n], qr), t
                if h is not None:
                    assert np.array_equal(h[:n], h_all[off:off + n]), t
                assert np.array_equal(qi[:n], qi_ref), t
                assert np.array_equal(qs[: qs_ref.size], qs_ref), t
                continue
            r = rng.random()
            if r < 0.3:
                time.sleep(0.006)     # past the idle limit: the launch leaves
                stats["relaunch_gaps"] += 1
            elif r < 0.4:
                res = eng.dispatch_dev(win_d, lens_d, 64, 1 << 16)
                torch.cuda.synchronize()
                assert res.q is not None
                stats["dev_batches"] += 1
        eng.worker_stop()
        eng.unregister_host_memory(arena.ctypes.data)
        eng.unregister_host_memory(pool.ctypes.data)
    print("soak ok", stats, flush=True)


if __name__ == "__main__":
    main()
