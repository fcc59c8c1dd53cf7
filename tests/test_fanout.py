"""The fan-out's host logic on CPU (yrss_fanout_route, in-order hand-off).

One dispatcher thread spreads consecutive bursts round-robin over N contexts
(GPUs) and takes them back in submission order; handing each burst's
per-queue lists to the rings in that order keeps every queue FIFO over the
whole stream, the invariant rte_ring gives the reference
(fs/lib/ff_dpdk_if.c:1087-1093).  Checked here with the oracle standing in
for the GPUs; tests/test_gpu_fanout.py runs the real thing.
"""
import ctypes

import numpy as np
import pytest

from yastack_amd import abi


def _route(lib, g, n):
    k, t = ctypes.c_uint32(), ctypes.c_uint64()
    rc = lib.yrss_fanout_route(g, n, ctypes.byref(k), ctypes.byref(t))
    return rc, k.value, t.value


def test_route_round_robin():
    lib = abi.load()
    for nctx in (1, 2, 3, 8):
        seen = {k: [] for k in range(nctx)}
        for g in range(1, 200):
            rc, k, t = _route(lib, g, nctx)
            assert rc == 0 and k == (g - 1) % nctx
            seen[k].append(t)
        for k, ts in seen.items():      # every context numbers its bursts 1, 2, 3, ...
            assert ts == list(range(1, len(ts) + 1))
    assert _route(lib, 0, 2)[0] == -22 and _route(lib, 1, 0)[0] == -22


def _bursts(oracle_mod, seed, total=20000):
    rng = np.random.default_rng(seed)
    win, lens = oracle_mod.synth(abi.SYN_IMIX, total, seed, stride=80)
    c = oracle_mod.cfg(5, 4, 1, 1)
    q, _ = oracle_mod.dispatch_windows(win, 80, lens, c)
    sizes, off = [], 0
    while off < total:
        n = int(min(total - off, rng.integers(0, 1025)))
        sizes.append(n)
        off += n
    firsts = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    per = [oracle_mod.process_burst(q[f:f + n], 4) for f, n in zip(firsts, sizes)]
    return q, sizes, firsts, per


def _merge(lib, firsts, per, order):
    qis = [np.ascontiguousarray(per[i][0], np.uint32) for i in order]
    qss = [np.ascontiguousarray(per[i][1], np.uint32) for i in order]
    first = np.ascontiguousarray([firsts[i] for i in order], np.uint64)
    m = len(order)
    qi_p = (ctypes.c_void_p * m)(*[x.ctypes.data for x in qis])
    qs_p = (ctypes.c_void_p * m)(*[x.ctypes.data for x in qss])
    total = int(sum(x[-1] for x in qss))
    out_qi = np.zeros(max(total, 1), np.uint64)
    out_qs = np.zeros(6, np.uint64)
    assert lib.yrss_merge_queue_lists(m, 5, first.ctypes.data,
                                      ctypes.cast(qi_p, ctypes.c_void_p),
                                      ctypes.cast(qs_p, ctypes.c_void_p), out_qi.ctypes.data,
                                      out_qs.ctypes.data) == 0
    return out_qi[:total], out_qs


@pytest.mark.parametrize("nctx", [1, 2, 3, 8])
def test_in_order_handoff_keeps_queue_fifo(oracle_mod, nctx):
    """Bursts complete on their contexts in any order; the hand-off takes them
    in ticket order (what yrss_fanout_next does) and the rings' contents equal
    the single-dispatcher answer.  Taking them as they complete does not."""
    lib = abi.load()
    q, sizes, firsts, per = _bursts(oracle_mod, 100 + nctx)
    qi_all, qs_all = oracle_mod.process_burst(q, 4)
    rng = np.random.default_rng(nctx)
    # simulated completion: each context finishes its own bursts in order, the
    # contexts interleave at random
    queues = {k: [] for k in range(nctx)}
    for g in range(1, len(sizes) + 1):
        _, k, _ = _route(lib, g, nctx)
        queues[k].append(g)
    completion = []
    while any(queues.values()):
        k = int(rng.choice([k for k, v in queues.items() if v]))
        completion.append(queues[k].pop(0))
    # in-order hand-off: ticket g is released only after g-1
    done, handed, order = set(), 0, []
    for g in completion:
        done.add(g)
        while handed + 1 in done:
            handed += 1
            order.append(handed - 1)
    qi, qs = _merge(lib, firsts, per, order)
    assert np.array_equal(qs, qs_all.astype(np.uint64))
    assert np.array_equal(qi, qi_all.astype(np.uint64))
    if nctx > 1 and completion != sorted(completion):
        qi_c, _ = _merge(lib, firsts, per, [g - 1 for g in completion])
        assert not np.array_equal(qi_c, qi_all.astype(np.uint64))


def test_fanout_needs_a_gpu():
    """Without a GPU the fan-out fails loudly (no CPU fallback)."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    lib = abi.load()
    cfg = abi.default_config()
    devs = (ctypes.c_int * 2)(0, 0)
    f = ctypes.c_void_p()
    rc = lib.yrss_fanout_init(ctypes.byref(cfg), devs, 2, 16, 4, ctypes.byref(f))
    assert rc < 0 and not f.value
