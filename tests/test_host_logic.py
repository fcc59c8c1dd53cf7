"""Host-side logic on CPU: fs/lib config parsing, shard ranges, and the
shard-order merge of per-queue lists."""
import numpy as np
import pytest

from yastack_amd.ffconfig import load_ff_config, parse_lcore_mask, parse_list
from yastack_amd.shard import merge_queue_lists, shard_range

INI = """
[dpdk]
## Hexadecimal bitmask of cores to run on.
lcore_mask=7
channel=4
soft_dispatch=1
port_list=0,1

[system]
dispatch_only_core=1

[port0]
addr=10.0.0.2
netmask=255.255.255.0
broadcast=10.0.0.255
gateway=10.0.0.1

[port1]
addr=10.0.1.2
netmask=255.255.255.0
broadcast=10.0.1.255
gateway=10.0.1.1
lcore_list=0-1
"""


def test_ff_config(tmp_path):
    p = tmp_path / "f.ini"
    p.write_text(INI)
    fc = load_ff_config(str(p))
    assert fc.nb_procs == 3                       # popcount(0x7), ff_config.c:133
    assert fc.soft_dispatch == 1 and fc.dispatch_only_core == 1
    assert fc.nb_queues == {0: 3, 1: 2}           # default all lcores; port1 list


def test_lcore_mask_and_lists():
    assert parse_lcore_mask("f0") == [4, 5, 6, 7]
    assert parse_lcore_mask("0x1") == [0]
    with pytest.raises(ValueError):
        parse_lcore_mask("xyz")
    assert parse_list("1-3,0,7") == [0, 1, 2, 3, 7]


@pytest.mark.parametrize("n,w", [(0, 1), (10, 3), (1 << 20, 8), (7, 8)])
def test_shard_range_covers(n, w):
    got = [shard_range(n, w, r) for r in range(w)]
    assert got[0][0] == 0
    for (f0, c0), (f1, _) in zip(got, got[1:]):
        assert f0 + c0 == f1
    assert sum(c for _, c in got) == n
    assert max(c for _, c in got) - min(c for _, c in got) <= 1


def test_merge_matches_whole_batch(oracle_mod):
    win, lens = oracle_mod.synth(6, 5000, stride=80)
    c = oracle_mod.cfg(5, 4, 1, 0)
    q, _ = oracle_mod.dispatch_windows(win, 80, lens, c)
    qi_all, qs_all = oracle_mod.process_burst(q, 4)
    parts = []
    for r in range(3):
        f, cnt = shard_range(5000, 3, r)
        qi, qs = oracle_mod.process_burst(q[f:f + cnt], 4)
        parts.append((f, qi, qs))
    qi_m, qs_m = merge_queue_lists(parts)
    assert np.array_equal(qs_m, qs_all.astype(np.int64))
    assert np.array_equal(qi_m, qi_all.astype(np.int64))


def test_c_shard_helpers_match_python(oracle_mod):
    """yrss_shard_range / yrss_merge_queue_lists (C ABI, host-only) agree with
    shard.py and with the whole-batch lists."""
    import ctypes

    from yastack_amd import abi

    lib = abi.load()
    f, cnt = ctypes.c_uint64(), ctypes.c_uint64()
    for n, w in [(0, 1), (10, 3), (1 << 33, 8), (7, 8)]:
        for r in range(w):
            assert lib.yrss_shard_range(n, w, r, ctypes.byref(f), ctypes.byref(cnt)) == 0
            assert (f.value, cnt.value) == shard_range(n, w, r)
    assert lib.yrss_shard_range(5, 2, 2, ctypes.byref(f), ctypes.byref(cnt)) == -22

    win, lens = oracle_mod.synth(6, 5000, stride=80)
    c = oracle_mod.cfg(5, 4, 1, 0)
    q, _ = oracle_mod.dispatch_windows(win, 80, lens, c)
    qi_all, qs_all = oracle_mod.process_burst(q, 4)
    shards = [shard_range(5000, 4, r) for r in range(4)]
    parts = [oracle_mod.process_burst(q[a:a + k], 4) for a, k in shards]
    qis = [np.ascontiguousarray(p[0], np.uint32) for p in parts]
    qss = [np.ascontiguousarray(p[1], np.uint32) for p in parts]
    first = np.array([a for a, _ in shards], np.uint64)
    qi_ptrs = (ctypes.c_void_p * 4)(*[x.ctypes.data for x in qis])
    qs_ptrs = (ctypes.c_void_p * 4)(*[x.ctypes.data for x in qss])
    out_qi = np.zeros(5000, np.uint64)
    out_qs = np.zeros(6, np.uint64)
    assert lib.yrss_merge_queue_lists(4, 5, first.ctypes.data, ctypes.cast(qi_ptrs, ctypes.c_void_p),
                                      ctypes.cast(qs_ptrs, ctypes.c_void_p), out_qi.ctypes.data,
                                      out_qs.ctypes.data) == 0
    assert np.array_equal(out_qs, qs_all.astype(np.uint64))
    assert np.array_equal(out_qi, qi_all.astype(np.uint64))
    qi_py, qs_py = merge_queue_lists([(a, p[0], p[1]) for (a, _), p in zip(shards, parts)])
    assert np.array_equal(out_qi.astype(np.int64), qi_py)


def test_dispatch_dev_refuses_short_buffers():
    """The Python device-path wrapper checks buffer sizes before the raw
    pointers reach the GPU (a short buffer would fault the device)."""
    from yastack_amd.dispatch import DispatchResult, _check_dev_sizes

    class T:   # minimal tensor stand-in: numel / element_size
        def __init__(self, n, es):
            self.n, self.es = n, es

        def numel(self):
            return self.n

        def element_size(self):
            return self.es

    out = DispatchResult(T(100, 2), T(100, 4), T(100, 4), T(5, 4))
    _check_dev_sizes(100, 64, T(6400, 1), T(100, 2), out, 3)
    _check_dev_sizes(0, 64, T(64, 1), T(1, 2), out, 3)
    for bad in [dict(win=T(6399, 1)), dict(lens=T(99, 2))]:
        args = dict(win=T(6400, 1), lens=T(100, 2))
        args.update(bad)
        with pytest.raises(ValueError):
            _check_dev_sizes(100, 64, args["win"], args["lens"], out, 3)
    with pytest.raises(ValueError):
        _check_dev_sizes(101, 64, T(6464, 1), T(101, 2), out, 3)      # outputs too short
    with pytest.raises(ValueError):
        _check_dev_sizes(100, 64, T(6400, 1), T(100, 2),
                         DispatchResult(T(100, 2), T(100, 4), T(100, 4), T(3, 4)), 3)
    # the kernels write nb_queues+2 offsets (qstart[nb_queues+1] == n): a
    # nb_queues+1 array would take a 4-byte store past its end
    with pytest.raises(ValueError):
        _check_dev_sizes(100, 64, T(6400, 1), T(100, 2),
                         DispatchResult(T(100, 2), T(100, 4), T(100, 4), T(4, 4)), 3)
