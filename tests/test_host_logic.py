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

[port1]
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
