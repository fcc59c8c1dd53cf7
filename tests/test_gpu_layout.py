"""Parity across the parse kernel's work layouts (GPU).

The parse kernel deals chunks of tiles round-robin to its waves, counts per
chunk, and the scatter works per group of chunks (yrss.hip layout_for).  The
chunk size depends on the bucket count and on the batch size, and can be forced
with YRSS_CHUNK_TILES / YRSS_GROUP_TILES (read at yrss_init).  Every layout
must give the same bit-exact q, hash and per-queue FIFO lists as the oracle
(fs/lib/ff_dpdk_if.c:1945-2113 and the process_packets enqueue order,
:1058-1094).
"""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from yastack_amd import SoftRss, abi  # noqa: E402


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch.device("cuda", 0)


def to_np(t, dtype):
    return t.cpu().numpy().view(dtype)


def check(eng, oracle_mod, cfg_tuple, profile, n, stride=64, first=0):
    npr, nq, soft, only = cfg_tuple
    win, lens = eng.synth(profile, n, first, stride=stride)
    res = eng.dispatch_dev(win, lens, stride, n)
    torch.cuda.synchronize()
    assert eng.status() == 0   # no scan look-back or scatter guard fired
    w_h = win[: n * stride].cpu().numpy()
    l_h = to_np(lens[:n], np.uint16)
    c = oracle_mod.cfg(npr, nq, soft, only)
    q_ref, h_ref = oracle_mod.dispatch_windows(w_h, stride, l_h, c)
    q = to_np(res.q[:n], np.int16)
    h = to_np(res.hash[:n], np.uint32)
    bad = np.nonzero((q != q_ref) | (h != h_ref))[0]
    assert bad.size == 0, f"{bad.size} q/hash mismatches, first at {bad[:5]}"
    qi_ref, qs_ref = oracle_mod.process_burst(q_ref, nq)
    assert np.array_equal(to_np(res.qstart, np.uint32), qs_ref)
    assert np.array_equal(to_np(res.qidx[:n], np.uint32), qi_ref)


class _env:
    def __init__(self, **kv):
        self.kv = {k: str(v) for k, v in kv.items()}

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update(self.kv)

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("chunk,group", [(1, 1), (1, 64), (2, 2), (8, 64), (32, 32),
                                         (4, 256), (128, 128)])
@pytest.mark.parametrize("profile", [abi.SYN_TCP4, abi.SYN_FUZZ])
def test_forced_layouts(dev, oracle_mod, chunk, group, profile):
    """Chunk and group sizes are tuning knobs only: results never change."""
    cfg = (5, 5, 1, 1)
    with _env(YRSS_CHUNK_TILES=chunk, YRSS_GROUP_TILES=group):
        with SoftRss(*cfg, device=0, max_burst=0) as eng:
            check(eng, oracle_mod, cfg, profile, 300001, first=777)


@pytest.mark.parametrize("cfg", [(32, 32, 1, 0), (100, 100, 1, 1), (17, 17, 1, 0)])
def test_bucket_count_layouts(dev, oracle_mod, cfg):
    """Past 17 buckets chunks are 16 tiles while the count slots per wave
    hold them (yrss.hip layout_for), larger past that."""
    with SoftRss(*cfg, device=0, max_burst=0) as eng:
        for profile in (abi.SYN_TCP4, abi.SYN_IMIX):
            check(eng, oracle_mod, cfg, profile, 1 << 20, first=99)


@pytest.mark.parametrize("waves", [4, 12, 32])
def test_occupancy_knob(dev, oracle_mod, waves):
    """Fewer or more resident waves change the deal (chunks per wave), not results."""
    cfg = (3, 3, 1, 1)
    with _env(YRSS_WAVES_PER_CU=waves):
        with SoftRss(*cfg, device=0, max_burst=0) as eng:
            check(eng, oracle_mod, cfg, abi.SYN_IMIX, 1 << 21, first=5)


def test_batch_beyond_default_chunks(dev, oracle_mod):
    """2^26 packets: more tiles than 65 536 four-tile chunks, so chunks grow to
    16 tiles (layout_for); the whole batch is compared with the oracle."""
    cfg = (3, 3, 1, 1)
    with SoftRss(*cfg, device=0, max_burst=0) as eng:
        check(eng, oracle_mod, cfg, abi.SYN_TCP4, 1 << 26, first=3)


@pytest.mark.parametrize("cfg", [(9, 9, 1, 0), (32, 32, 1, 0), (4096, 256, 1, 1)])
def test_ballot_scatter_without_ranks(dev, oracle_mod, cfg):
    """YRSS_NO_RANK=1 keeps many-bucket batches on the ballot-ranked scatter
    (no per-packet ranks from the parse kernel); same lists either way."""
    with _env(YRSS_NO_RANK=1):
        with SoftRss(*cfg, device=0, max_burst=0) as eng:
            check(eng, oracle_mod, cfg, abi.SYN_FUZZ, 500001, first=11)
    with SoftRss(*cfg, device=0, max_burst=0) as eng:
        check(eng, oracle_mod, cfg, abi.SYN_FUZZ, 500001, first=11)


@pytest.mark.parametrize("profile", [abi.SYN_UDP4, abi.SYN_TCP4, abi.SYN_IMIX])
@pytest.mark.parametrize("shift", [1, 2, 3])
def test_unaligned_list_outputs(oracle_mod, profile, shift):
    """qidx (and q / hash) at 4-byte but not 16-byte alignment, n not a
    multiple of 4: the list paths' unaligned heads and tails (one-list
    grid-stride path on UDP, LDS-image path on TCP / IMIX)."""
    n, stride = 300007, 64
    with SoftRss(3, 3, 1, 1, device=0, max_burst=0) as eng:
        win, lens = eng.synth(profile, n, 17, stride=stride)
        dev = win.device
        qi_buf = torch.full((n + 8,), -1, dtype=torch.int32, device=dev)
        q_buf = torch.empty(n + 8, dtype=torch.int16, device=dev)
        h_buf = torch.empty(n + 8, dtype=torch.int32, device=dev)
        qs = torch.empty(3 + 2, dtype=torch.int32, device=dev)
        from yastack_amd.dispatch import DispatchResult
        out = DispatchResult(q_buf[2 * shift:2 * shift + n], h_buf[shift:shift + n],
                             qi_buf[shift:shift + n], qs)
        res = eng.dispatch_dev(win, lens, stride, n, out=out)
        torch.cuda.synchronize()
        w_h = win[: n * stride].cpu().numpy()
        l_h = lens[:n].cpu().numpy().view(np.uint16)
        q_ref, h_ref = oracle_mod.dispatch_windows(w_h, stride, l_h, oracle_mod.cfg(3, 3, 1, 1))
        qi_ref, qs_ref = oracle_mod.process_burst(q_ref, 3)
        assert np.array_equal(res.q.cpu().numpy(), q_ref)
        assert np.array_equal(res.hash.cpu().numpy().view(np.uint32), h_ref)
        assert np.array_equal(qs.cpu().numpy().view(np.uint32), qs_ref)
        qi_all = qi_buf.cpu().numpy()
        assert np.array_equal(qi_all[shift:shift + n].view(np.uint32), qi_ref)
        assert (qi_all[:shift] == -1).all() and (qi_all[shift + n:] == -1).all()   # no overrun


@pytest.mark.parametrize("xcd", [0, 1])
@pytest.mark.parametrize("cfg", [(3, 3, 1, 1), (8, 8, 1, 0), (16, 16, 1, 0), (48, 48, 1, 0),
                                 (64, 64, 1, 1), (255, 255, 1, 0)])
def test_scatter_xcd_mapping(dev, oracle_mod, cfg, xcd):
    """YRSS_SCATTER_XCD moves scatter groups between workgroups (XCD-contiguous
    or round-robin; default by bucket count): every path's lists are the same,
    including ragged grids (n not a multiple of a group)."""
    with _env(YRSS_SCATTER_XCD=xcd):
        with SoftRss(*cfg, device=0, max_burst=0) as eng:
            for profile in (abi.SYN_TCP4, abi.SYN_FUZZ):
                check(eng, oracle_mod, cfg, profile, 777777, first=31)


@pytest.mark.parametrize("group", [16, 32, 64])
@pytest.mark.parametrize("cfg", [(7, 7, 1, 0), (8, 8, 1, 0), (12, 12, 1, 1), (16, 16, 1, 0), (48, 48, 1, 0),
                                 (100, 100, 1, 1), (255, 255, 1, 0), (4096, 256, 1, 1)])
def test_ranked_group_stage(dev, oracle_mod, cfg, group):
    """YRSS_RANK_GSTAGE: the ranked scatter sorts a whole group in one packed
    LDS stage (YRSS_RANK_IMG=0 so it also runs at 49 buckets); same lists for
    any group size, ragged and small batches included."""
    with _env(YRSS_RANK_GSTAGE=1, YRSS_RANK_IMG=0, YRSS_GROUP_TILES=group):
        with SoftRss(*cfg, device=0, max_burst=0) as eng:
            for profile, n in ((abi.SYN_TCP4, 1 << 20), (abi.SYN_FUZZ, 777777), (abi.SYN_IMIX, 5001)):
                check(eng, oracle_mod, cfg, profile, n, first=47)
