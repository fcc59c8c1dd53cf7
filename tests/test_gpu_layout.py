"""Parity across the work layouts and scatter paths (GPU).

The parse kernel deals chunks of tiles round-robin to its waves, counts per
chunk and ranks every packet in its chunk; the line scatter places each span
of chunks by those ranks (packed beside the bucket when it fits, else read
beside q) and writes whole list lines, carrying a bucket's unfinished line to
the next span; chunks longer than a span take the fallback scatter, which
ranks from q itself (yrss.hip layout_for, line_plan, yrss_scatter_lines,
yrss_scatter).  Chunk size, span size, parse grid and the XCD-contiguous
range mapping are layout choices only (yrss_set_tuning): every combination,
with the fused protocol_filter on or off, ragged batch sizes and window
strides 64 and 80, must give the oracle's q, hash and per-queue FIFO lists
bit-exactly (fs/lib/ff_dpdk_if.c:1945-2113 and the process_packets enqueue
order, :1058-1094), and no device guard may fire (fault record empty).

Paths and how the tests reach them: line scatter packed (<= 128 buckets at
default chunks), line scatter with q (257 buckets: 16-tile chunks leave no
room beside the rank), fallback (chunk_tiles=256: a chunk past the 8192-packet
span), one list (all-UDP), each with filter on and off.
"""
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


KNI = ("accept", "0-32767", "1000-40000,53,123")


def check(eng, oracle_mod, cfg_tuple, profile, n, stride=64, first=0, want_filter=False):
    """One device batch against the oracle: q, hash, qstart, qidx (and the
    filter class when asked), plus an empty fault record."""
    npr, nq, soft, only = cfg_tuple
    if want_filter:
        eng.set_kni(True, *KNI)
    win, lens = eng.synth(profile, n, first, stride=stride)
    res = eng.dispatch_dev(win, lens, stride, n, want_filter=want_filter)
    torch.cuda.synchronize()
    fault = eng.fault_info()
    assert fault[0] == abi.FAULT_NONE, f"device guard fired: {fault}"
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
    qi = to_np(res.qidx[:n], np.uint32)
    d = np.nonzero(qi != qi_ref)[0]
    assert d.size == 0, f"{d.size} qidx mismatches, first at {d[:5]}: {qi[d[:5]]} vs {qi_ref[d[:5]]}"
    if want_filter:
        want = oracle_mod.filter_windows(w_h, stride, l_h, True, oracle_mod.kni_bitmap(KNI[1]),
                                         oracle_mod.kni_bitmap(KNI[2]))
        assert np.array_equal(res.filter[:n].cpu().numpy(), want)
    return res


@pytest.mark.parametrize("want_filter", [False, True])
@pytest.mark.parametrize("chunk,span", [(1, 1), (1, 64), (2, 2), (8, 64), (32, 32),
                                        (4, 256), (128, 128), (256, 256)])
@pytest.mark.parametrize("profile", [abi.SYN_TCP4, abi.SYN_FUZZ])
def test_forced_layouts(dev, oracle_mod, chunk, span, profile, want_filter):
    """Chunk and span sizes are layout choices only: results never change
    (one-chunk spans, spans shorter than requested, and chunks past the line
    scatter's span, which take the fallback scatter, included)."""
    cfg = (5, 5, 1, 1)
    with SoftRss(*cfg, device=0, max_burst=0) as eng:
        eng.set_tuning(chunk_tiles=chunk, span_tiles=span)
        check(eng, oracle_mod, cfg, profile, 300001, first=777, want_filter=want_filter)


@pytest.mark.parametrize("stride", [64, 80])
@pytest.mark.parametrize("want_filter", [False, True])
@pytest.mark.parametrize("n", [4097, 5000, 77777, 1 << 20])
@pytest.mark.parametrize("cfg", [(2, 2, 1, 0), (3, 3, 1, 1), (8, 8, 1, 0), (16, 16, 1, 1),
                                 (64, 64, 1, 0), (255, 255, 1, 0), (4096, 256, 1, 1)])
def test_bucket_counts(dev, oracle_mod, cfg, n, want_filter, stride):
    """2 to 257 buckets, ragged sizes, filter on and off, strides 64 and 80."""
    with SoftRss(*cfg, device=0, max_burst=0) as eng:
        for profile in (abi.SYN_FUZZ, abi.SYN_IMIX):
            check(eng, oracle_mod, cfg, profile, n, stride=stride, first=n + 99,
                  want_filter=want_filter)


@pytest.mark.parametrize("cfg", [(8, 8, 1, 0), (8, 8, 1, 1)])
def test_filter_parity_fuzz_lists(dev, oracle_mod, cfg):
    """The configuration of round 2's faulted run (9 buckets, the fused
    filter, stride 64, n = 60001, fuzz then IMIX in one context), lists and
    fault record included."""
    with SoftRss(*cfg, device=0, max_burst=0) as eng:
        for profile in (abi.SYN_FUZZ, abi.SYN_IMIX):
            check(eng, oracle_mod, cfg, profile, 60001, first=99, want_filter=True)


@pytest.mark.parametrize("blocks", [1, 7, 64, 1000])
def test_parse_grid(dev, oracle_mod, blocks):
    """Fewer or more parse workgroups change the deal (chunks per wave and,
    with few waves, larger chunks so the count slots fit), not results."""
    for cfg in ((3, 3, 1, 1), (100, 100, 1, 1)):
        with SoftRss(*cfg, device=0, max_burst=0) as eng:
            eng.set_tuning(parse_blocks=blocks)
            check(eng, oracle_mod, cfg, abi.SYN_IMIX, 1 << 21, first=5)


def test_batch_beyond_default_chunks(dev, oracle_mod):
    """2^26 packets: more tiles than 65 536 four-tile chunks, so chunks grow to
    16 tiles (layout_for); the whole batch is compared with the oracle."""
    cfg = (3, 3, 1, 1)
    with SoftRss(*cfg, device=0, max_burst=0) as eng:
        check(eng, oracle_mod, cfg, abi.SYN_TCP4, 1 << 26, first=3)


@pytest.mark.parametrize("cfg", [(255, 255, 1, 0), (64, 64, 1, 1)])
def test_many_buckets_large_chunks(dev, oracle_mod, cfg):
    """Many buckets at 2^25 packets: chunks past the span size (a span is
    then one chunk, worked in several pieces)."""
    with SoftRss(*cfg, device=0, max_burst=0) as eng:
        check(eng, oracle_mod, cfg, abi.SYN_TCP4, 1 << 25, first=17)


@pytest.mark.parametrize("cfg", [(255, 255, 1, 0), (200, 200, 1, 1)])
def test_many_buckets_two_chunks_a_wave(dev, oracle_mod, cfg):
    """Past 128 buckets chunks grow with the batch up to 64 tiles, two a parse
    wave at 2^24 (layout_for): a ragged batch just past 2^24, fuzz traffic,
    compared in full."""
    with SoftRss(*cfg, device=0, max_burst=0) as eng:
        check(eng, oracle_mod, cfg, abi.SYN_FUZZ, (1 << 24) + 12345, first=23)


@pytest.mark.parametrize("profile", [abi.SYN_UDP4, abi.SYN_TCP4, abi.SYN_IMIX])
@pytest.mark.parametrize("shift", [1, 2, 3])
def test_unaligned_list_outputs(oracle_mod, profile, shift):
    """qidx (and q / hash) at 4-byte but not 16-byte alignment, n not a
    multiple of 4: the lists' 16-byte quads follow the address, not the index
    (one-list path on UDP, staged scatter on TCP / IMIX)."""
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
        assert eng.status() == 0
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
@pytest.mark.parametrize("cfg", [(3, 3, 1, 1), (8, 8, 1, 0), (48, 48, 1, 0), (255, 255, 1, 0)])
def test_scatter_xcd_mapping(dev, oracle_mod, cfg, xcd):
    """XCD-contiguous or round-robin spans: the same lists, ragged grids
    included (n not a multiple of a span)."""
    with SoftRss(*cfg, device=0, max_burst=0) as eng:
        eng.set_tuning(scatter_xcd=xcd)
        for profile in (abi.SYN_TCP4, abi.SYN_FUZZ):
            check(eng, oracle_mod, cfg, profile, 777777, first=31)


def test_line_scatter_capacity_is_enforced(dev, oracle_mod):
    """The line scatter's kG = 2 instantiation holds 128 buckets' layout words
    (line_nb_max).  Forced onto 256 buckets (round 4's hang) it is refused by
    the host with -EINVAL before anything runs; launched past that check it
    reports YRSS_FAULT_LINE_CAPACITY at kernel entry and leaves, with q and
    hash still exact.  Run once, through libyrss_test.so's hook."""
    import errno

    cfg = (255, 255, 1, 0)
    n = 1 << 20
    with SoftRss(*cfg, device=0, max_burst=0, lib_path=str(abi.TEST_LIB_PATH)) as eng:
        lib, ctx = eng._lib, eng._ctx
        win, lens = eng.synth(abi.SYN_TCP4, n, 5)
        assert lib.yrss_debug_line_groups(ctx, 3, 0) == -errno.EINVAL
        assert lib.yrss_debug_line_groups(ctx, 2, 0) == 0
        with pytest.raises(abi.YrssError) as ei:
            eng.dispatch_dev(win, lens, 64, n)
        assert ei.value.errno == errno.EINVAL
        torch.cuda.synchronize()
        assert eng.fault_info()[0] == abi.FAULT_NONE
        assert lib.yrss_debug_line_groups(ctx, 2, 1) == 0   # past the host check
        res = eng.dispatch_dev(win, lens, 64, n)
        torch.cuda.synchronize()
        assert eng.fault_info() == (abi.FAULT_LINE_CAPACITY, abi.K_SCATTER, 256, 128)
        w_h = win[: n * 64].cpu().numpy()
        q_ref, h_ref = oracle_mod.dispatch_windows(w_h, 64, to_np(lens[:n], np.uint16),
                                                   oracle_mod.cfg(*cfg))
        assert np.array_equal(to_np(res.q[:n], np.int16), q_ref)
        assert np.array_equal(to_np(res.hash[:n], np.uint32), h_ref)
        # the built-in choice again: lists exact, no fault
        assert lib.yrss_debug_line_groups(ctx, 0, 0) == 0
        check(eng, oracle_mod, cfg, abi.SYN_TCP4, n, first=5)


@pytest.mark.parametrize("n", [8191, 8193, 300001, (1 << 22) + 77])
@pytest.mark.parametrize("cfg", [(128, 128, 1, 0), (200, 200, 1, 1), (256, 256, 1, 0),
                                 (4096, 256, 1, 1)])
def test_many_bucket_counts(dev, oracle_mod, cfg, n):
    """129 to 257 buckets (the kG = 4 line scatter, rank beside q), spans cut
    short by n, fuzz, TCP and IMIX, filter on and off, compared in full."""
    with SoftRss(*cfg, device=0, max_burst=0) as eng:
        for profile, filt in ((abi.SYN_FUZZ, False), (abi.SYN_IMIX, True), (abi.SYN_TCP4, False)):
            check(eng, oracle_mod, cfg, profile, n, first=n + 7, want_filter=filt)


@pytest.mark.parametrize("groups", [2, 4])
@pytest.mark.parametrize("cfg", [(3, 3, 1, 1), (64, 64, 1, 0), (127, 127, 1, 0)])
def test_forced_line_kernels(dev, oracle_mod, cfg, groups):
    """Both line-scatter instantiations give the same lists wherever they
    may run: the 16 384-packet kG = 4 kernel forced below 128 buckets, through
    libyrss_test.so's hook; chunk and span overrides on top."""
    with SoftRss(*cfg, device=0, max_burst=0, lib_path=str(abi.TEST_LIB_PATH)) as eng:
        assert eng._lib.yrss_debug_line_groups(eng._ctx, groups, 0) == 0
        for profile in (abi.SYN_TCP4, abi.SYN_FUZZ):
            check(eng, oracle_mod, cfg, profile, 777777, first=41)
        eng.set_tuning(chunk_tiles=16, span_tiles=64)
        check(eng, oracle_mod, cfg, abi.SYN_FUZZ, 1 << 20, first=3)


@pytest.mark.parametrize("cfg", [(8, 8, 1, 0), (64, 64, 1, 1), (255, 255, 1, 0)])
def test_partial_line_merge_parity(dev, oracle_mod, cfg):
    """The partial list lines of each workgroup's range written with plain
    stores (yrss_debug_partial_merge: the two parts meet in L2) give the same
    lists, XCD mapping on and off (off: neighbouring ranges on other XCDs)."""
    with SoftRss(*cfg, device=0, max_burst=0, lib_path=str(abi.TEST_LIB_PATH)) as eng:
        assert eng._lib.yrss_debug_partial_merge(eng._ctx, 1) == 0
        for xcd in (1, 0):
            eng.set_tuning(scatter_xcd=xcd)
            for profile in (abi.SYN_TCP4, abi.SYN_FUZZ):
                check(eng, oracle_mod, cfg, profile, (1 << 22) + 999, first=7)


def test_tuning_rejects_bad_values(dev):
    with SoftRss(3, device=0, max_burst=0) as eng:
        for kw in ({"chunk_tiles": 3}, {"span_tiles": 6}, {"one_launch": 3}, {"scatter_xcd": 2},
                   {"scan_kernel": 2}):
            with pytest.raises(abi.YrssError):
                eng.set_tuning(**kw)


@pytest.mark.parametrize("cfg", [(1, 1, 1, 0), (3, 3, 1, 1), (8, 8, 1, 0), (15, 15, 1, 0),
                                 (16, 16, 1, 1)])
def test_in_scatter_prefixes(dev, oracle_mod, cfg):
    """Up to 16 buckets the line scatter makes its own list prefixes: the parse
    kernel adds each workgroup's counts to a totals set (the previous batch's
    scatter zeroed it), each scatter workgroup scans its range's chunk counts
    and adds the earlier ranges' aggregates; no scan kernel runs.  The same
    lists as the scan kernel (scan_kernel=1) batch after batch in one context,
    the two alternating (the totals sets must stay in step), ragged sizes, and
    layouts with one-chunk spans and many spans a workgroup; 17 buckets take
    the scan kernel either way."""
    with SoftRss(*cfg, device=0, max_burst=0) as eng:
        k = 0
        for n in (4097, 77777, (1 << 22) + 77, 1 << 24):
            for scan in (0, 1, 0, 0):
                eng.set_tuning(scan_kernel=scan)
                profile = (abi.SYN_TCP4, abi.SYN_FUZZ, abi.SYN_IMIX)[k % 3]
                check(eng, oracle_mod, cfg, profile, n, first=k * 1009)
                k += 1
        for chunk, span in ((1, 1), (4, 4), (1, 64)):
            eng.set_tuning(chunk_tiles=chunk, span_tiles=span)
            check(eng, oracle_mod, cfg, abi.SYN_FUZZ, (1 << 21) + 3, first=13)

