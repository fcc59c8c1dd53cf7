"""GPU parity of the one-launch small-burst path (yrss_burst_small, n <= 4096
and nb_queues + 1 <= 64) against the oracle, on every host-resident entry
point, at sizes on both sides of the threshold.  The multi-kernel path
(YRSS_NO_SMALL=1) must give identical results.
"""

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from yastack_amd import SoftRss, abi  # noqa: E402

from test_gpu_parity import _fake_mbufs  # noqa: E402

SIZES = [1, 31, 32, 33, 1024, 4095, 4096, 4097]


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch.device("cuda", 0)


def _frames(oracle_mod, n, seed):
    win, lens = oracle_mod.synth(abi.SYN_FUZZ, n, seed, stride=80)
    out = []
    for i in range(n):
        L = min(int(lens[i]), 2048)
        f = win[i * 80:(i + 1) * 80].tobytes()
        out.append((f + bytes(max(0, L - 80)))[:L])
    return out


def _expect(oracle_mod, frames, cfg):
    c = oracle_mod.cfg(*cfg)
    want = [oracle_mod.toeplitz_dispatch(f, len(f), c) for f in frames]
    q = np.array([x for x, _ in want], np.int16)
    h = np.array([y for _, y in want], np.uint32)
    qi, qs = oracle_mod.process_burst(q, cfg[1])
    return q, h, qi, qs


def _check(r, q, h, qi, qs):
    assert np.array_equal(np.asarray(r.q), q)
    assert np.array_equal(np.asarray(r.hash), h)
    assert np.array_equal(np.asarray(r.qidx), qi)
    assert np.array_equal(np.asarray(r.qstart)[: qs.size], qs)


@pytest.mark.parametrize("n", SIZES)
def test_small_burst_all_host_apis(dev, oracle_mod, n):
    cfg = (5, 4, 1, 1)
    frames = _frames(oracle_mod, n, 1000 + n)
    q, h, qi, qs = _expect(oracle_mod, frames, cfg)
    pool, ptrs, stride = _fake_mbufs(frames, headroom=131)
    with SoftRss(*cfg, device=0, max_burst=0) as eng:
        _check(eng.dispatch_frames(frames), q, h, qi, qs)
        _check(eng.dispatch_burst(ptrs, write_rss=True), q, h, qi, qs)
        rss = pool.reshape(-1, stride)[:, 44:48].copy().view(np.uint32).ravel()
        assert np.array_equal(rss, h)
        pool.reshape(-1, stride)[:, 44:48] = 0
        eng.register_host_memory(pool.ctypes.data, pool.nbytes)
        _check(eng.dispatch_burst_zc(ptrs, write_rss=True), q, h, qi, qs)
        rss = pool.reshape(-1, stride)[:, 44:48].copy().view(np.uint32).ravel()
        assert np.array_equal(rss, h)
        # frames_zc with pageable pointer/length arrays (staged by the library)
        data = (ptrs + np.uint64(128 + 131)).astype(np.uint64)
        flen = np.array([len(f) for f in frames], np.uint16)
        lib = abi.load()
        qq = np.empty(n, np.int16)
        hh = np.empty(n, np.uint32)
        qii = np.empty(n, np.uint32)
        qss = np.empty(cfg[1] + 2, np.uint32)
        rc = lib.yrss_dispatch_frames_zc(eng._ctx, data.ctypes.data, flen.ctypes.data, n,
                                         qq.ctypes.data, hh.ctypes.data, qii.ctypes.data,
                                         qss.ctypes.data)
        assert rc == 0
        assert np.array_equal(qq, q) and np.array_equal(hh, h)
        assert np.array_equal(qii, qi) and np.array_equal(qss[: qs.size], qs)
        eng.unregister_host_memory(pool.ctypes.data)


def test_small_burst_registered_outputs(dev, oracle_mod):
    """Outputs in registered memory are written by the kernel in place."""
    n, cfg = 1500, (8, 8, 1, 0)
    frames = _frames(oracle_mod, n, 77)
    q, h, qi, qs = _expect(oracle_mod, frames, cfg)
    pool, ptrs, _ = _fake_mbufs(frames, headroom=128)
    raw = np.zeros(n * 32 + 3 * 4096, np.uint8)
    off = (-raw.ctypes.data) % 4096
    arena = raw[off: off + n * 32 + 4096]
    a_ptr = arena[: n * 8].view(np.uint64)
    a_q = arena[n * 8: n * 10].view(np.int16)
    a_h = arena[n * 12: n * 16].view(np.uint32)
    a_qi = arena[n * 16: n * 20].view(np.uint32)
    a_qs = arena[n * 20: n * 20 + 4 * (cfg[1] + 2)].view(np.uint32)
    a_ptr[:] = ptrs
    lib = abi.load()
    with SoftRss(*cfg, device=0, max_burst=0) as eng:
        eng.register_host_memory(pool.ctypes.data, pool.nbytes)
        eng.register_host_memory(arena.ctypes.data, arena.nbytes)
        rc = lib.yrss_dispatch_burst_zc(eng._ctx, a_ptr.ctypes.data, n, a_q.ctypes.data,
                                        a_h.ctypes.data, a_qi.ctypes.data, a_qs.ctypes.data, 0)
        assert rc == 0
        assert np.array_equal(a_q, q) and np.array_equal(a_h, h)
        assert np.array_equal(a_qi, qi) and np.array_equal(a_qs[: qs.size], qs)
        eng.unregister_host_memory(arena.ctypes.data)
        eng.unregister_host_memory(pool.ctypes.data)


@pytest.mark.parametrize("nq", [62, 63, 64])
def test_small_burst_bucket_limit(dev, oracle_mod, nq):
    """nb = nb_queues + 1 <= 64 takes the one-launch path; 65 falls back."""
    cfg = (64, nq, 1, 0)
    frames = _frames(oracle_mod, 3000, nq)
    q, h, qi, qs = _expect(oracle_mod, frames, cfg)
    with SoftRss(*cfg, device=0, max_burst=0) as eng:
        _check(eng.dispatch_frames(frames), q, h, qi, qs)


def test_small_burst_fault_reported(dev, oracle_mod):
    frames = _frames(oracle_mod, 100, 5)
    pool, ptrs, _ = _fake_mbufs(frames)
    with SoftRss(3, 3, 1, 1, device=0, max_burst=0) as eng:
        eng.register_host_memory(pool.ctypes.data, pool.nbytes)
        bad = ptrs.copy()
        bad[17] = np.uint64(pool.ctypes.data + pool.nbytes + 4096)
        with pytest.raises(abi.YrssError):
            eng.dispatch_burst_zc(bad)
        r = eng.dispatch_burst_zc(ptrs)          # the fault does not stick
        q, h, qi, qs = _expect(oracle_mod, frames, (3, 3, 1, 1))
        _check(r, q, h, qi, qs)
        eng.unregister_host_memory(pool.ctypes.data)


@pytest.mark.parametrize("n", [32, 2000, 9000])
def test_small_and_multi_kernel_paths_agree(dev, oracle_mod, n, monkeypatch):
    frames = _frames(oracle_mod, n, 4242)
    outs = []
    for one_launch in (0, 2):   # default / never (multi-kernel path)
        with SoftRss(3, 3, 1, 1, device=0, max_burst=0) as eng:
            eng.set_tuning(one_launch=one_launch)
            outs.append(eng.dispatch_frames(frames))
            assert eng.status() == 0
    a, b = outs
    for f in ("q", "hash", "qidx", "qstart"):
        assert np.array_equal(np.asarray(getattr(a, f)), np.asarray(getattr(b, f))), f
    q, h, qi, qs = _expect(oracle_mod, frames, (3, 3, 1, 1))
    _check(a, q, h, qi, qs)


@pytest.mark.parametrize("n", [1000, 6000])   # one-launch path / multi-kernel path
def test_async_bursts_over_two_contexts(dev, oracle_mod, n):
    """YRSS_F_ASYNC: bursts in flight on two contexts sharing one registered
    pool; -EBUSY for a second burst on a busy context; yrss_wait delivers."""
    cfg = (5, 4, 1, 1)
    frames = _frames(oracle_mod, 2 * n, 99)
    q, h, qi, qs = _expect(oracle_mod, frames[:n], cfg)
    q2, h2, qi2, qs2 = _expect(oracle_mod, frames[n:], cfg)
    pool, ptrs, stride = _fake_mbufs(frames, headroom=128)
    lib = abi.load()
    outs = [(np.empty(n, np.int16), np.empty(n, np.uint32), np.empty(n, np.uint32),
             np.empty(cfg[1] + 2, np.uint32)) for _ in range(2)]
    with SoftRss(*cfg, device=0, max_burst=0) as e0, SoftRss(*cfg, device=0, max_burst=0) as e1:
        for e in (e0, e1):
            e.register_host_memory(pool.ctypes.data, pool.nbytes)   # refcounted
        halves = [ptrs[:n].copy(), ptrs[n:].copy()]
        for e, hp, o in zip((e0, e1), halves, outs):
            rc = lib.yrss_dispatch_burst_zc(e._ctx, hp.ctypes.data, n, o[0].ctypes.data,
                                            o[1].ctypes.data, o[2].ctypes.data,
                                            o[3].ctypes.data, abi.F_ASYNC | abi.F_WRITE_RSS)
            assert rc == 0
        # a second burst on a busy context, and the device path, are refused
        rc = lib.yrss_dispatch_burst_zc(e0._ctx, halves[0].ctypes.data, n, outs[0][0].ctypes.data,
                                        None, None, None, 0)
        assert rc == -16   # -EBUSY
        assert lib.yrss_wait(e0._ctx) == 0
        assert lib.yrss_wait(e1._ctx) == 0
        assert lib.yrss_wait(e1._ctx) == 0   # nothing in flight
        for o, (a, b, c_, d) in zip(outs, ((q, h, qi, qs), (q2, h2, qi2, qs2))):
            assert np.array_equal(o[0], a) and np.array_equal(o[1], b)
            assert np.array_equal(o[2], c_) and np.array_equal(o[3][: d.size], d)
        rss = pool.reshape(-1, stride)[:, 44:48].copy().view(np.uint32).ravel()
        assert np.array_equal(rss, np.concatenate([h, h2]))
        # dropping one context's registration keeps the other's working
        e0.unregister_host_memory(pool.ctypes.data)
        _check(e1.dispatch_burst_zc(ptrs[:n]), q, h, qi, qs)
        e1.unregister_host_memory(pool.ctypes.data)


def test_async_staged_and_frames(dev, oracle_mod):
    cfg = (8, 8, 1, 0)
    n = 3000
    frames = _frames(oracle_mod, n, 7)
    q, h, qi, qs = _expect(oracle_mod, frames, cfg)
    pool, ptrs, stride = _fake_mbufs(frames, headroom=130)
    data = (ptrs + np.uint64(128 + 130)).astype(np.uint64)
    flen = np.array([len(f) for f in frames], np.uint16)
    lib = abi.load()
    with SoftRss(*cfg, device=0, max_burst=0) as eng:
        oq, oh = np.empty(n, np.int16), np.empty(n, np.uint32)
        oqi, oqs = np.empty(n, np.uint32), np.empty(cfg[1] + 2, np.uint32)
        rc = lib.yrss_dispatch_burst(eng._ctx, ptrs.ctypes.data, n, oq.ctypes.data,
                                     None, oqi.ctypes.data, oqs.ctypes.data,
                                     abi.F_ASYNC | abi.F_WRITE_RSS)
        assert rc == 0
        assert lib.yrss_wait(eng._ctx) == 0
        assert np.array_equal(oq, q) and np.array_equal(oqi, qi)
        assert np.array_equal(oqs[: qs.size], qs)
        rss = pool.reshape(-1, stride)[:, 44:48].copy().view(np.uint32).ravel()
        assert np.array_equal(rss, h)
        eng.register_host_memory(pool.ctypes.data, pool.nbytes)
        rc = lib.yrss_dispatch_frames_zc_ex(eng._ctx, data.ctypes.data, flen.ctypes.data, n,
                                            oq.ctypes.data, oh.ctypes.data, oqi.ctypes.data,
                                            oqs.ctypes.data, abi.F_ASYNC)
        assert rc == 0
        assert lib.yrss_wait(eng._ctx) == 0
        assert np.array_equal(oq, q) and np.array_equal(oh, h) and np.array_equal(oqi, qi)
        eng.unregister_host_memory(pool.ctypes.data)


def test_async_python_wrapper(dev, oracle_mod):
    """SoftRss.dispatch_burst(_zc)(async_=True) + wait() on two engines."""
    cfg = (3, 3, 1, 1)
    n = 2500
    frames = _frames(oracle_mod, 2 * n, 321)
    want = [_expect(oracle_mod, frames[:n], cfg), _expect(oracle_mod, frames[n:], cfg)]
    pool, ptrs, _ = _fake_mbufs(frames)
    with SoftRss(*cfg, device=0, max_burst=0) as e0, SoftRss(*cfg, device=0, max_burst=0) as e1:
        r0 = e0.dispatch_burst(ptrs[:n], async_=True)
        e1.register_host_memory(pool.ctypes.data, pool.nbytes)
        r1 = e1.dispatch_burst_zc(ptrs[n:], async_=True)
        e0.wait()
        e1.wait()
        _check(r0, *want[0])
        _check(r1, *want[1])
        e1.unregister_host_memory(pool.ctypes.data)


@pytest.mark.parametrize("n", [1, 63, 65, 1000, 4096, 4097])
@pytest.mark.parametrize("stride", [64, 80, 2176])
def test_device_batch_small_path(dev, oracle_mod, monkeypatch, n, stride):
    """yrss_dispatch_dev batches of <= 4096 packets take the one-launch kernel;
    outputs (q, hash, filter class, lists) equal the three-kernel path's and
    the oracle's."""
    cfg = (5, 4, 1, 1)
    outs = []
    for one_launch in (0, 1):   # device batches in one launch / through the batch kernels
        with SoftRss(*cfg, device=0, max_burst=0) as eng:
            eng.set_tuning(one_launch=one_launch)
            eng.set_kni(True, "reject", "80,443", "53")
            win, lens = eng.synth(abi.SYN_FUZZ, n, 77, stride=stride)
            r = eng.dispatch_dev(win, lens, stride, n, want_filter=True)
            torch.cuda.synchronize()
            assert eng.status() == 0
            outs.append([x[: (n if x.numel() >= n else x.numel())].cpu().numpy()
                         for x in (r.q, r.hash, r.qidx, r.qstart, r.filter)])
            w_h = win[: n * stride].cpu().numpy()
            l_h = lens[:n].cpu().numpy().view(np.uint16)
    for a, b in zip(*outs):
        assert np.array_equal(a, b)
    c = oracle_mod.cfg(*cfg)
    q_ref, h_ref = oracle_mod.dispatch_windows(w_h, stride, l_h, c)
    assert np.array_equal(outs[0][0].view(np.int16), q_ref)
    assert np.array_equal(outs[0][1].view(np.uint32), h_ref)
