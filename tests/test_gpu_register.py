"""The per-packet registration shim (yrss_toeplitz_dispatch, SURVEY §8(b)
item 1): called through a dispatch_func_t pointer exactly as F-Stack's
process_packets calls the registered dispatcher (ff_dpdk_if.c:1078-1079), it
returns toeplitz_dispatch's value for every packet, from the GPU."""
import ctypes

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from yastack_amd import SoftRss, abi  # noqa: E402

from test_gpu_small_burst import _expect, _frames  # noqa: E402

DISPATCH_FUNC_T = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_uint16,
                                   ctypes.c_uint16, ctypes.c_uint16)


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch.device("cuda", 0)


@pytest.mark.parametrize("cfg", [(3, 3, 1, 1), (5, 4, 1, 0), (4, 2, 0, 1)])
def test_registered_dispatcher_matches_oracle(dev, oracle_mod, cfg):
    lib = abi.load()
    frames = _frames(oracle_mod, 300, 500 + cfg[0])
    q, _, _, _ = _expect(oracle_mod, frames, cfg)
    fn = DISPATCH_FUNC_T(ctypes.cast(lib.yrss_toeplitz_dispatch, ctypes.c_void_p).value)
    with SoftRss(*cfg, device=0) as eng:
        assert lib.yrss_set_dispatch_ctx(eng._ctx) == 0
        got = []
        for j, f in enumerate(frames):
            buf = ctypes.create_string_buffer(f, len(f))
            got.append(fn(ctypes.cast(buf, ctypes.c_void_p), len(f), j % 7, cfg[1]))
        assert np.array_equal(np.array(got, np.int16), q)
    # yrss_fini cleared the context it owned: back to the error value
    buf = ctypes.create_string_buffer(frames[0], len(frames[0]))
    assert fn(ctypes.cast(buf, ctypes.c_void_p), len(frames[0]), 0, cfg[1]) == -1


def test_python_wrappers(dev, oracle_mod):
    """SoftRss.toeplitz_dispatch and SoftRss.worker_submit_frames."""
    cfg = (3, 3, 1, 1)
    frames = _frames(oracle_mod, 200, 606)
    q, h, _, _ = _expect(oracle_mod, frames, cfg)
    from test_gpu_parity import _fake_mbufs
    pool, ptrs, _ = _fake_mbufs(frames, headroom=128)
    data = (ptrs + np.uint64(128 + 128)).astype(np.uint64)
    lens = np.array([len(f) for f in frames], np.uint16)
    with SoftRss(*cfg, device=0, max_burst=0) as eng:
        assert [eng.toeplitz_dispatch(f) for f in frames[:40]] == [int(x) for x in q[:40]]
        eng.register_host_memory(pool.ctypes.data, pool.nbytes)
        eng.worker_start(4, 2)
        tks = [eng.worker_submit_frames(data[i:i + 50], lens[i:i + 50]) for i in (0, 50, 100, 150)]
        for k, t in enumerate(tks):
            r = eng.worker_poll(t)
            sl = slice(50 * k, 50 * k + 50)
            qi, qs = oracle_mod.process_burst(q[sl], cfg[1])
            assert np.array_equal(r.q, q[sl]) and np.array_equal(r.hash, h[sl])
            assert np.array_equal(r.qidx, qi) and np.array_equal(r.qstart[: qs.size], qs)
        eng.worker_stop()
        eng.unregister_host_memory(pool.ctypes.data)


@pytest.mark.parametrize("cfg", [(3, 3, 1, 1), (4, 2, 0, 1)])
def test_registered_dispatcher_through_worker(dev, oracle_mod, cfg):
    """A context with a resident worker serves each shim call as a one-packet
    worker burst: same answers, frames from unregistered memory (the shim
    copies each window into its own registered slot), lengths past the
    80-byte window included."""
    lib = abi.load()
    frames = _frames(oracle_mod, 300, 700 + cfg[0])
    q, _, _, _ = _expect(oracle_mod, frames, cfg)
    fn = DISPATCH_FUNC_T(ctypes.cast(lib.yrss_toeplitz_dispatch, ctypes.c_void_p).value)
    with SoftRss(*cfg, device=0) as eng:
        eng.worker_start(4, 1)
        assert lib.yrss_set_dispatch_ctx(eng._ctx) == 0
        got = []
        for j, f in enumerate(frames):
            buf = ctypes.create_string_buffer(f, len(f))
            got.append(fn(ctypes.cast(buf, ctypes.c_void_p), len(f), j % 7, cfg[1]))
        assert np.array_equal(np.array(got, np.int16), q)
        assert max(len(f) for f in frames) > 80
        eng.worker_stop()
        # without the worker the same context falls back to one launch per call
        buf = ctypes.create_string_buffer(frames[0], len(frames[0]))
        assert fn(ctypes.cast(buf, ctypes.c_void_p), len(frames[0]), 0, cfg[1]) == int(q[0])
