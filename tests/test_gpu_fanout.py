"""GPU parity of the host-burst fan-out (yrss_fanout_*): one dispatcher thread,
consecutive bursts round-robin over several contexts (here on one device),
returned in submission order; every burst bit-exact against the oracle and
the per-queue lists, handed off in ticket order, equal to the single-stream
answer (per-queue FIFO as rte_ring keeps it, fs/lib/ff_dpdk_if.c:1087-1093)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from yastack_amd import FanOut  # noqa: E402

from test_gpu_parity import _fake_mbufs  # noqa: E402
from test_gpu_small_burst import _check, _expect, _frames  # noqa: E402


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch.device("cuda", 0)


@pytest.mark.parametrize("nctx,frames_form", [(2, False), (3, True), (1, False)])
def test_fanout_in_order_fifo(dev, oracle_mod, nctx, frames_form):
    cfg = (5, 4, 1, 1)
    rng = np.random.default_rng(nctx * 7 + frames_form)
    sizes = [32, 1024, 0, 1, 33] + [int(x) for x in rng.integers(0, 1025, 40)]
    total = sum(sizes)
    frames = _frames(oracle_mod, total, 77 + nctx)
    pool, ptrs, _ = _fake_mbufs(frames, headroom=128)
    data = (ptrs + np.uint64(256)).astype(np.uint64)
    flen = np.array([len(f) for f in frames], np.uint16)
    q_all, h_all, qi_all, qs_all = _expect(oracle_mod, frames, cfg)
    nslots = 8
    with FanOut([0] * nctx, *cfg, nslots=nslots, nblocks=2) as fo:
        fo.register_host_memory(pool.ctypes.data, pool.nbytes)
        firsts = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
        got = []
        issued = 0
        for i, n in enumerate(sizes):
            if issued - len(got) >= nctx * nslots:       # every slot busy: hand one off
                got.append(fo.next())
            f0 = int(firsts[i])
            t = (fo.submit_frames(data[f0:f0 + n], flen[f0:f0 + n]) if frames_form
                 else fo.submit(ptrs[f0:f0 + n]))
            issued += 1
            assert t == issued
        while len(got) < issued:
            got.append(fo.next())
        assert fo.next(wait=False) is None                # nothing outstanding
        assert [t for t, _ in got] == list(range(1, issued + 1))
        # every burst bit-exact; lists merged in hand-off order = one stream
        lists = {b: [] for b in range(cfg[1] + 1)}
        for (t, r), f0, n in zip(got, firsts, sizes):
            q = q_all[f0:f0 + n]
            qi, qs = oracle_mod.process_burst(q, cfg[1])
            _check(r, q, h_all[f0:f0 + n], qi, qs)
            rq = np.asarray(r.qstart)
            for b in range(cfg[1] + 1):
                lists[b].extend(int(f0) + int(x) for x in np.asarray(r.qidx)[rq[b]:rq[b + 1]])
        merged = np.array([x for b in range(cfg[1] + 1) for x in lists[b]], np.int64)
        assert np.array_equal(merged, qi_all.astype(np.int64))
        fo.unregister_host_memory(pool.ctypes.data)
