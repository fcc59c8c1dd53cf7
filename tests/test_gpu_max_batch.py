"""yrss_dispatch_dev at YRSS_MAX_BATCH (2^31 packets, 128 GiB of windows in
one MI355X's HBM): every address, chunk layout and list offset at its widest.
Checked against the oracle on eight 4096-packet blocks spread over the batch
(both ends included: generator and dispatch at packet indices near 2^31), and
on the whole batch through size-independent properties of the per-queue lists
(counts = q histogram, FIFO order, each index in its own bucket, hence a
permutation), computed in chunks so the checks need a few GiB beside the batch.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from yastack_amd import SoftRss, abi  # noqa: E402

CHUNK = 1 << 27


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch.device("cuda", 0)


def test_max_batch(dev, oracle_mod):
    n = 1 << 31   # YRSS_MAX_BATCH
    free, _ = torch.cuda.mem_get_info(dev)
    if free < (170 << 30):
        pytest.skip(f"needs ~160 GiB of free HBM, {free >> 30} GiB free")
    cfg = (8, 6, 1, 0)
    nbk = cfg[1] + 1
    with SoftRss(*cfg, device=0, max_burst=0) as eng:
        win, lens = eng.synth(abi.SYN_TCP4, n, stride=64)
        res = eng.dispatch_dev(win, lens, 64, n)
        torch.cuda.synchronize()
        assert eng.status() == 0

        c = oracle_mod.cfg(*cfg)
        rng = np.random.default_rng(31)
        starts = [0, n - 4096] + sorted(int(x) for x in rng.integers(0, n - 4096, 6))
        for s in starts:
            w = win[s * 64:(s + 4096) * 64].cpu().numpy()
            ln = lens[s:s + 4096].cpu().numpy().view(np.uint16)
            w_o, l_o = oracle_mod.synth(abi.SYN_TCP4, 4096, s, stride=64)
            assert np.array_equal(w, w_o) and np.array_equal(ln, l_o), s
            q_ref, h_ref = oracle_mod.dispatch_windows(w, 64, ln, c)
            assert np.array_equal(res.q[s:s + 4096].cpu().numpy().view(np.int16), q_ref), s
            assert np.array_equal(res.hash[s:s + 4096].cpu().numpy().view(np.uint32), h_ref), s
        del win, lens

        def bucket(qv):
            qv = qv.long()
            return torch.where((qv >= 0) & (qv < cfg[1]), qv, torch.full_like(qv, cfg[1]))

        counts = torch.zeros(nbk, dtype=torch.long, device=dev)
        for lo in range(0, n, CHUNK):
            counts += torch.bincount(bucket(res.q[lo:lo + CHUNK]), minlength=nbk)
        qs = res.qstart[: nbk + 1].long() & 0xFFFFFFFF   # uint32 in an int32 tensor
        assert int(qs[0]) == 0 and int(qs[-1]) == n
        assert torch.equal(qs[1:] - qs[:-1], counts)
        for b in range(nbk):
            lo_b, hi_b = int(qs[b]), int(qs[b + 1])
            prev = -1
            for lo in range(lo_b, hi_b, CHUNK):
                idx = res.qidx[lo:min(lo + CHUNK, hi_b)].long() & 0xFFFFFFFF
                assert int(idx[0]) > prev, (b, lo)
                assert bool(torch.all(idx[1:] > idx[:-1])), (b, lo)
                assert bool(torch.all(bucket(res.q[idx]) == b)), (b, lo)
                prev = int(idx[-1])
