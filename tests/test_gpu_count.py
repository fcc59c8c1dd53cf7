"""Count-mode scatter parity (GPU).

With 10..YRSS_COUNT_MAXNB buckets (off by default since the ranked group stage), groups
that feed more than YRSS_COUNT_KMIN buckets (default 8) are ranked by a
lane-serial counting sort in LDS and leave through the LDS list image
(yrss.hip scatter_count / image_layout / flush_image); groups feeding fewer
take the few-bucket path in the same launch.  Every combination of bucket
count, group size (32 or 64 packets per lane), threshold, ragged batch size
and output alignment must give the oracle's per-queue FIFO lists
(fs/lib/ff_dpdk_if.c:1058-1094 enqueue order) bit-exactly, as must the
ballot path it replaces (YRSS_NO_COUNT=1).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from yastack_amd import SoftRss, abi  # noqa: E402
from yastack_amd.dispatch import DispatchResult  # noqa: E402

from test_gpu_layout import _env, check  # noqa: E402

ANY_NB = 257   # YRSS_COUNT_MAXNB: count mode for every bucket count that fits LDS


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch.device("cuda", 0)


@pytest.mark.parametrize("cfg", [(9, 9, 1, 0), (16, 16, 1, 1), (17, 17, 1, 0), (32, 32, 1, 0),
                                 (64, 64, 1, 1), (254, 254, 1, 0), (300, 255, 1, 0)])
@pytest.mark.parametrize("group", [32, 64])
def test_count_mode_bucket_counts(dev, oracle_mod, cfg, group):
    """10..256 buckets with count mode allowed for all (past ~180 buckets
    the image and counters outgrow a wave's LDS share and the launch keeps
    the ballot path), both group sizes."""
    with _env(YRSS_GROUP_TILES=group, YRSS_COUNT_MAXNB=ANY_NB):
        with SoftRss(*cfg, device=0, max_burst=0) as eng:
            for profile in (abi.SYN_TCP4, abi.SYN_FUZZ):
                check(eng, oracle_mod, cfg, profile, 400003, first=21)


@pytest.mark.parametrize("kmin", [1, 2, 4, 7])
@pytest.mark.parametrize("profile", [abi.SYN_UDP4, abi.SYN_IMIX, abi.SYN_FUZZ])
def test_count_mode_threshold(dev, oracle_mod, kmin, profile):
    """A low threshold sends groups with few buckets (IMIX / UDP stretches)
    through count mode too, mixed with few-bucket groups in one launch."""
    cfg = (12, 12, 1, 1)
    with _env(YRSS_COUNT_KMIN=kmin, YRSS_COUNT_MAXNB=ANY_NB):
        with SoftRss(*cfg, device=0, max_burst=0) as eng:
            check(eng, oracle_mod, cfg, profile, 262144 + 4097, first=5)


@pytest.mark.parametrize("n", [1, 4095, 4096, 4097, 8191, 65536 + 63, 1 << 20])
def test_count_mode_ragged(dev, oracle_mod, n):
    """Batch sizes around the group size: the last group's lanes past the
    end hold no packets, a lane's run may end mid-run."""
    cfg = (20, 20, 1, 0)
    with _env(YRSS_COUNT_MAXNB=ANY_NB):
        with SoftRss(*cfg, device=0, max_burst=0) as eng:
            check(eng, oracle_mod, cfg, abi.SYN_FUZZ, n, first=n)


def test_count_mode_matches_ballot_path(dev, oracle_mod):
    """YRSS_NO_COUNT=1 (ballot ranking, per-lane stores): identical lists."""
    cfg = (24, 24, 1, 1)
    for flag in ("1", "0"):
        with _env(YRSS_NO_COUNT=flag, YRSS_COUNT_MAXNB=ANY_NB):
            with SoftRss(*cfg, device=0, max_burst=0) as eng:
                check(eng, oracle_mod, cfg, abi.SYN_TCP4, 1 << 21, first=8)


@pytest.mark.parametrize("count_maxnb", [ANY_NB, 9])
@pytest.mark.parametrize("qshift,ishift", [(1, 1), (3, 2), (5, 3)])
def test_count_mode_unaligned(oracle_mod, qshift, ishift, count_maxnb):
    """q at 2-byte alignment (count mode loads it as 16-byte vectors) and qidx
    at 4-byte alignment, n odd; nothing written outside qidx.  Count mode, and
    the default ranked group stage at the same bucket count."""
    n, stride, cfg = 300007, 64, (16, 16, 1, 0)
    with _env(YRSS_COUNT_MAXNB=count_maxnb), SoftRss(*cfg, device=0, max_burst=0) as eng:
        win, lens = eng.synth(abi.SYN_TCP4, n, 3, stride=stride)
        d = win.device
        qi_buf = torch.full((n + 8,), -1, dtype=torch.int32, device=d)
        q_buf = torch.empty(n + 8, dtype=torch.int16, device=d)
        h_buf = torch.empty(n + 8, dtype=torch.int32, device=d)
        qs = torch.empty(16 + 2, dtype=torch.int32, device=d)
        out = DispatchResult(q_buf[qshift:qshift + n], h_buf[:n], qi_buf[ishift:ishift + n], qs)
        res = eng.dispatch_dev(win, lens, stride, n, out=out)
        torch.cuda.synchronize()
        w_h = win[: n * stride].cpu().numpy()
        l_h = lens[:n].cpu().numpy().view(np.uint16)
        q_ref, h_ref = oracle_mod.dispatch_windows(w_h, stride, l_h, oracle_mod.cfg(*cfg))
        qi_ref, qs_ref = oracle_mod.process_burst(q_ref, 16)
        assert np.array_equal(res.q.cpu().numpy(), q_ref)
        assert np.array_equal(qs.cpu().numpy().view(np.uint32), qs_ref)
        qi_all = qi_buf.cpu().numpy()
        assert np.array_equal(qi_all[ishift:ishift + n].view(np.uint32), qi_ref)
        assert (qi_all[:ishift] == -1).all() and (qi_all[ishift + n:] == -1).all()


@pytest.mark.parametrize("cfg", [(20, 20, 1, 0), (32, 32, 1, 1), (48, 48, 1, 0)])
@pytest.mark.parametrize("n", [1025, 4097, 400003])
@pytest.mark.parametrize("img,gstage", [(0, 1), (1, 0), (0, 0)])
def test_ranked_image(dev, oracle_mod, cfg, n, img, gstage):
    """The ranked path (18..65 buckets with count mode held to 17) with its
    lists built in one packed stage per group (the default), a packed LDS image
    (YRSS_RANK_IMG=1) or the per-chunk stage: the same FIFO lists."""
    with _env(YRSS_RANK_IMG=img, YRSS_RANK_GSTAGE=gstage, YRSS_COUNT_MAXNB=17):
        with SoftRss(*cfg, device=0, max_burst=0) as eng:
            for profile in (abi.SYN_TCP4, abi.SYN_FUZZ):
                check(eng, oracle_mod, cfg, profile, n, first=n + 3)
