"""Device-fault containment (include/yrss_remote.h), on the CPU.

The lcore-side client holds no HIP context; the yrss_helper child owns the GPU.
These tests need no GPU: a helper started with YRSS_HELPER_INJECT=1 comes up
and never completes a burst (as if its GPU hung), and the tests kill it.  The
ABI must answer -EPIPE (helper gone) or -ETIMEDOUT (no progress) within its
timeout instead of hanging, restart must bring up a new helper that takes the
queued bursts again, and stop must reap a hung helper.  Without a GPU a real
helper fails its yrss_init, and yrss_remote_start returns that error."""
import errno
import os
import signal
import time

import pytest

from yastack_amd import abi
from yastack_amd.remote import RemoteRss


def _frames(n):
    from frames import ipv4_frame
    return [ipv4_frame("10.0.0.1", 1000 + i, "10.0.0.2", 80) for i in range(n)]


@pytest.fixture
def inject(monkeypatch):
    monkeypatch.setenv("YRSS_HELPER_INJECT", "1")


def _cfg(nq=3):
    c = abi.default_config()
    c.nb_procs = nq
    c.nb_queues = nq
    return c


def test_killed_helper_is_reported_not_waited_on(inject):
    with RemoteRss(_cfg(), nslots=8, max_burst=64, nblocks=2, timeout_ms=5000) as r:
        pid = r.pid
        assert pid > 0
        t = r.submit(_frames(32))
        assert r.poll(t, wait=False)[0] == -errno.EAGAIN
        os.kill(pid, signal.SIGKILL)
        t0 = time.monotonic()
        rc = r.poll(t, wait=True)[0]
        assert rc == -errno.EPIPE and time.monotonic() - t0 < 4.0
        # the dead helper refuses new bursts too, until restart
        with pytest.raises(abi.YrssError):
            r.submit(_frames(4))
        r.restart()
        assert r.pid > 0 and r.pid != pid
        # the queued ticket is served by the new helper (this one hangs by design)
        assert r.poll(t, wait=False)[0] == -errno.EAGAIN
        t2 = r.submit(_frames(8))
        assert t2 == t + 1


def test_hung_helper_times_out(inject):
    with RemoteRss(_cfg(), nslots=4, max_burst=32, nblocks=1, timeout_ms=300) as r:
        t = r.submit(_frames(16))
        t0 = time.monotonic()
        assert r.poll(t, wait=True)[0] == -errno.ETIMEDOUT
        assert 0.2 < time.monotonic() - t0 < 5.0
        r.restart()                      # kills the hung helper, starts another
        assert r.poll(t, wait=False)[0] == -errno.EAGAIN


def test_stop_reaps_a_hung_helper(inject):
    r = RemoteRss(_cfg(), nslots=4, max_burst=32, nblocks=1, timeout_ms=300)
    pid = r.pid
    r.submit(_frames(4))
    os.kill(pid, signal.SIGSTOP)         # frozen: it cannot see the stop word
    t0 = time.monotonic()
    assert r.stop() == -errno.ETIMEDOUT
    assert time.monotonic() - t0 < 5.0
    with pytest.raises(ProcessLookupError):
        os.kill(pid, 0)


def test_ring_full_and_bad_args(inject):
    with RemoteRss(_cfg(), nslots=2, max_burst=16, nblocks=1, timeout_ms=1000) as r:
        r.submit(_frames(2))
        r.submit(_frames(2))
        with pytest.raises(abi.YrssError) as e:
            r.submit(_frames(2))
        assert e.value.errno == errno.EBUSY
        with pytest.raises(abi.YrssError):
            r.submit(_frames(17))        # past max_burst
    with pytest.raises(abi.YrssError):
        RemoteRss(_cfg(), nslots=3, max_burst=16, nblocks=2)   # nslots % nblocks


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU is present")
def test_helper_without_gpu_reports_its_init_error(monkeypatch):
    monkeypatch.delenv("YRSS_HELPER_INJECT", raising=False)
    with pytest.raises(abi.YrssError) as e:
        RemoteRss(_cfg(), nslots=4, max_burst=32, nblocks=1, timeout_ms=20000)
    assert e.value.errno in (errno.ENODEV, errno.EIO)
