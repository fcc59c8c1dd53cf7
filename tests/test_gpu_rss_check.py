"""GPU parity for SURVEY §8(f) rank 2: ff_rss_check (fs/lib/ff_dpdk_if.c:1904-1940)
as a device batch and as the full ephemeral-lport sweep of in_pcbconnect_setup
(fs/freebsd/netinet/in_pcb.c:1131-1170), against the oracle restatement."""
import socket
import struct

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from yastack_amd import SoftRss  # noqa: E402

CFGS = [(1, 128, 0), (2, 128, 1), (3, 512, 2), (8, 128, 5), (4, 0, 3), (5, 64, 0)]


@pytest.mark.parametrize("nq,reta,qid", CFGS)
def test_rss_check_batch(oracle_mod, nq, reta, qid):
    rng = np.random.default_rng(nq * 1000 + reta)
    tuples = rng.integers(0, 256, (100003, 12), dtype=np.uint8)
    ok_ref, h_ref = oracle_mod.rss_check_batch(tuples, nq, reta, qid)
    with SoftRss(3, device=0, max_burst=0) as eng:
        ok, h = eng.rss_check_dev(torch.from_numpy(tuples.reshape(-1)).cuda(), nq, reta, qid)
        torch.cuda.synchronize()
        assert np.array_equal(ok.cpu().numpy(), ok_ref)
        assert np.array_equal(h.cpu().numpy().view(np.uint32), h_ref)


@pytest.mark.parametrize("nq,reta,qid", CFGS)
def test_lport_sweep(oracle_mod, nq, reta, qid):
    faddr = struct.unpack("<I", socket.inet_aton("172.31.27.43"))[0]
    laddr = struct.unpack("<I", socket.inet_aton("192.168.1.100"))[0]
    fport = struct.unpack("<H", struct.pack(">H", 443))[0]
    lports = np.arange(65536, dtype=np.uint32)
    tup = np.zeros((65536, 12), np.uint8)
    tup[:, 0:4] = np.frombuffer(struct.pack("<I", faddr), np.uint8)
    tup[:, 4:8] = np.frombuffer(struct.pack("<I", laddr), np.uint8)
    tup[:, 8:10] = np.frombuffer(struct.pack("<H", fport), np.uint8)
    tup[:, 10] = lports & 0xFF
    tup[:, 11] = lports >> 8
    ok_ref, _ = oracle_mod.rss_check_batch(tup, nq, reta, qid)
    want = np.zeros(2048, np.uint32)
    for w in range(2048):
        bits = ok_ref[w * 32:(w + 1) * 32].astype(np.uint64)
        want[w] = int((bits << np.arange(32, dtype=np.uint64)).sum())
    with SoftRss(3, device=0, max_burst=0) as eng:
        got = eng.rss_lport_sweep(faddr, laddr, fport, nq, reta, qid)
    assert np.array_equal(got, want)
    if nq > 1:
        frac = ok_ref.mean()
        assert 0.5 / nq < frac < 2.0 / nq
